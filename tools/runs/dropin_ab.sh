#!/bin/bash
# Interleaved A/B of the per-epoch drop-in (host-side waits, servers) between library builds:
# tools/dropin_bench and tools/mailbox_threads at 16 and 32 threads, each lib via LD_LIBRARY_PATH.
#   TAG=r06d LIBS="new: prev:tools/ab/prev" REPS=2 bash tools/runs/dropin_ab.sh
set -uo pipefail
OUT=gpurun_out/${TAG:?}; mkdir -p $OUT
for rep in $(seq ${REPS:-2}); do
  for lv in ${LIBS:-new:}; do
    name=${lv%%:*}; dir=${lv#*:}
    LP=""; [ -n "$dir" ] && LP="$(pwd)/$dir"
    f=$OUT/${name}_$rep
    LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 300 tools/dropin_bench . 2000 1 > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "
import json
d = json.load(open('$f.json'))
m = d['mailbox']['threads']
print('$name rep$rep', 'single %.2f us' % d['single_epoch']['median_us'],
      ' '.join('T%s med %.1f p99 %.1f max %.0f res %d' % (t, v['median_us'], v['p99_us'], v['max_us'], v['resident_servers']) for t, v in m.items()))
" | tee -a $OUT/ab.log
    for T in 16 32; do
      echo -n "$name rep$rep harness: " >> $OUT/ab.log
      LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 120 tools/mailbox_threads tests/golden/test-data/DoD/DoD2015_01.vhdr $T 500 2>&1 | tee -a $OUT/ab.log || exit 1
    done
  done
done
