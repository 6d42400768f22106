#!/bin/bash
# configs[4] streamed ingest: interleaved bench lines over chunk sizes and library builds.
#   TAG=r06h CHUNKS="4194304 8388608 16777216" LIBS="new:" REPS=2 bash tools/runs/stream_ab.sh
set -uo pipefail
OUT=gpurun_out/${TAG:?}; mkdir -p $OUT
for rep in $(seq ${REPS:-2}); do
  for c in ${CHUNKS:-8388608}; do
    for lv in ${LIBS:-new:}; do
      name=${lv%%:*}; lib=${lv#*:}
      LB=""; [ -n "$lib" ] && LB="--lib $lib"
      f=$OUT/${name}_c${c}_$rep
      timeout -k 10 300 python bench.py --workload stream --steps 10 --warmup 3 --cpu-sample 0 \
        --chunk-frames $c $LB > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
      python3 -c "
import json; d = json.load(open('$f.json')); h = d['host_link']
print('$name chunk $c rep$rep', 'step ms', d['ms_per_step'], 'copy ms', h['copy_only_ms'], 'frac', h['frac'])" | tee -a $OUT/ab.log
    done
  done
done
