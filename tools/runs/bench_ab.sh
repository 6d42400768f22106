#!/bin/bash
# Interleaved bench.py A/B of library builds and/or plant specs on one box.
#   TAG=r06c LIBS="new: rowsoff:tools/ab/rowsoff/libeegfx.so" SPECS="none flat:0.32" REPS=3 \
#     ARGS="--steps 50 --warmup 20" bash tools/runs/bench_ab.sh
# LIBS: name:path pairs (empty path = the product library); SPECS: --plant specs ("none" = no
# plant).  PRE: an optional command run first (e.g. a pytest selection), its log in $TAG/pre.log.
set -uo pipefail
OUT=gpurun_out/${TAG:?}; mkdir -p $OUT
if [ -n "${PRE:-}" ]; then
  timeout -k 10 600 bash -c "$PRE" > $OUT/pre.log 2>&1 || { tail -30 $OUT/pre.log; exit 1; }
  tail -3 $OUT/pre.log
fi
B="--cpu-sample 0 --alt-steps 0 ${ARGS:---steps 50 --warmup 20}"
for rep in $(seq ${REPS:-3}); do
  for spec in ${SPECS:-none}; do
    for lv in ${LIBS:-new:}; do
      name=${lv%%:*}; lib=${lv#*:}
      PL=""; [ "$spec" != none ] && PL="--plant $spec"
      LB=""; [ -n "$lib" ] && LB="--lib $lib"
      f=$OUT/${name}_${spec/:/_}_$rep
      timeout -k 10 300 python bench.py $B $PL $LB > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
      python3 -c "
import json
d = json.load(open('$f.json'))
g = d['config'].get('guard') or {}
print('$name $spec rep$rep', 'step ms %.4f' % d['ms_per_step'], 'window ms %.4f' % d['roofline']['kernel_ms'], 'guard', g)
" | tee -a $OUT/ab.log
    done
  done
done
