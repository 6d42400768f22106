#!/bin/bash
# 32-channel streaming variant: wide-kernel GPU tests, then c32 bench A/B (EEGFX_DMA_NT=0 vs auto).
set -euo pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-c32nt}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  for F in 0 auto; do
    if [ $F = auto ]; then unset EEGFX_DMA_NT; else export EEGFX_DMA_NT=$F; fi
    timeout -k 10 300 python bench.py --workload c32 --cpu-sample 0 > $OUT/bench_${F}_$i.json 2> $OUT/bench_${F}_$i.err || { tail -20 $OUT/bench_${F}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" $OUT/bench_${F}_$i.json
  done
done
