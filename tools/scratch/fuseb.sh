#!/bin/bash
# In-kernel baselines (EEGFX_FUSE_BASELINE=1): GPU parity suite with it on, then A/B benches.
set -euo pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-fuseb}; mkdir -p $OUT
EEGFX_FUSE_BASELINE=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_on.log 2>&1 || { tail -30 $OUT/pytest_on.log; exit 1; }
tail -2 $OUT/pytest_on.log
for i in 1 2; do
  for F in 0 1; do
    EEGFX_FUSE_BASELINE=$F timeout -k 10 300 python bench.py --cpu-sample 0 > $OUT/bench_${F}_$i.json 2> $OUT/bench_${F}_$i.err || { tail -20 $OUT/bench_${F}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['bytes_per_epoch'], d['roofline']['frac'], d['alt_numerics'])" $OUT/bench_${F}_$i.json
  done
done
