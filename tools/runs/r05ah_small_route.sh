#!/bin/bash
# Per-epoch drop-in after the whole-wave levels and single-epoch mailbox routing: GPU tests of the
# small path, the drop-in bench in both numerics, and the kernel durations under rocprofv3.
set -o pipefail
OUT=gpurun_out/r05ah
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_mailbox.py tests/test_gpu_c_abi.py \
    tests/test_gpu_guard.py tests/test_gpu_robustness.py -x -q --timeout 120 \
    --timeout-method thread > $OUT/pytest.log 2>&1 &&
timeout -k 10 180 tools/dropin_bench . 2000 0 > $OUT/dropin_exact.json 2> $OUT/dropin_exact.err &&
timeout -k 10 180 tools/dropin_bench . 2000 1 > $OUT/dropin_fma.json 2> $OUT/dropin_fma.err &&
TAG=r05ah/prof timeout -k 10 200 bash tools/dropin_prof.sh > $OUT/prof.txt 2>&1
