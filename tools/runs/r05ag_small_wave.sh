#!/bin/bash
# Per-epoch drop-in: whole-wave EXACT levels (new libeegfx.so) against the round-5 8-lane cascade
# (tools/ab_old/libeegfx.so), both numerics, interleaved twice; then the mailbox GPU tests.
set -o pipefail
OUT=gpurun_out/r05ag
mkdir -p $OUT
for rep in 1 2; do
  for num in 0 1; do
    LD_LIBRARY_PATH=$PWD/tools/ab_old timeout -k 10 180 tools/dropin_bench . 2000 $num \
        > $OUT/old_n${num}_r${rep}.json 2> $OUT/old_n${num}_r${rep}.err || exit 1
    timeout -k 10 180 tools/dropin_bench . 2000 $num \
        > $OUT/new_n${num}_r${rep}.json 2> $OUT/new_n${num}_r${rep}.err || exit 1
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_mailbox.py tests/test_gpu_guard.py \
    tests/test_gpu_robustness.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
