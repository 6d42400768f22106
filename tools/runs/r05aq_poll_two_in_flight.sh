#!/bin/bash
# Two polls in flight (product) against one poll per round trip
# (tools/ab_poll/libeegfx.so = the previous commit's kernels.hip), tools/dropin_bench fma,
# interleaved, three repetitions; then the mailbox GPU tests.
set -o pipefail
OUT=gpurun_out/r05aq
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_mailbox.py -x -q --timeout 120 \
    --timeout-method thread > $OUT/pytest_mailbox.log 2>&1 || exit 1
for rep in 1 2 3; do
  LD_LIBRARY_PATH=$PWD/tools/ab_poll timeout -k 10 180 tools/dropin_bench . 2000 1 \
      > $OUT/old_r${rep}.json 2> $OUT/old_r${rep}.err || exit 1
  timeout -k 10 180 tools/dropin_bench . 2000 1 > $OUT/new_r${rep}.json 2> $OUT/new_r${rep}.err || exit 1
done
