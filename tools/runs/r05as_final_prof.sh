#!/bin/bash
# Final tree: the default bench line under rocprofv3 --kernel-trace --stats (window_kernel average
# against the bench's HIP-event kernel_ms).
set -o pipefail
OUT=$PWD/gpurun_out/r05as
ROOT=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $ROOT/bench.py > $OUT/bench.json 2> $OUT/bench.err
