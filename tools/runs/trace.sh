#!/bin/bash
# rocprofv3 kernel (+ memory-copy) trace of one bench.py command, e.g. the configs[4] chunk
# pipeline:  TAG=r06d ARGS="--workload stream --steps 3 --warmup 1" COPIES=1 bash tools/runs/trace.sh
set -uo pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:?}; mkdir -p $OUT
export TMPDIR=/tmp
EXTRA=""; [ "${COPIES:-0}" = "1" ] && EXTRA="--memory-copy-trace"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace $EXTRA --stats --output-format csv -d $OUT/trace -o run \
  -- python3 $ROOT/bench.py --cpu-sample 0 --alt-steps 0 ${ARGS:-} > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
find $OUT/trace -name "*stats.csv" -exec cut -c1-160 {} \;
