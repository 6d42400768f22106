#!/bin/bash
# Kernel durations of the per-epoch drop-in path (tools/dropin_bench under rocprofv3).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-dropin_prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "$ROOT/tools/dropin_bench" "$ROOT" 500 1 > "$OUT/run.log" 2>&1 || { tail -20 "$OUT/run.log"; exit 1; }
cut -c1-180 "$OUT/trace/run_kernel_stats.csv"
