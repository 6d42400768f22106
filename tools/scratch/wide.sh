#!/bin/bash
set -euo pipefail
mkdir -p gpurun_out/wide
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mfma.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wide/pytest.log 2>&1 || { tail -30 gpurun_out/wide/pytest.log; exit 1; }
tail -2 gpurun_out/wide/pytest.log
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/wide/tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c32 --cpu-sample 0 --alt-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/wide/b.json 2>$GRAFT_REPO_ROOT/gpurun_out/wide/b.err
cat $GRAFT_REPO_ROOT/gpurun_out/wide/b.json | cut -c1-700
find $GRAFT_REPO_ROOT/gpurun_out/wide/tr -name "*kernel_stats.csv" -exec cut -c1-160 {} \; | head -4
