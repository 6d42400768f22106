#!/bin/bash
# Parity tests of the fused path + window probes (product / no filter bank / DMA only) + bench.
set -euo pipefail
mkdir -p gpurun_out/quick
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quick/pytest.log 2>&1 || { tail -30 gpurun_out/quick/pytest.log; exit 1; }
tail -2 gpurun_out/quick/pytest.log
for A in 0 4 6; do timeout -k 10 60 tools/probes/window_probe_$A; done
timeout -k 10 60 tools/probes/window_probe_0
timeout -k 10 200 python bench.py --cpu-sample 0 --alt-steps 0
