#!/bin/bash
# A/B of the window-kernel decode (EEGFX_DECODE_SCALAR 1 vs 2) after the GPU parity suite.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-decode_ab}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
for R in 1 2; do
  for P in window_probe_d1 window_probe_0; do
    for EX in "" 1; do
      PROBE_RANDOM=1 PROBE_ITERS=3000 PROBE_EXACT=$EX timeout -k 10 120 tools/probes/$P | sed "s/^/$P exact=$EX: /"
    done
  done
done
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
