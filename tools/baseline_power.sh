#!/bin/bash
# Socket power / clock while baseline_kernel runs back to back (is the memory-bound pass below the
# 1.4 kW cap?  DESIGN.md 11, the single-launch idea).  One GPU box.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-basepower}
mkdir -p "$OUT"
PROBE_BASELINE=1 PROBE_ITERS=30000 timeout -k 10 60 tools/probes/window_probe > "$OUT/baseline.txt" 2>&1 &
pid=$!
sleep 2.0
timeout 20 amd-smi metric -p -c -g 0 > "$OUT/baseline_smi.txt" 2>&1
wait $pid || { cat "$OUT/baseline.txt"; exit 1; }
echo "baseline_kernel: $(tail -1 "$OUT/baseline.txt" | cut -c1-70) | $(grep -E 'SOCKET_POWER' "$OUT/baseline_smi.txt" | head -1 | xargs) | $(grep -A2 'GFX_0:' "$OUT/baseline_smi.txt" | grep -E 'CLK:' | head -1 | xargs)"
