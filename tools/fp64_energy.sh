#!/bin/bash
# Energy per fp64 multiply-add on the two pipes (cost an FP64-MFMA form of the
# filter against the measured VALU energy per MAC).  fp64_probe runs one mode back to back on every
# CU (8 waves per SIMD) for a few seconds; amd-smi samples socket power and the XCD clocks mid-run.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-fp64energy}
mkdir -p "$OUT"
P=tools/probes/fp64_probe
[ -x $P ] || /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -w tools/probes/fp64_probe.hip -o $P || exit 1
for m in 0 1; do
  L=$([ $m = 0 ] && echo 3000 || echo 1000)
  PROBE_MODE=$m PROBE_LAUNCHES=$L timeout -k 10 120 $P > "$OUT/mode$m.txt" 2>&1 &
  pid=$!
  sleep 2.0
  timeout 20 amd-smi metric -p -c -g 0 > "$OUT/mode${m}_smi.txt" 2>&1
  wait $pid || { cat "$OUT/mode$m.txt"; exit 1; }
  echo "mode $m: $(cat "$OUT/mode$m.txt") | $(grep -E 'SOCKET_POWER' "$OUT/mode${m}_smi.txt" | head -1 | xargs)"
done
M=tools/probes/mfma44_probe
[ -x $M ] || /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -w tools/probes/mfma44_probe.hip -o $M || exit 1
PROBE_LAUNCHES=${L44:-1500} timeout -k 10 120 $M > "$OUT/mfma44.txt" 2>&1 &
pid=$!
sleep 2.5
timeout 20 amd-smi metric -p -c -g 0 > "$OUT/mfma44_smi.txt" 2>&1
wait $pid || { cat "$OUT/mfma44.txt"; exit 1; }
echo "mfma44: $(tail -1 "$OUT/mfma44.txt") | $(grep -E 'SOCKET_POWER' "$OUT/mfma44_smi.txt" | head -1 | xargs)"
timeout 20 amd-smi metric -p -c -g 0 > "$OUT/idle_smi.txt" 2>&1
echo "idle: $(grep -E 'SOCKET_POWER' "$OUT/idle_smi.txt" | head -1 | xargs)"
