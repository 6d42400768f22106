#!/bin/bash
# Throughput and socket power per instruction mix of an exact-integer matrix-core form of the
# dwt-8 operator: v_fma_f64 (today's filter), v_pk_fma_f32 (the
# decode residuals), int8 MFMA (M_q . v) and f16 MFMA (M . e), each back to back on every CU with
# amd-smi sampled mid-run, then the idle power.
#   TAG=r04j bash tools/pipe_energy.sh
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pipe_energy}
mkdir -p "$OUT"
P=tools/probes/pipe_energy_probe
[ -x $P ] || /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -w tools/probes/pipe_energy_probe.hip -o $P || exit 1
for m in 0 1 2 3; do
  L=$(case $m in 0) echo 8000;; 1) echo 8000;; *) echo 4000;; esac)
  PROBE_MODE=$m PROBE_LAUNCHES=$L timeout -k 10 90 $P > "$OUT/mode$m.txt" 2>&1 &
  pid=$!
  sleep 2.0
  timeout 20 amd-smi metric -p -c -g 0 > "$OUT/mode${m}_smi.txt" 2>&1
  wait $pid || { echo "mode $m failed"; cat "$OUT/mode$m.txt"; exit 1; }
  echo "$(cat "$OUT/mode$m.txt") | $(grep -E 'SOCKET_POWER' "$OUT/mode${m}_smi.txt" | head -1 | xargs) | $(grep -A2 'GFX_0:' "$OUT/mode${m}_smi.txt" | grep -E 'CLK:' | head -1 | xargs)"
done
sleep 1
timeout 20 amd-smi metric -p -c -g 0 > "$OUT/idle_smi.txt" 2>&1
echo "idle: $(grep -E 'SOCKET_POWER' "$OUT/idle_smi.txt" | head -1 | xargs)"
