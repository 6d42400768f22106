#!/bin/bash
# Shader clock / power while the window kernel (product, compute only, memory only) runs ~3 s.
set -uo pipefail
mkdir -p gpurun_out/clk2
for A in 0 1 6; do
  PROBE_ITERS=3000 timeout -k 10 60 tools/probes/window_probe_$A > gpurun_out/clk2/p$A.txt 2>&1 &
  PID=$!
  sleep 1.5
  timeout 20 amd-smi metric -c -p -g 0 > gpurun_out/clk2/smi$A.txt 2>&1
  wait $PID; echo "rc $? $(cat gpurun_out/clk2/p$A.txt)"
  grep -iE "GFX_0|CLK\b|SOCKET_POWER|POWER|gfx" gpurun_out/clk2/smi$A.txt | head -12
done
