#!/bin/bash
# Power / clock under sustained load: product (random and constant input), compute only (no DMA),
# DMA only, and dense markers; amd-smi sampled mid-run.
set -uo pipefail
OUT=gpurun_out/power; mkdir -p $OUT
run() {  # name, probe, env...
  local name=$1 probe=$2; shift 2
  env "$@" PROBE_ITERS=3000 timeout -k 10 60 $probe > $OUT/$name.txt 2>&1 &
  local pid=$!
  sleep 1.5
  timeout 20 amd-smi metric -c -p -g 0 > $OUT/${name}_smi.txt 2>&1
  wait $pid
  echo "$name: $(cat $OUT/$name.txt | tail -1) | $(grep -E 'SOCKET_POWER' $OUT/${name}_smi.txt | head -1 | xargs) | $(grep -A1 'GFX_0:' $OUT/${name}_smi.txt | grep CLK | xargs)"
}
run product_random tools/probes/window_probe_0 PROBE_RANDOM=1
run product_const tools/probes/window_probe_0 X=1
run compute_only_random tools/probes/window_probe_1 PROBE_RANDOM=1
run dma_only tools/probes/window_probe_6 X=1
run dense_markers_random tools/probes/window_probe_0 PROBE_RANDOM=1 PROBE_SPACING=100
for I in 10 30 100 1000; do echo -n "random iters $I: "; PROBE_RANDOM=1 PROBE_ITERS=$I timeout -k 10 60 tools/probes/window_probe_0; done
