#!/bin/bash
# DMA cache policy with dense markers (a window every 100 frames: each frame in ~6 windows).
set -euo pipefail
for R in 1 2; do
  for P in 0 nt; do
    PROBE_SPACING=100 PROBE_RANDOM=1 PROBE_ITERS=3000 timeout -k 10 120 tools/probes/window_probe_$P | sed "s/^/dense $P: /"
    PROBE_RANDOM=1 PROBE_ITERS=3000 timeout -k 10 120 tools/probes/window_probe_$P | sed "s/^/sparse $P: /"
  done
done
