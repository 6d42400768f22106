#!/bin/bash
# DMA cache-policy study: window_probe (3,000 back-to-back window_kernel launches, random samples)
# with the default, nt, sc1 and sc0+sc1+nt modifiers on every window DMA, interleaved twice.
set -euo pipefail
for R in 1 2; do
  for P in 0 nt sc1 all; do
    PROBE_RANDOM=1 PROBE_ITERS=3000 timeout -k 10 120 tools/probes/window_probe_$P | sed "s/^/$P: /"
  done
done
