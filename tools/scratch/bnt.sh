#!/bin/bash
# Non-temporal baseline reads (baseline_kernel) and non-temporal row stores (window_kernel).
set -euo pipefail
for R in 1 2; do
  for P in 0 bnt; do PROBE_BASELINE=1 PROBE_RANDOM=1 timeout -k 10 120 tools/probes/window_probe_$P | sed "s/^/$P: /"; done
  for P in 0 s2; do PROBE_RANDOM=1 PROBE_ITERS=3000 timeout -k 10 120 tools/probes/window_probe_$P | sed "s/^/$P: /"; done
done
