#!/bin/bash
set -euo pipefail
for V in d41 d51; do
  echo -n "exact scalar $V: "; EEGFX_FUSED_IMPL=$V PROBE_EXACT=1 PROBE_RANDOM=1 PROBE_ITERS=1000 timeout -k 10 60 tools/probes/window_probe_0
  echo -n "exact packed $V: "; EEGFX_FUSED_IMPL=$V PROBE_EXACT=1 PROBE_RANDOM=1 PROBE_ITERS=1000 timeout -k 10 60 tools/probes/window_probe_pk
done
