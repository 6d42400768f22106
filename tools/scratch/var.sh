#!/bin/bash
# window_kernel variants (EEGFX_FUSED_IMPL = halo transport, min waves, sub-tiles per WG) and
# the level-0 halo-by-shuffle probe.
set -euo pipefail
for V in d41 d31 d42 d32 d44 d34 d48; do echo -n "$V "; EEGFX_FUSED_IMPL=$V timeout -k 10 60 tools/probes/window_probe_0; done
for V in d41 d31 d42; do echo -n "h1 $V "; EEGFX_FUSED_IMPL=$V timeout -k 10 60 tools/probes/window_probe_h1; done
echo -n "h1 nodma "; timeout -k 10 60 tools/probes/window_probe_h1a1
echo -n "d41 again "; timeout -k 10 60 tools/probes/window_probe_0
