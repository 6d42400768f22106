#!/bin/bash
set -euo pipefail
for V in d41 d32 d34 d31; do for A in 0 1 6; do echo -n "$V "; EEGFX_FUSED_IMPL=$V timeout -k 10 60 tools/probes/window_probe_$A; done; done
