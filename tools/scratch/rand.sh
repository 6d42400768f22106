#!/bin/bash
set -euo pipefail
echo -n "const 3000: "; PROBE_ITERS=3000 timeout -k 10 60 tools/probes/window_probe_0
echo -n "random 3000: "; PROBE_RANDOM=1 PROBE_ITERS=3000 timeout -k 10 60 tools/probes/window_probe_0
echo -n "random 10: "; PROBE_RANDOM=1 PROBE_ITERS=10 timeout -k 10 60 tools/probes/window_probe_0
