#!/bin/bash
set -euo pipefail
for V in d41 d51; do
  echo -n "packed $V: "; EEGFX_FUSED_IMPL=$V PROBE_RANDOM=1 PROBE_ITERS=2000 timeout -k 10 60 tools/probes/window_probe_0
  echo -n "scalar $V: "; EEGFX_FUSED_IMPL=$V PROBE_RANDOM=1 PROBE_ITERS=2000 timeout -k 10 60 tools/probes/window_probe_sc
done
echo -n "packed d41 again: "; PROBE_RANDOM=1 PROBE_ITERS=2000 timeout -k 10 60 tools/probes/window_probe_0
timeout -k 10 200 python bench.py --cpu-sample 0 --alt-steps 0 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])'
