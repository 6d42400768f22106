#!/bin/bash
set -euo pipefail
for I in 10 30 100 300 1000 3000; do echo -n "iters $I: "; PROBE_ITERS=$I timeout -k 10 60 tools/probes/window_probe_0; done
for V in d31 d32 d34; do echo -n "$V 3000: "; EEGFX_FUSED_IMPL=$V PROBE_ITERS=3000 timeout -k 10 60 tools/probes/window_probe_0; done
echo -n "h1 3000: "; PROBE_ITERS=3000 timeout -k 10 60 tools/probes/window_probe_h1
for W in 3 50 200; do for S in 20 200; do echo "bench warmup $W steps $S: $(timeout -k 10 120 python bench.py --cpu-sample 0 --alt-steps 0 --warmup $W --steps $S | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"; done; done
