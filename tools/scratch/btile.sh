#!/bin/bash
set -euo pipefail
for T in 64 32 16 128; do echo -n "tile $T: "; EEGFX_BASE_TILE=$T timeout -k 10 200 python bench.py --cpu-sample 0 --alt-steps 0 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], round(d["ms_per_step"]-d["roofline"]["kernel_ms"],4))'; done
EEGFX_BASE_TILE=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
