#!/bin/bash
set -euo pipefail
for P in 1 2 4 1 2; do echo -n "split $P: "; EEGFX_SPLIT=$P timeout -k 10 200 python bench.py --cpu-sample 0 --alt-steps 0 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])'; done
EEGFX_SPLIT=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "device_memory or fma" --timeout 120 --timeout-method thread 2>&1 | tail -1
