#!/bin/bash
set -euo pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "streamed" --timeout 120 --timeout-method thread 2>&1 | tail -1
for C in 8388608 16777216; do echo -n "chunk $C: "; timeout -k 10 200 python bench.py --workload stream --chunk-frames $C | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); h=d["host_link"]; print(d["value"], d["ms_per_step"], h["h2d_GBps"], h["copy_only_ms"], h["frac"])'; done
