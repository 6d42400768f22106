#!/bin/bash
set -euo pipefail
for C in 2097152 4194304 8388608 16777216; do echo -n "chunk $C: "; timeout -k 10 200 python bench.py --workload stream --chunk-frames $C --steps 20 --warmup 3 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["host_link"]["h2d_GBps"])'; done
