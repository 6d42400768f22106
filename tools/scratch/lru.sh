#!/bin/bash
set -euo pipefail
for G in 1024 512; do echo -n "U4 G=$G: "; EEGFX_LR_G=$G timeout -k 10 200 python bench.py --workload logreg --cpu-sample 0 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["ms_per_iteration"], r["achieved"])'; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_logreg.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
