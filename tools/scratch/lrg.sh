#!/bin/bash
set -euo pipefail
for G in 1024 512 256 2048; do echo -n "G=$G: "; EEGFX_LR_G=$G timeout -k 10 200 python bench.py --workload logreg --cpu-sample 0 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["ms_per_iteration"], r["achieved"])'; done
