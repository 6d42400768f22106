#!/bin/bash
set -euo pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_logreg.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
timeout -k 10 300 python bench.py --workload logreg | cut -c 400-900
