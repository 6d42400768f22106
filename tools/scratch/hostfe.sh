#!/bin/bash
set -euo pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread 2>&1 | tail -1
PYTHONPATH=. timeout -k 10 200 python tools/scratch/host_fe.py 2>&1 | tail -2
