#!/bin/bash
set -euo pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
PYTHONPATH=. timeout -k 10 200 python tools/scratch/epochs_path.py 2>&1 | tail -1
