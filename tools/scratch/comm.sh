#!/bin/bash
set -euo pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread 2>&1 | tail -15
