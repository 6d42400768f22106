#!/bin/bash
set -euo pipefail
echo "pack:"; PYTHONPATH=. timeout -k 10 200 python tools/scratch/host_fe.py 2>&1 | tail -2
echo "2d:"; EEGFX_2D=1 PYTHONPATH=. timeout -k 10 200 python tools/scratch/host_fe.py 2>&1 | tail -2
echo "pack:"; PYTHONPATH=. timeout -k 10 200 python tools/scratch/host_fe.py 2>&1 | tail -2
