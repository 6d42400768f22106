#!/bin/bash
set -euo pipefail
for i in 1 2; do
echo "pool:"; PYTHONPATH=. timeout -k 10 200 python tools/scratch/host_fe.py 2>&1 | tail -2
echo "spawn:"; EEGFX_SPAWN=1 PYTHONPATH=. timeout -k 10 200 python tools/scratch/host_fe.py 2>&1 | tail -2
done
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
