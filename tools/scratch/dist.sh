#!/bin/bash
# Rehearsal of the N>1 bench control flow on a one-GPU box: 2 ranks on cuda:0 over gloo.
set -euo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --epochs 200000 --dist-backend gloo --same-device > gpurun_out/dist_c3.log 2>&1 || { grep -v "^\s*$" gpurun_out/dist_c3.log | grep -iE "error|Traceback|File|raise" | head -30; exit 1; }; tail -2 gpurun_out/dist_c3.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 3 --warmup 1 --epochs 100000 --workload c32 --dist-backend gloo --same-device 2>&1 | tail -3 | cut -c1-300
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --steps 2 --warmup 1 --workload stream --dist-backend gloo --same-device 2>&1 | tail -3 | cut -c1-300
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29536 bench.py --gpus 2 --steps 2 --warmup 1 --epochs 100000 --workload logreg --dist-backend gloo --same-device 2>&1 | tail -3 | cut -c1-300
