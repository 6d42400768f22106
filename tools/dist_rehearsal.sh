#!/bin/bash
# The N > 1 bench path rehearsed on a one-GPU box (the driver runs the real 1/2/4/8-GPU lines):
#   force_dist  one rank, nccl process group, --force-dist: configs[2]'s 8M-epoch rank shard, the
#               C-ABI rooted gather (eegfx_gather_root), the all-ranks gather and the torch legs
#   torchrun2   torch.distributed.run with 2 ranks sharing cuda:0 (gloo process group: RCCL
#               refuses two ranks on one device), 8M epochs per rank, barriers + max-over-ranks
#               timing + the single rank-0 line
#   TAG=r03b bash tools/dist_rehearsal.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-dist}
mkdir -p "$OUT"
echo "== force_dist (world 1, nccl)"; date
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --force-dist --steps 20 --warmup 10 --alt-steps 0 \
  > "$OUT/bench_force_dist.json" 2> "$OUT/bench_force_dist.err" || { tail -30 "$OUT/bench_force_dist.err"; exit 1; }
cat "$OUT/bench_force_dist.json"
echo "== torchrun 2 ranks, same device"; date
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 10 --alt-steps 0 --same-device \
  --dist-backend gloo --no-gather > "$OUT/bench_torchrun2.json" 2> "$OUT/bench_torchrun2.err" || { tail -30 "$OUT/bench_torchrun2.err"; exit 1; }
cat "$OUT/bench_torchrun2.json"
echo "== torchrun 2 ranks, same device, gather legs over gloo (shard checksums)"; date
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29535 bench.py --gpus 2 --steps 5 --warmup 2 --alt-steps 0 --same-device \
  --dist-backend gloo --epochs 20000 > "$OUT/bench_torchrun2_gather.json" 2> "$OUT/bench_torchrun2_gather.err" || { tail -30 "$OUT/bench_torchrun2_gather.err"; exit 1; }
cat "$OUT/bench_torchrun2_gather.json"
echo "== done"; date
