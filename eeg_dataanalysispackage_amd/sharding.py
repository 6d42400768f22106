"""Epoch-range sharding over ranks and the feature gather.

After marker planning (a sequential, host-side pass -- the class-balance state of
OffLineDataProvider.java:248-260 carries across markers and files) every selected epoch is
independent, so ranks take contiguous ranges of the selected-epoch list and run the fused kernel on
their range with no data-path collective.  The only exchange is moving the per-rank feature
matrices to their consumers, in rank order, which is the reference's list order
(``getData()`` order).  On MI355X nodes that is one RCCL all-gather over xGMI (backend "nccl");
the same code runs on gloo for the CPU tests.
"""
from __future__ import annotations

from typing import Tuple


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced [start, end) of n items for `rank` (first n % world ranks get +1)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_features(local, n_total: int, group=None):
    """All-gathers the per-rank feature rows [n_r][F] into [n_total][F] in rank order.

    Shards may differ by one row (shard_range), so rows are padded to the largest shard for the
    collective and the padding is dropped afterwards.  Works for any torch.distributed backend
    (RCCL "nccl" on the GPUs, gloo on CPU)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    sizes = [shard_range(n_total, r, world) for r in range(world)]
    width = max(e - s for s, e in sizes)
    feat = local.shape[1] if local.dim() == 2 else 0
    padded = torch.zeros((width, feat), dtype=local.dtype, device=local.device)
    padded[: local.shape[0]] = local
    full = torch.empty((world * width, feat), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(full, padded, group=group)
    parts = [full[r * width: r * width + (e - s)] for r, (s, e) in enumerate(sizes)]
    return torch.cat(parts, dim=0)
