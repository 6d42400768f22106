"""Epoch-range sharding over ranks and the feature gather.

After marker planning (a sequential, host-side pass -- the class-balance state of
OffLineDataProvider.java:248-260 carries across markers and files) every selected epoch is
independent, so ranks take contiguous ranges of the selected-epoch list and run the fused kernel on
their range with no data-path collective.  The only exchange is moving the per-rank feature
matrices to their consumers, in rank order, which is the reference's list order
(``getData()`` order).  The product gathers are :class:`Comm` over the C ABI:
``Comm.gather_root`` (``eegfx_gather_root``: the matrix on one rank -- the reference's single
consumer, ``getData()`` in one JVM -- by grouped RCCL send/recv, ragged shards landing directly in
their rows) and ``Comm.gather`` (``eegfx_gather``: the matrix on every rank, one RCCL broadcast
per rank inside a group).  :func:`gather_features_root` / :func:`gather_features` are the same
exchanges through ``torch.distributed`` (any backend -- gloo in the CPU tests), following the
same plans; ``bench.py`` times them beside the C-ABI legs.
"""
from __future__ import annotations

from typing import Sequence, Tuple


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


def gather_schedule(n_total: int, world: int):
    """eegfx_gather_schedule through the C ABI: per root, (first row, row count) of the broadcast
    eegfx_gather issues for it (host only)."""
    import numpy as np
    from ._lib import check, lib, ptr
    off = np.empty(world, dtype=np.int64)
    cnt = np.empty(world, dtype=np.int64)
    check(lib().eegfx_gather_schedule(n_total, world, ptr(off), ptr(cnt)))
    return [(int(o), int(c)) for o, c in zip(off, cnt)]


def gather_root_plan(n_total: int, world: int, rank: int, root: int = 0):
    """eegfx_gather_root_plan through the C ABI: the point-to-point operations eegfx_gather_root
    issues on `rank`, as (kind, peer, first row, rows) with kind "send" / "recv" / "copy"."""
    from ctypes import byref, c_int32
    from ._lib import GatherOp, check, lib
    ops = (GatherOp * max(1, world))()
    k = c_int32()
    check(lib().eegfx_gather_root_plan(n_total, world, rank, root, ops, byref(k)))
    kinds = ("send", "recv", "copy")
    return [(kinds[o.kind], int(o.peer), int(o.row), int(o.rows)) for o in ops[:k.value]]


def gather_features_root(local, n_total: int, root: int = 0, group=None):
    """The rooted gather through torch.distributed point-to-point ops, following
    gather_root_plan: returns [n_total][F] on `root`, None elsewhere."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    plan = gather_root_plan(n_total, world, rank, root)
    feat = local.shape[1]
    out = (torch.empty((n_total, feat), dtype=local.dtype, device=local.device)
           if rank == root else None)
    reqs = []
    for kind, peer, row, rows in plan:
        if kind == "send":
            reqs.append(dist.isend(local.contiguous(), peer, group=group))
        elif kind == "recv":
            reqs.append(dist.irecv(out[row:row + rows], peer, group=group))
        else:
            out[row:row + rows] = local
    for r in reqs:
        r.wait()
    return out


def native_shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """eegfx_shard_range through the C ABI (same partition as shard_range)."""
    from ctypes import byref, c_int64
    from ._lib import check, lib
    s, e = c_int64(), c_int64()
    check(lib().eegfx_shard_range(n, rank, world, byref(s), byref(e)))
    return s.value, e.value


class Comm:
    """An RCCL communicator bound to a Context (eegfx_comm_* in include/eegfx.h).

    ``Comm.unique_id()`` on rank 0, shipped to the other ranks out of band, then
    ``Comm(ctx, world, rank, uid)`` on every rank; ``Comm.init_all(ctxs)`` for one process that
    drives several devices.  ``gather_root(local, n_total, root)`` returns the [n_total][F]
    feature matrix in rank order on the root (None elsewhere); ``gather(local, n_total)`` returns
    it on every rank (device tensors, the context's stream)."""

    ID_BYTES = 128

    def __init__(self, ctx, world: int, rank: int, uid: bytes, _handle=None):
        from ctypes import byref, c_void_p, create_string_buffer
        from ._lib import check, lib
        self.ctx = ctx
        if _handle is not None:
            self.handle = _handle
            return
        if len(uid) != self.ID_BYTES:
            raise ValueError(f"unique id must be {self.ID_BYTES} bytes")
        h = c_void_p()
        buf = create_string_buffer(bytes(uid), self.ID_BYTES)
        check(lib().eegfx_comm_create(ctx.handle, world, rank, buf, byref(h)))
        self.handle = h

    @classmethod
    def unique_id(cls) -> bytes:
        from ctypes import create_string_buffer
        from ._lib import check, lib
        buf = create_string_buffer(cls.ID_BYTES)
        check(lib().eegfx_comm_unique_id(buf))
        return buf.raw

    @classmethod
    def init_all(cls, ctxs: Sequence) -> list:
        from ctypes import c_void_p
        from ._lib import check, lib
        n = len(ctxs)
        hs = (c_void_p * n)(*[c.handle for c in ctxs])
        out = (c_void_p * n)()
        check(lib().eegfx_comm_init_all(hs, n, out))
        return [cls(c, n, i, b"", _handle=c_void_p(out[i])) for i, c in enumerate(ctxs)]

    def rank_world(self) -> Tuple[int, int]:
        from ctypes import byref, c_int32
        from ._lib import check, lib
        r, w = c_int32(), c_int32()
        check(lib().eegfx_comm_rank(self.handle, byref(r), byref(w)))
        return r.value, w.value

    def gather(self, local, n_total: int, out=None):
        """local: this rank's rows [e - s][cols] (float64, on the communicator's device) with
        (s, e) = shard_range(n_total, rank, world); returns [n_total][cols] on every rank."""
        import torch
        from ._lib import lib
        rank, world = self.rank_world()
        s, e = shard_range(n_total, rank, world)
        if local.dim() != 2 or local.dtype != torch.float64 or not local.is_cuda:
            raise ValueError("local rows must be a 2-D float64 device tensor")
        if local.shape[0] != e - s:
            raise ValueError(f"rank {rank} holds {local.shape[0]} rows, its shard of {n_total} "
                             f"over {world} ranks is [{s}, {e})")
        cols = int(local.shape[1])
        if out is None:
            out = torch.empty((n_total, cols), dtype=torch.float64, device=local.device)
        elif (tuple(out.shape) != (n_total, cols) or out.dtype != torch.float64
              or not out.is_contiguous()):
            raise ValueError(f"out must be a contiguous float64 tensor of shape ({n_total}, {cols})")
        local = local.contiguous()
        self.ctx._call(1, local, lib().eegfx_gather, self.handle,
                       local.data_ptr() if local.numel() else None, n_total, cols, out.data_ptr())
        return out

    def gather_root(self, local, n_total: int, root: int = 0, out=None):
        """local: this rank's rows, as for gather(); returns [n_total][cols] on `root` (in
        getData() order) and None on every other rank (eegfx_gather_root)."""
        import torch
        from ._lib import lib
        rank, world = self.rank_world()
        if not 0 <= root < world:
            raise ValueError(f"root {root} outside world {world}")
        s, e = shard_range(n_total, rank, world)
        if local.dim() != 2 or local.dtype != torch.float64 or not local.is_cuda:
            raise ValueError("local rows must be a 2-D float64 device tensor")
        if local.shape[0] != e - s:
            raise ValueError(f"rank {rank} holds {local.shape[0]} rows, its shard of {n_total} "
                             f"over {world} ranks is [{s}, {e})")
        cols = int(local.shape[1])
        if rank == root:
            if out is None:
                out = torch.empty((n_total, cols), dtype=torch.float64, device=local.device)
            elif (tuple(out.shape) != (n_total, cols) or out.dtype != torch.float64
                  or not out.is_contiguous()):
                raise ValueError(f"out must be a contiguous float64 tensor of shape "
                                 f"({n_total}, {cols})")
        else:
            out = None
        local = local.contiguous()
        self.ctx._call(1, local, lib().eegfx_gather_root, self.handle,
                       local.data_ptr() if local.numel() else None, n_total, cols, root,
                       out.data_ptr() if out is not None and out.numel() else None)
        return out

    def close(self) -> None:
        from ._lib import check, lib
        if getattr(self, "handle", None):
            h, self.handle = self.handle, None
            check(lib().eegfx_comm_destroy(h))
