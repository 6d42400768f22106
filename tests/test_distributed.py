"""Multi-rank path on CPU (gloo, world_size 2): epoch-range sharding + feature gather.

The per-rank compute here is the oracle (the CPU checker; the GPU ranks run the fused kernel on
the same ranges in bench.py).  Asserts that sharded extraction + all-gather reproduces the
single-process feature matrix bit for bit and in the reference's list order.
"""
import os
import socket

import numpy as np
import pytest

from eeg_dataanalysispackage_amd.sharding import shard_range


def test_shard_range_partitions():
    for n in (0, 1, 7, 64, 1000, 1_000_003):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def test_native_shard_range_matches():
    from eeg_dataanalysispackage_amd.sharding import native_shard_range
    import eeg_dataanalysispackage_amd as fx
    for n in (0, 1, 7, 64, 1_000_003, 64_000_000):
        for world in (1, 2, 3, 8):
            for r in range(world):
                assert native_shard_range(n, r, world) == shard_range(n, r, world)
    with pytest.raises(fx.EegfxError):
        native_shard_range(10, 2, 2)


def test_gather_schedule_matches_shard_range():
    """eegfx_gather_schedule (the per-root broadcast plan eegfx_gather runs) against shard_range,
    ragged n over 1..8 ranks: offsets are the shard starts, counts the shard sizes, and the plan
    covers [0, n) in rank (= getData()) order."""
    import eeg_dataanalysispackage_amd as fx
    from eeg_dataanalysispackage_amd.sharding import gather_schedule
    for n in (0, 1, 5, 7, 8, 9, 63, 64, 65, 1_000_003, 64_000_000, 64_000_007):
        for world in range(1, 9):
            plan = gather_schedule(n, world)
            assert plan == [(s, e - s) for s, e in (shard_range(n, r, world) for r in range(world))]
            assert sum(c for _, c in plan) == n
            assert all(o1 + c1 == o2 for (o1, c1), (o2, _) in zip(plan, plan[1:]))
    with pytest.raises(fx.EegfxError):
        gather_schedule(10, 0)
    with pytest.raises(fx.EegfxError):
        gather_schedule(-1, 2)


def test_gather_root_plan_matches_shard_range():
    """eegfx_gather_root_plan (the send/recv plan of the rooted gather) for ragged n over 1..8
    ranks and every root: the root receives each other rank's shard_range rows once, in rank
    order, and copies its own; every other rank with rows sends exactly its shard to the root;
    ranks without rows issue nothing; the root's operations tile [0, n) in getData() order."""
    import eeg_dataanalysispackage_amd as fx
    from eeg_dataanalysispackage_amd.sharding import gather_root_plan
    for n in (0, 1, 5, 7, 8, 9, 63, 64, 65, 1_000_003, 64_000_000, 64_000_007):
        for world in range(1, 9):
            spans = [shard_range(n, r, world) for r in range(world)]
            for root in range(world):
                plans = [gather_root_plan(n, world, r, root) for r in range(world)]
                got = plans[root]
                want = [("copy" if r == root else "recv", r, s, e - s)
                        for r, (s, e) in enumerate(spans) if e > s]
                assert got == want, (n, world, root)
                assert sum(op[3] for op in got) == n
                assert all(a[2] + a[3] == b[2] for a, b in zip(got, got[1:]))
                for r in range(world):
                    if r == root:
                        continue
                    s, e = spans[r]
                    assert plans[r] == ([("send", root, s, e - s)] if e > s else []), (n, world, r)
    with pytest.raises(fx.EegfxError):
        gather_root_plan(10, 2, 2, 0)
    with pytest.raises(fx.EegfxError):
        gather_root_plan(10, 2, 0, 2)
    with pytest.raises(fx.EegfxError):
        gather_root_plan(-1, 2, 0, 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, out_dir):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eeg_dataanalysispackage_amd.sharding import gather_features
    from oracle import oracle
    rng = np.random.default_rng(123)  # same recording on every rank
    nf = 1000 * n + 2000
    raw = (rng.integers(-26000, -24000, size=(1, 3)) +
           np.cumsum(rng.integers(-40, 41, size=(nf, 3)), axis=0)).astype(np.int16)
    pos = np.arange(1000, 1000 * (n + 1), 1000)
    s, e = shard_range(n, rank, world)
    local = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos[s:e])
    full = gather_features(torch.from_numpy(local), n).numpy()
    if rank == 0:
        ref = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos)
        np.save(os.path.join(out_dir, "ok.npy"), np.array([np.array_equal(full, ref)]))
    dist.barrier()
    dist.destroy_process_group()


def _schedule_worker(rank, world, port, n, out_dir):
    """eegfx_gather's collective pattern rehearsed on gloo: for every root of
    eegfx_gather_schedule one broadcast of that root's rows into out[offset : offset + count]
    (ncclBroadcast in eegfx_gather, dist.broadcast here); roots without rows issue nothing."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eeg_dataanalysispackage_amd.sharding import gather_schedule
    cols = 48
    full_ref = torch.arange(n * cols, dtype=torch.float64).reshape(n, cols)
    s, e = shard_range(n, rank, world)
    local = full_ref[s:e].clone()
    out = torch.full((n, cols), float("nan"), dtype=torch.float64)
    for root, (off, cnt) in enumerate(gather_schedule(n, world)):
        if cnt == 0:
            continue
        buf = local if root == rank else out[off:off + cnt]
        buf = buf.contiguous()
        dist.broadcast(buf, src=root)
        out[off:off + cnt] = buf
    np.save(os.path.join(out_dir, f"ok{rank}.npy"), np.array([torch.equal(out, full_ref)]))
    dist.barrier()
    dist.destroy_process_group()


def _root_worker(rank, world, port, n, root, out_dir):
    """eegfx_gather_root's pattern rehearsed on gloo (gather_features_root follows
    eegfx_gather_root_plan): extraction on each rank's shard (the oracle stands in for the kernels
    here), the matrix assembled on the root only, equal to the single-process matrix bit for bit
    in getData() order (OffLineDataProvider.java:370-372)."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eeg_dataanalysispackage_amd.sharding import gather_features_root
    from oracle import oracle
    rng = np.random.default_rng(321)
    nf = 1000 * n + 2000
    raw = (rng.integers(-26000, -24000, size=(1, 3)) +
           np.cumsum(rng.integers(-40, 41, size=(nf, 3)), axis=0)).astype(np.int16)
    pos = np.arange(1000, 1000 * (n + 1), 1000)
    s, e = shard_range(n, rank, world)
    local = torch.from_numpy(oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos[s:e])
                             .reshape(e - s, 48))
    full = gather_features_root(local, n, root)
    if rank == root:
        ref = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos)
        ok = np.array_equal(full.numpy(), ref)
    else:
        ok = full is None
    np.save(os.path.join(out_dir, f"ok{rank}.npy"), np.array([ok]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,root", [(2, 37, 0), (3, 7, 2), (4, 2, 1), (4, 9, 0)])
def test_gather_root_send_recv_world_n(tmp_path, world, n, root):
    import torch.multiprocessing as mp
    mp.spawn(_root_worker, args=(world, _free_port(), n, root, str(tmp_path)), nprocs=world,
             join=True)
    assert all(bool(np.load(tmp_path / f"ok{r}.npy")[0]) for r in range(world))


@pytest.mark.parametrize("world,n", [(3, 7), (4, 2), (2, 37)])
def test_gather_schedule_broadcasts_world_n(tmp_path, world, n):
    import torch.multiprocessing as mp
    mp.spawn(_schedule_worker, args=(world, _free_port(), n, str(tmp_path)), nprocs=world,
             join=True)
    assert all(bool(np.load(tmp_path / f"ok{r}.npy")[0]) for r in range(world))


@pytest.mark.parametrize("n", [37, 64])
def test_sharded_extraction_gather_world2(tmp_path, n):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(2, _free_port(), n, str(tmp_path)), nprocs=2, join=True)
    assert bool(np.load(tmp_path / "ok.npy")[0])
