"""The N>1 path with the device doing the work, rehearsed on the one-GPU box.

Every rank is its own process with its own eegfx context on device 0. It extracts its
`eegfx_shard_range` slice of the selected epochs through the C ABI (the fused kernels), and the
rows are assembled with the per-root broadcast plan that `eegfx_gather` runs
(`eegfx_gather_schedule`). gloo carries the broadcasts here, because RCCL refuses two ranks on one
device. Rank 0 checks the assembled matrix against the oracle over the whole recording, in
getData() order (OffLineDataProvider.java:370-372): bit-exact under EXACT, within 1e-9 under fma.
The RCCL transport itself runs at world 1 in tests/test_gpu_comm.py."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _recording(n):
    rng = np.random.default_rng(2024)  # the same recording on every rank
    nf = 1000 * n + 700
    raw = (rng.integers(-26000, -24000, size=(1, 3)) +
           np.cumsum(rng.integers(-40, 41, size=(nf, 3)), axis=0)).astype(np.int16)
    pos = np.arange(1000, 1000 * (n + 1), 1000, dtype=np.int64)
    pos[-1] = nf - 200  # the last window runs past the end: zero padding on the last rank
    return raw, pos


def _rank(rank, world, port, n, numerics, out_dir, mode="broadcast"):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import eeg_dataanalysispackage_amd as fx
    from eeg_dataanalysispackage_amd.sharding import gather_schedule, native_shard_range
    raw, pos = _recording(n)
    s, e = native_shard_range(n, rank, world)
    ctx = fx.Context(0, numerics=numerics)
    d_raw = torch.from_numpy(raw).cuda()
    d_pos = torch.from_numpy(pos[s:e]).cuda()
    local = ctx.process_recording(d_raw, 3, [0, 1, 2], [0.1] * 3, d_pos)  # device rows
    local = local.cpu()
    ctx.close()
    if mode == "root":  # eegfx_gather_root's send/recv plan, assembled on the last rank
        from eeg_dataanalysispackage_amd.sharding import gather_features_root
        full = gather_features_root(local, n, world - 1)
        if rank == world - 1:
            np.save(os.path.join(out_dir, "rows_root.npy"), full.numpy())
        else:
            assert full is None
        dist.barrier()
        dist.destroy_process_group()
        return
    out = torch.full((n, 48), float("nan"), dtype=torch.float64)
    for root, (off, cnt) in enumerate(gather_schedule(n, world)):
        if cnt == 0:
            continue
        buf = local.clone() if root == rank else torch.empty((cnt, 48), dtype=torch.float64)
        dist.broadcast(buf, src=root)
        out[off:off + cnt] = buf
    np.save(os.path.join(out_dir, f"rows{rank}.npy"), out.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,numerics", [(2, 37, "exact"), (3, 64, "exact"),
                                              (3, 10, "fma")])
def test_device_shards_assemble_in_getdata_order(tmp_path, world, n, numerics):
    import torch.multiprocessing as mp
    from oracle import oracle
    mp.spawn(_rank, args=(world, _free_port(), n, numerics, str(tmp_path)), nprocs=world,
             join=True)
    raw, pos = _recording(n)
    want = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos)
    for r in range(world):
        got = np.load(tmp_path / f"rows{r}.npy")
        if numerics == "exact":
            assert np.array_equal(got, want), f"rank {r}"
        else:
            assert np.max(np.abs(got - want)) <= 1e-9, f"rank {r}"


@pytest.mark.parametrize("world,n,numerics", [(3, 64, "exact"), (2, 11, "fma")])
def test_device_shards_gathered_on_root_in_getdata_order(tmp_path, world, n, numerics):
    """The rooted plan (eegfx_gather_root_plan): only the root holds the matrix, equal to the
    oracle over the whole recording in getData() order."""
    import torch.multiprocessing as mp
    from oracle import oracle
    mp.spawn(_rank, args=(world, _free_port(), n, numerics, str(tmp_path), "root"), nprocs=world,
             join=True)
    raw, pos = _recording(n)
    want = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos)
    got = np.load(tmp_path / "rows_root.npy")
    if numerics == "exact":
        assert np.array_equal(got, want)
    else:
        assert np.max(np.abs(got - want)) <= 1e-9
