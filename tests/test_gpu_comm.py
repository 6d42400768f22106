"""The multi-GPU boundary through the C ABI (eegfx_comm_*, eegfx_gather).

The GPU box has one device, so the RCCL communicators here have one rank (the ragged multi-rank
partition and rank-order assembly are covered on CPU by tests/test_distributed.py through the
same shard_range; eegfx_gather's per-root broadcasts use exactly those ranges)."""
import numpy as np
import pytest
import torch

import eeg_dataanalysispackage_amd as fx
from eeg_dataanalysispackage_amd._lib import check
from eeg_dataanalysispackage_amd.sharding import Comm, native_shard_range

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = fx.Context(0)
    yield c
    c.close()


def _rows(n, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn((n, 48), generator=g, dtype=torch.float64).cuda()


def test_single_rank_gather(ctx):
    comm = Comm(ctx, 1, 0, Comm.unique_id())
    assert comm.rank_world() == (0, 1)
    local = _rows(1000, 1)
    torch.cuda.synchronize()
    out = comm.gather(local, 1000)
    ctx.synchronize()
    assert torch.equal(out, local)
    comm.close()


def test_init_all_and_group(ctx):
    comms = Comm.init_all([ctx])
    local = _rows(37, 2)
    out = torch.full((37, 48), float("nan"), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    fx.lib().eegfx_group_start()
    comms[0].gather(local, 37, out=out)
    fx.lib().eegfx_group_end()
    ctx.synchronize()
    assert torch.equal(out, local)
    for c in comms:
        c.close()


def test_gather_after_fused_path(ctx):
    """Shard -> fused kernels -> gather, world 1: the gathered matrix is the resident result."""
    comm = Comm(ctx, 1, 0, Comm.unique_id())
    rng = np.random.default_rng(4)
    raw = (rng.integers(-26000, -24000, size=(1, 3)) +
           np.cumsum(rng.integers(-40, 41, size=(70000, 3)), axis=0)).astype(np.int16)
    pos = np.arange(1000, 69000, 1000)
    s, e = native_shard_range(len(pos), 0, 1)
    local = torch.from_numpy(ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos[s:e])).cuda()
    torch.cuda.synchronize()
    out = comm.gather(local, len(pos))
    ctx.synchronize()
    assert torch.equal(out, local)
    comm.close()


def test_single_rank_gather_root(ctx):
    """eegfx_gather_root at world 1: the root's own shard is copied (or left in place when
    `local` already is the output rows); `out` comes back on the root."""
    comm = Comm(ctx, 1, 0, Comm.unique_id())
    local = _rows(999, 5)
    torch.cuda.synchronize()
    out = comm.gather_root(local, 999, root=0)
    ctx.synchronize()
    assert torch.equal(out, local) and out.data_ptr() != local.data_ptr()
    same = comm.gather_root(local, 999, root=0, out=local)  # in place: no copy issued
    ctx.synchronize()
    assert same.data_ptr() == local.data_ptr() and torch.equal(same, out)
    empty = comm.gather_root(_rows(0, 6), 0)
    ctx.synchronize()
    assert tuple(empty.shape) == (0, 48)
    with pytest.raises(ValueError):
        comm.gather_root(local, 999, root=1)
    with pytest.raises(fx.EegfxError):
        check(fx.lib().eegfx_gather_root(comm.handle, local.data_ptr(), 999, 48, 0, None))
    comm.close()


def test_gather_errors(ctx):
    comm = Comm(ctx, 1, 0, Comm.unique_id())
    with pytest.raises(fx.EegfxError):
        check(fx.lib().eegfx_gather(comm.handle, None, 5, 48, None))
    with pytest.raises(ValueError):
        Comm(ctx, 1, 0, b"short")
    comm.close()
