"""Device marker planning (scan over 3-state balance maps) against the sequential host planner,
which is pinned to the reference goldens (OfflineDataProviderTest / Epochs.csv selections)."""
import numpy as np
import pytest

import eeg_dataanalysispackage_amd as fx
from eeg_dataanalysispackage_amd.brainvision import EEGMarker
from conftest import DOD01, DOD02

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = fx.Context(0)
    yield c
    c.close()


def markers(pos, stim):
    return [EEGMarker(i + 1, "Stimulus", f"S {s + 1}", int(p), 1, 0, int(s))
            for i, (p, s) in enumerate(zip(pos, stim))]


@pytest.mark.parametrize("n,seed,balance", [(1, 0, 0), (7, 1, 1), (1000, 2, -1),
                                            (200_003, 3, 0), (1_000_000, 4, 1)])
def test_scan_equals_sequential(ctx, n, seed, balance):
    rng = np.random.default_rng(seed)
    nf = 10 * n + 5000
    pos = rng.integers(-50, nf + 300, size=n)      # some cuts leave the recording
    stim = rng.integers(-1, 6, size=n).astype(np.int32)
    guessed = 3
    hp, hl, hb = fx.plan_markers(markers(pos, stim), nf, guessed, balance) if n <= 200_003 else \
        host_plan(pos, stim, nf, guessed, balance)
    dp, dl, db = ctx.plan_markers(pos, stim, nf, guessed, balance)
    assert np.array_equal(dp, hp) and np.array_equal(dl, hl) and db == hb
    import torch
    tp, tl, tb = ctx.plan_markers(torch.from_numpy(pos).cuda(),
                                  torch.from_numpy(stim).cuda(), nf, guessed, balance)
    torch.cuda.synchronize()
    assert np.array_equal(tp.cpu().numpy(), hp) and np.array_equal(tl.cpu().numpy(), hl)
    assert tb == hb


def host_plan(pos, stim, nf, guessed, d):
    """Sequential restatement (same rules as eegfx_plan_markers) for sizes where building
    EEGMarker objects is slow."""
    out_p, out_l = [], []
    for p, s in zip(pos.tolist(), stim.tolist()):
        if p - 100 < 0 or p - 100 > nf:
            continue
        t = s + 1 == guessed
        if t and d <= 0:
            d += 1
            out_p.append(p); out_l.append(1.0)
        elif not t and d >= 0:
            d -= 1
            out_p.append(p); out_l.append(0.0)
    return np.array(out_p, dtype=np.int64), np.array(out_l), d


@pytest.mark.parametrize("base,guessed", [(DOD01, 1), (DOD02, 4)])
def test_reference_recordings(ctx, base, guessed):
    mk = fx.read_markers(base + ".vmrk")
    nf = fx.read_raw(base + ".vhdr", base + ".eeg").shape[0]
    hp, hl, hb = fx.plan_markers(mk, nf, guessed)
    pos = np.array([m.position for m in mk], dtype=np.int64)
    stim = np.array([m.stimulus_index for m in mk], dtype=np.int32)
    dp, dl, db = ctx.plan_markers(pos, stim, nf, guessed)
    assert np.array_equal(dp, hp) and np.array_equal(dl, hl) and db == hb


def test_unparsable_description_keeps_prefix(ctx):
    pos = np.arange(200, 2200, 100, dtype=np.int64)
    stim = np.array([0, 1] * 10, dtype=np.int32)
    stim[13] = np.iinfo(np.int32).min
    with pytest.raises(fx.EegfxError) as e:
        ctx.plan_markers(pos, stim, 10_000, 1)
    assert e.value.args[0] in (-3, "EFORMAT") or "EFORMAT" in str(e.value)
    with pytest.raises(fx.EegfxError):
        ctx.plan_markers(pos, stim, 10_000, 1, balance=2)
