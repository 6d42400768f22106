"""Randomised parity sweep of the fused path (seeded, so every run checks the same cases): random
layouts (int16 / float32, 1-40 channels, any selection and order, per-channel resolutions),
random marker sets with the legal edges (pos = 100, windows past the end, pos - 100 = n_frames)
and both numerics.  EXACT must equal the oracle value for value; FMA within 1e-9 per feature."""
import numpy as np
import pytest

import eeg_dataanalysispackage_amd as fx
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctxs():
    a, b = fx.Context(0, numerics="exact"), fx.Context(0, numerics="fma")
    yield a, b
    a.close()
    b.close()


def case(seed):
    rng = np.random.default_rng(1000 + seed)
    ct = int(rng.integers(1, 41))
    C = int(rng.integers(1, min(ct, 8) + 1)) if seed % 5 else ct  # every 5th: all channels
    cols = [int(c) for c in rng.permutation(ct)[:C]]
    res = [float(np.float32(r)) for r in rng.choice([0.1, 0.5, 1.0, 0.0488281, 2.5], size=C)]
    nf = int(rng.integers(800, 6000))
    if seed % 3 == 0:
        raw = (rng.standard_normal((nf, ct)) * rng.choice([1.0, 50.0, 3000.0])).astype(np.float32)
    else:
        base = rng.integers(-30000, 30000, size=(1, ct))
        raw = np.clip(base + np.cumsum(rng.integers(-60, 61, size=(nf, ct)), axis=0), -32768,
                      32767).astype(np.int16)
    n = int(rng.integers(1, 40))
    pos = rng.integers(100, nf + 101, size=n)
    pos[0] = 100
    if n > 1:
        pos[-1] = nf + 100
    return raw, ct, cols, res, pos


@pytest.mark.parametrize("seed", range(40))
def test_random_layouts(ctxs, seed):
    exact, fma = ctxs
    raw, ct, cols, res, pos = case(seed)
    want = oracle.process_recording(raw, cols, res, pos)
    got = exact.process_recording(raw, ct, cols, res, pos)
    assert np.array_equal(got, want, equal_nan=True), (seed, ct, cols)
    got_f = fma.process_recording(raw, ct, cols, res, pos)
    fin = np.isfinite(want)
    assert np.array_equal(np.isfinite(got_f), fin)
    assert np.max(np.abs(got_f[fin] - want[fin]), initial=0.0) <= 1e-9, (seed, ct, cols)
