"""Randomised parity sweep of the two specialised window kernels (seeded): window_kernel (int16,
3 of 3 channels: configs[1] / configs[2]) and window_c32_kernel (int16, 32 of 32: configs[3]).

Each case varies what those kernels branch on:
- the channel order and per-channel resolutions;
- the marker density: sparse markers take the non-temporal window DMA, dense ones (windows
  overlapping) the cached one;
- unsorted and duplicate positions, pos = 100, windows past the end, pos - 100 = n_frames;
- batch sizes that leave partial 8-epoch sub-tiles and 64-epoch baseline tiles.

EXACT must equal the oracle value for value; FMA within 1e-9 per feature."""
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


def case(seed, ct):
    rng = np.random.default_rng(5000 + seed + 100 * ct)
    cols = [int(c) for c in rng.permutation(ct)]
    res = [float(np.float32(r)) for r in rng.choice([0.1, 0.5, 1.0, 0.0488281, 2.5], size=ct)]
    n = int(rng.integers(1, 300 if ct == 3 else 90))
    dense = seed % 2 == 1
    spacing = int(rng.integers(60, 400)) if dense else int(rng.integers(900, 1500))
    nf = 200 + spacing * n + int(rng.integers(0, 900))
    base = rng.integers(-30000, 30000, size=(1, ct))
    raw = np.clip(base + np.cumsum(rng.integers(-80, 81, size=(nf, ct)), axis=0), -32768,
                  32767).astype(np.int16)
    pos = 100 + spacing * np.arange(n, dtype=np.int64) + rng.integers(0, spacing // 2, size=n)
    pos = np.minimum(pos, nf + 100)
    if seed % 3 == 0:
        rng.shuffle(pos)                      # unsorted
    if n > 3 and seed % 4 == 0:
        pos[1] = pos[2]                       # a duplicate
    pos[0] = 100
    if n > 1:
        pos[-1] = nf + 100 if seed % 5 else nf - 300  # empty epoch / window past the end
    return raw, cols, res, pos


@pytest.mark.parametrize("seed", range(24))
def test_window_kernel_c3(ctxs, seed):
    _check(ctxs, *case(seed, 3), 3, seed)


@pytest.mark.parametrize("seed", range(8))
def test_window_c32_kernel(ctxs, seed):
    _check(ctxs, *case(seed, 32), 32, seed)


def _check(ctxs, raw, cols, res, pos, ct, seed):
    exact, fma = ctxs
    want = oracle.process_recording(raw, cols, res, pos)
    got = exact.process_recording(raw, ct, cols, res, pos)
    assert np.array_equal(got, want, equal_nan=True), (seed, cols)
    got_f = fma.process_recording(raw, ct, cols, res, pos)
    fin = np.isfinite(want)
    assert np.array_equal(np.isfinite(got_f), fin)
    assert np.max(np.abs(got_f[fin] - want[fin]), initial=0.0) <= 1e-9, (seed, cols)
