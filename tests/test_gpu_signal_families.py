"""Parity of the fused path on structured signals, not only random walks (test_gpu_fuzz_fused.py).

The fma filter bank regroups the fp64 sums (levels 1-5 as one 280-tap filter, each
sample pair's update in the four-point form), so its rounding differs from the reference's
level-by-level order. These families probe where that could matter: full-scale white noise,
sinusoids from 1 Hz up to 450 Hz (the upper ones sit in the low-pass filter's stop band, so the
kept coefficients are small against the samples), square waves clipped at the int16 limits, and
steps. EXACT must equal the oracle value for value; FMA within 1e-9 per feature (the north_star
tolerance), for the 3-channel and the 32-channel kernels.
"""
import zlib

import numpy as np
import pytest

import eeg_dataanalysispackage_amd as fx
from oracle import oracle

pytestmark = pytest.mark.gpu

FAMILIES = ["noise", "sine1", "sine10", "sine40", "sine120", "sine250", "sine450", "square",
            "step"]


@pytest.fixture(scope="module")
def ctxs():
    a, b = fx.Context(0, numerics="exact"), fx.Context(0, numerics="fma")
    yield a, b
    a.close()
    b.close()


def signal(family, nf, ct, rng):
    t = np.arange(nf, dtype=np.float64)[:, None] / 1000.0
    phase = rng.uniform(0, 2 * np.pi, size=(1, ct))
    if family == "noise":
        x = rng.integers(-32768, 32768, size=(nf, ct))
    elif family.startswith("sine"):
        f = float(family[4:])
        x = -5000 + 20000 * np.sin(2 * np.pi * f * t + phase)
    elif family == "square":
        x = np.where(np.sin(2 * np.pi * 7.0 * t + phase) >= 0, 40000, -40000)  # clipped
    else:  # steps every 333 frames
        x = 3000 * ((np.arange(nf)[:, None] // 333) % 5) - 6000 + np.zeros((1, ct))
    return np.clip(np.rint(x), -32768, 32767).astype(np.int16)


@pytest.mark.parametrize("ct", [3, 32])
@pytest.mark.parametrize("family", FAMILIES)
def test_signal_family(ctxs, family, ct):
    rng = np.random.default_rng(zlib.crc32(f"{family}/{ct}".encode()))
    n = 40 if ct == 3 else 12
    nf = 1000 * n + 1500
    raw = signal(family, nf, ct, rng)
    pos = 1000 + 1000 * np.arange(n, dtype=np.int64) + rng.integers(0, 300, size=n)
    cols = list(range(ct))
    res = [0.1] * ct
    want = oracle.process_recording(raw, cols, res, pos)
    exact, fma = ctxs
    got = exact.process_recording(raw, ct, cols, res, pos)
    assert np.array_equal(got, want, equal_nan=True), family
    got_f = fma.process_recording(raw, ct, cols, res, pos)
    fin = np.isfinite(want)
    assert np.array_equal(np.isfinite(got_f), fin)
    assert np.max(np.abs(got_f[fin] - want[fin]), initial=0.0) <= 1e-9, family
