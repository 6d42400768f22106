"""The fma conditioning guard's constants (csrc/guard.h) against their derivation
(tools/fma_bound.py), and the derivation against exact arithmetic (CPU only).

* guard.h's K2 for each fma form is at least the bound tools/fma_bound.py derives (and not
  needlessly larger);
* the EXACT cascade of the oracle (the reference's operation order) stays within the derived
  E_exact * max|x| of the exact rational result M x, on random, smooth, alternating and
  impulse windows -- the bound is an upper bound in practice, not only on paper;
* on the reference's recordings the balanced selections are certified by the a-priori X bound
  of int16 data (no recomputation on the golden flows), while the flat windows at the end of
  DoD2015_01 are not (they are rounding residue: the guard sends them to EXACT).
"""
import os
import re
import sys
from fractions import Fraction

import numpy as np
import pytest

from conftest import DOD01, DOD02, REPO
from oracle import oracle

sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "eeg_dataanalysispackage_amd", "csrc"))
import fma_bound  # noqa: E402
import gen_taps  # noqa: E402

GUARD_H = os.path.join(REPO, "eeg_dataanalysispackage_amd", "csrc", "guard.h")


def header_constant(name):
    text = open(GUARD_H).read()
    m = re.search(r"constexpr double %s = ([0-9.eE+-]+);" % name, text)
    assert m, name
    return float(m.group(1))


def test_guard_constants_match_derivation():
    c = fma_bound.constants()
    for name, key in (("kGuardK2Collapsed", "collapsed_k2"), ("kGuardK2Cascade", "cascade_k2"),
                      ("kGuardK2Toom6", "toom6_k2")):
        k2 = header_constant(name)
        assert c[key] <= k2 <= 1.02 * c[key], (name, k2, c[key])


def exact_features(x):
    """a6 || d6 of one 512-sample window in exact rational arithmetic (12-decimal taps)."""
    H = gen_taps.combined_taps()
    h = [Fraction(v) for v in gen_taps.H_LITERALS]
    g = [h[9 - j] if j & 1 else -h[9 - j] for j in range(10)]
    xf = [Fraction(float(v)) for v in x]
    a5 = [sum(H[m] * xf[(32 * k + m) % 512] for m in range(280)) for k in range(16)]
    a6 = [sum(h[j] * a5[(2 * i + j) % 16] for j in range(10)) for i in range(8)]
    d6 = [sum(g[j] * a5[(2 * i + j) % 16] for j in range(10)) for i in range(8)]
    return a6 + d6


H64 = np.array([float(v) for v in gen_taps.H_LITERALS])
G64 = np.array([H64[9 - j] if j & 1 else -H64[9 - j] for j in range(10)])


def cascade_unnormalised(x):
    """The reference's EXACT cascade on one window, before normalisation: each tap one rounded
    multiply and one rounded add, j = 0..9, periodic (numpy does not fuse).  Its normalised rows
    are checked bit-equal to the oracle's below."""
    a = np.asarray(x, dtype=np.float64)
    for level in range(6):
        n = a.size
        idx = (2 * np.arange(n // 2)[:, None] + np.arange(10)[None, :]) % n
        lo = a[idx[:, 0]] * H64[0]
        hi = a[idx[:, 0]] * G64[0]
        for j in range(1, 10):
            lo = lo + a[idx[:, j]] * H64[j]
            hi = hi + a[idx[:, j]] * G64[j]
        if level == 5:
            return np.concatenate([lo, hi])
        a = lo


@pytest.mark.parametrize("kind", ["random", "smooth", "alternating", "impulse", "dc"])
def test_exact_cascade_within_derived_bound(kind):
    rng = np.random.default_rng(sum(map(ord, kind)))
    t = np.arange(512)
    x = {"random": rng.standard_normal(512) * 1e3,
         "smooth": 500 * np.sin(2 * np.pi * t / 200) + 30 * t / 512,
         "alternating": np.where(t % 2 == 0, 1.0, -1.0) * 3276.7,
         "impulse": np.where(t == 301, 2.5e3, 0.0),
         "dc": np.full(512, -2500.25)}[kind].astype(np.float32).astype(np.float64)
    f_exact = exact_features(x)
    f = cascade_unnormalised(x)
    ep = np.zeros((1, 1, 750))
    ep[0, 0, 175:687] = x
    acc = 0.0
    for v in f:
        acc = acc + v * v
    assert np.array_equal(f / np.sqrt(acc), oracle.extract_features(ep)[0])  # the oracle's order
    c = fma_bound.constants()
    X = float(np.max(np.abs(x)))
    for i in range(16):
        E = c["exact_a6"] if i < 8 else c["exact_d6"]
        assert abs(Fraction(float(f[i])) - f_exact[i]) <= Fraction(E * X), (kind, i)


def crude_ratio(raw, pos, measured=False, three_max=False):
    """|f| / sqrt(sum_c X_c^2) per epoch with the a-priori int16 bound of guard.h, or (measured)
    with the second stage's X_c = max |x_c| over the window (guard_measured_x2_wave), or
    (three_max) with the 3-channel kernels' cheaper 3 max_c X_c^2 >= sum_c X_c^2 (recheck_c3)."""
    ep = oracle.decode_epochs(raw, [0, 1, 2], [0.1] * 3, pos)
    feats = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos)
    out = []
    for e, p in enumerate(pos):
        f = np.concatenate([cascade_unnormalised(ep[e, c, 175:687]) for c in range(3)])
        nf = float(np.sqrt(np.sum(f * f)))
        assert np.allclose(f / nf, feats[e], atol=1e-12, equal_nan=True)
        sx = 0.0
        for c in range(3):
            b = np.float32(0.0)
            for i in range(100):
                b = np.float32(b + np.float32(np.float32(raw[p - 100 + i, c]) * np.float32(0.1)))
            b = np.float32(b / np.float32(100))
            if measured:
                X = float(np.max(np.abs(ep[e, c, 175:687]))) * (1 + 2.0 ** -20)
            else:
                X = (32768 * abs(float(np.float32(0.1))) + abs(float(b))) * (1 + 2.0 ** -20)
            sx += X * X
        if three_max:
            sx = 3 * max(float(np.max(np.abs(ep[e, c, 175:687]))) for c in range(3)) ** 2 * (1 + 2.0 ** -20)
        out.append(nf / np.sqrt(sx))
    return np.array(out)


def test_reference_selections_certified_by_int16_bound():
    from eeg_dataanalysispackage_amd import brainvision as bv
    k2 = max(header_constant("kGuardK2Collapsed"), header_constant("kGuardK2Cascade"),
             header_constant("kGuardK2Toom6"))
    for base, guessed in ((DOD01, 1), (DOD02, 4)):
        raw = bv.read_raw(base + ".vhdr", base + ".eeg")
        pos, _, _ = bv.plan_markers(bv.read_markers(base + ".vmrk"), raw.shape[0], guessed)
        r = crude_ratio(raw, pos)
        assert np.all(r * r >= k2), (base, r.min())
    # the flat end of DoD2015_01 (constant samples) is below the bound: recomputed under EXACT
    raw = bv.read_raw(DOD01 + ".vhdr", DOD01 + ".eeg")
    flat = [m.position for m in bv.read_markers(DOD01 + ".vmrk")
            if m.position >= 100 and m.position + 687 <= raw.shape[0]
            and np.ptp(raw[m.position + 175:m.position + 687], axis=0).max() == 0]
    assert flat
    r = crude_ratio(raw, flat[:2])
    assert np.all(r * r < header_constant("kGuardK2Collapsed"))
    assert np.all(r * r < header_constant("kGuardK2Toom6"))


def test_flat_windows_certified_by_the_second_stage():
    """Every marker of DoD2015_01 with a window (the flat end included) passes the guard's second
    stage, the row's measured max |x| per channel: the device recomputes none of them (asserted
    on the GPU by test_gpu_guard.py), while null-space windows still fail it."""
    from eeg_dataanalysispackage_amd import brainvision as bv
    k2 = max(header_constant("kGuardK2Collapsed"), header_constant("kGuardK2Toom6"))
    raw = bv.read_raw(DOD01 + ".vhdr", DOD01 + ".eeg")
    allpos = [m.position for m in bv.read_markers(DOD01 + ".vmrk") if m.position >= 100]
    crude = crude_ratio(raw, allpos)
    meas = crude_ratio(raw, allpos, measured=True)
    assert np.sum(crude * crude < k2) >= 9          # the a-priori test flags the flat windows
    assert np.all(meas * meas >= k2), meas.min()     # the measured one certifies all of them
    three = crude_ratio(raw, allpos, three_max=True)  # and so does recheck_c3's looser form,
    assert np.all(three * three >= 1e5 * k2), three.min()  # with five orders of magnitude to spare
    t = np.arange(12000)[:, None]
    alt = (np.where(t % 2 == 0, 1, -1) * 700 - 2000 + np.zeros((1, 3))).astype(np.int16)
    r = crude_ratio(alt, [1000, 2001, 3000], measured=True)
    assert np.all(r * r < k2)
    r = crude_ratio(alt, [1000, 2001, 3000], three_max=True)
    assert np.all(r * r < k2)
