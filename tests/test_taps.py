"""The collapsed filter table (csrc/dwt8_taps.h) against its generator and the cascade it replaces.

dwt8_collapsed_cascade (csrc/dwt8.h) runs levels 1-5 of the fe=dwt-8 pyramid
(WaveletTransform.java:126-137) as one 280-tap filter at stride 32.  These
checks pin the committed header to gen_taps.py, the table to the exact rational composition of
the 12-decimal taps, and the kernel's lane algebra (ten partial sums per lane, four received from
lanes s+1..s+4; each pair's update in the direct and in the four-point Toom form; the six-point
form of the 4-lanes-per-signal window kernel) to the level-by-level cascade of the oracle.
"""
import ctypes
import os
import sys
from fractions import Fraction

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "eeg_dataanalysispackage_amd", "csrc")
sys.path.insert(0, CSRC)
import gen_taps  # noqa: E402


def test_header_is_generated():
    with open(os.path.join(CSRC, "dwt8_taps.h")) as f:
        assert f.read() == gen_taps.header_text()


def test_table_is_the_rounded_exact_composition():
    H = gen_taps.combined_taps()
    assert len(H) == 280
    h = [Fraction(v) for v in gen_taps.H_LITERALS]
    # the composition is the polyphase product of the five stages: its sum is sum(h)^5
    assert sum(H) == sum(h) ** 5
    for n in range(32):
        for j in range(9):
            m = n + 32 * j
            assert gen_taps.tap(n, j) == (float(H[m]) if m < 280 else 0.0)
    rows, tail = gen_taps.table()
    assert len(rows) == 32 and all(len(r) == 8 for r in rows) and len(tail) == 32
    assert tail[24:] == (0.0,) * 8


def _lane_model(x, tab):
    """The direct form's arithmetic order for one 512-sample signal (8 lanes), in numpy doubles."""
    P = np.zeros((8, 10))
    for s in range(8):
        xs = x[64 * s:64 * s + 64]
        for n in range(32):
            for j in range(9):
                if n + 32 * j >= 280:
                    continue
                P[s][j + 1] = P[s][j + 1] + xs[n] * tab(n, j)
                P[s][j] = P[s][j] + xs[n + 32] * tab(n, j)
    a5 = np.zeros(16)
    for s in range(8):
        a5[2 * s] = P[s][1] + sum(P[(s + d) % 8][2 * d + 1] for d in range(1, 5))
        a5[2 * s + 1] = P[s][0] + sum(P[(s + d) % 8][2 * d] for d in range(1, 5))
    return a5


def test_lane_algebra_matches_the_cascade():
    h = np.array([float(v) for v in gen_taps.H_LITERALS])
    tab = gen_taps.tap
    rng = np.random.default_rng(7)
    for _ in range(4):
        x = rng.normal(size=512) * 300.0 + rng.normal() * 1000.0
        a = x
        for _lev in range(5):
            N = len(a)
            a = np.array([sum(h[t] * a[(2 * k + t) % N] for t in range(10)) for k in range(N // 2)])
        for got in (_lane_model(x, tab), _toom_lane_model(x, gen_taps.toom_rows()),
                    _toom6_lane_model(x, gen_taps.toom6_rows())):
            assert np.max(np.abs(got - a)) <= 1e-12 * np.max(np.abs(a))


def _toom_lane_model(x, rows):
    """The four-point (Toom) form of each pair's update: the nine taps of row n in three blocks
    (j mod 3); A0 += B0 x1, Ai += B2 x0, Bp += (B0+B1+B2)/2 (x1+x0), Bm += (B0-B1+B2)/2 (x1-x0)."""
    P = np.zeros((8, 10))
    for s in range(8):
        xs = x[64 * s:64 * s + 64]
        A0, Ai, Bp, Bm = np.zeros(3), np.zeros(3), np.zeros(3), np.zeros(3)
        for n in range(32):
            x0, x1 = xs[n], xs[n + 32]
            R = rows[n]
            for q in range(3):
                A0[q] += x1 * R[q]
                Ai[q] += x0 * R[3 + q]
                Bp[q] += (x1 + x0) * R[6 + q]
                Bm[q] += (x1 - x0) * R[9 + q]
        for q in range(3):
            P[s][3 * q] = A0[q] + (Ai[q - 1] if q else 0.0)
            P[s][3 * q + 1] = Bp[q] - Bm[q] - Ai[q]
            P[s][3 * q + 2] = Bp[q] + Bm[q] - A0[q]
        P[s][9] = Ai[2]
    a5 = np.zeros(16)
    for s in range(8):
        a5[2 * s] = P[s][1] + sum(P[(s + d) % 8][2 * d + 1] for d in range(1, 5))
        a5[2 * s + 1] = P[s][0] + sum(P[(s + d) % 8][2 * d] for d in range(1, 5))
    return a5


def toom6_interpolate(V0, Vi, V1, Vm1, V2, Vm2):
    """dwt8.h toom6_finish's interpolation of one q: the six coefficients c0..c5 of
    (B0 + w B1 + w^2 B2)(x3 + w x2 + w^2 x1 + w^3 x0) from the products at 0, inf, 1, -1, 2, -2
    (V1, Vm1 scaled by 1/2, V2, Vm2 by 1/24 through the table)."""
    S1, D1 = V1 + Vm1, V1 - Vm1        # c0 + c2 + c4, c1 + c3 + c5
    T2, U2 = V2 + Vm2, V2 - Vm2        # (c0 + 4 c2 + 16 c4) / 12, (c1 + 4 c3 + 16 c5) / 6
    c0, c5 = V0, Vi
    c4 = T2 - S1 / 3 + c0 / 4
    c2 = S1 - c0 - c4
    c3 = 2 * U2 - D1 / 3 - 5 * c5
    c1 = D1 - c3 - c5
    return [c0, c1, c2, c3, c4, c5]


def _toom6_lane_model(x, rows):
    """The six-point form with 4 lanes per signal: lane s owns samples 128 s + k; group n is the
    samples n + 32 t, t < 4, against the nine taps of row n; twelve partials P[m] (m = j + 3 - t),
    the lane's a5[4 s + i] = P_s[3 - i] + P_{s+1}[7 - i] + P_{s+2}[11 - i]."""
    P = np.zeros((4, 12))
    for s in range(4):
        xs = x[128 * s:128 * s + 128]
        acc = np.zeros((6, 3))  # V0, Vi, V1, Vm1, V2, Vm2
        for n in range(32):
            x0, x1, x2, x3 = (xs[n + 32 * t] for t in range(4))
            E1, O1 = x3 + x1, x2 + x0
            E2, O2 = 4 * x1 + x3, 4 * x0 + x2
            X = [x3, x0, E1 + O1, E1 - O1, 2 * O2 + E2, -2 * O2 + E2]
            R = rows[n]
            for k in range(6):
                for q in range(3):
                    acc[k][q] += X[k] * R[3 * k + q]
        c = [toom6_interpolate(*(acc[k][q] for k in range(6))) for q in range(3)]  # c[q][r]
        for m in range(12):
            q, r = divmod(m, 3)
            P[s][m] = (c[q][r] if q < 3 else 0.0) + (c[q - 1][r + 3] if q > 0 else 0.0)
    a5 = np.zeros(16)
    for s in range(4):
        for i in range(4):
            a5[4 * s + i] = P[s][3 - i] + P[(s + 1) % 4][7 - i] + P[(s + 2) % 4][11 - i]
    return a5


def test_toom6_rows_are_exactly_rounded():
    H = gen_taps.combined_taps()
    h = lambda m: H[m] if m < 280 else 0
    for n in range(32):
        R = gen_taps.toom6_rows()[n]
        for q in range(3):
            b0, b1, b2 = (Fraction(h(n + 32 * (3 * q + r))) for r in range(3))
            want = [b0, b2, (b0 + b1 + b2) / 2, (b0 - b1 + b2) / 2, (b0 + 2 * b1 + 4 * b2) / 24,
                    (b0 - 2 * b1 + 4 * b2) / 24]
            assert [R[3 * k + q] for k in range(6)] == [float(v) for v in want]


def test_toom_rows_are_exactly_rounded():
    """B0, B2 and the halved block sums (B0 + B1 + B2) / 2, (B0 - B1 + B2) / 2, exact and rounded
    once (0 past tap 279)."""
    H = gen_taps.combined_taps()
    h = lambda m: H[m] if m < 280 else 0
    for n in range(32):
        R = gen_taps.toom_rows()[n]
        for q in range(3):
            b0, b1, b2 = (h(n + 32 * (3 * q + r)) for r in range(3))
            assert R[q] == float(b0) and R[3 + q] == float(b2)
            assert R[6 + q] == float((b0 + b1 + b2) / 2) and R[9 + q] == float((b0 - b1 + b2) / 2)


def test_literals_are_the_kernel_taps():
    import re
    with open(os.path.join(CSRC, "dwt8.h")) as f:
        src = f.read()
    got = [re.search(r"#define EEGFX_H%d (\S+)" % j, src).group(1) for j in range(10)]
    assert got == gen_taps.H_LITERALS
