"""Rigorous forward-error constants of the two dwt-8 filter banks, for the fma conditioning guard.

Both numerics compute the 16 kept coefficients f = M x of one 512-sample window from the SAME
decoded doubles x (the fp32 decode is shared and order-exact), so they differ only by fp64
rounding.  This script propagates, operation by operation and in the kernels' own order, a bound
m on |value| and a bound e on |computed - exact| (exact = rational arithmetic with the 12-decimal
taps of WaveletTransform's eegdsp filter) for inputs |x_i| <= 1:

  rounded op:  e_out = (propagated e) + u * (m_out + propagated e),  u = 2^-53
  constants:   a stored double c of an exact rational c* adds |c - c*| * m_in

* EXACT (dwt8.h dwt8_cascade<false>, the reference's order): six levels of 10-tap dot products,
  each tap one rounded multiply and one rounded add.
* fma (dwt8.h dwt8_collapsed_core): levels 1-5 as the 280-tap filter in the four-point (Toom)
  pair form -- 32 pairs of 12 fma into A0/Ai/Bp/Bm, the interpolation, the cross-lane partial
  adds -- then level 6 as fir10 with fma; and dwt8_cascade<true> (the per-epoch drop-in kernel):
  six levels of fir10 with fma.  The larger of the two fma bounds is used.

The result, E_a6 / E_d6 = max over coefficients of (e_fma + e_exact), bounds
|f_fma - f_exact| <= E * X per coefficient for a signal with |x_i| <= X.  With rows normalised
(SignalProcessing.java:38-52), |f_fma/|f_fma| - f_exact/|f_exact|| <= 2 |f_fma - f_exact| / |f_fma|
(+ a few ulps of normalisation rounding), so a row is certified within TOL when
|f_fma|^2 >= (2 / TOL)^2 * sum_c 8 (E_a6^2 + E_d6^2) X_c^2.  Prints the constant the kernels use
(K2 = (2/TOL)^2 * 8 * (E_a6^2 + E_d6^2) * SAFETY, one per fma form) for TOL = 0.5e-9 (half the
1e-9 contract; the other half covers the normalisations' own rounding, ~1e-15).

Run:  python3 tools/fma_bound.py
"""
from fractions import Fraction
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "eeg_dataanalysispackage_amd", "csrc"))
import gen_taps  # noqa: E402

U = 2.0 ** -53
LIT = [Fraction(v) for v in gen_taps.H_LITERALS]


def ghigh(j):  # high-pass g[j] = (-1)^(j+1) h[9-j]
    return LIT[9 - j] if j & 1 else -LIT[9 - j]


class V:
    """(m, e): bound on |exact value| and on |computed - exact|."""
    __slots__ = ("m", "e")

    def __init__(self, m, e=0.0):
        self.m, self.e = float(m), float(e)


def rnd(m, e):
    return V(m, e + U * (m + e))


def cmul(a, c_exact):  # a * fl(c), rounded
    c = float(c_exact)
    rep = abs(Fraction(c) - c_exact)
    return rnd(abs(c_exact) * a.m, abs(c) * a.e + float(rep) * a.m)


def add(a, b):
    return rnd(a.m + b.m, a.e + b.e)


def fma(a, c_exact, s):  # a * fl(c) + s, one rounding
    c = float(c_exact)
    rep = abs(Fraction(c) - c_exact)
    return rnd(abs(c_exact) * a.m + s.m, abs(c) * a.e + float(rep) * a.m + s.e)


def exact_cascade():
    """Uniform bounds per level (every output of a level has the same operation structure)."""
    a = V(1.0)
    for _level in range(5):
        acc = cmul(a, LIT[0])
        for j in range(1, 10):
            acc = add(acc, cmul(a, LIT[j]))
        a = acc
    lo = cmul(a, LIT[0])
    hi = cmul(a, ghigh(0))
    for j in range(1, 10):
        lo = add(lo, cmul(a, LIT[j]))
        hi = add(hi, cmul(a, ghigh(j)))
    return lo, hi


def fma_collapsed():
    H = gen_taps.combined_taps()
    hh = lambda m: H[m] if m < len(H) else Fraction(0)
    x = V(1.0)
    xp = add(x, x)  # x1 + x0 (exact for decoded fp32 pairs; bounded as rounded)
    xm = add(x, x)
    # per lane: A0[q], Ai[q], Bp[q], Bm[q] over 32 pairs
    acc = {}
    for n in range(32):
        b = [[hh(n + 32 * (3 * q + r)) for q in range(3)] for r in range(3)]
        consts = {}
        for q in range(3):
            consts[("A0", q)] = (x, b[0][q])
            consts[("Ai", q)] = (x, b[2][q])
            consts[("Bp", q)] = (xp, (b[0][q] + b[1][q] + b[2][q]) / 2)
            consts[("Bm", q)] = (xm, (b[0][q] - b[1][q] + b[2][q]) / 2)
        for k, (src, c) in consts.items():
            if k[0] == "Ai" and n + 32 * (3 * k[1] + 2) >= 280:
                continue
            acc[k] = cmul(src, c) if k not in acc else fma(src, c, acc[k])
    P = [None] * 10
    for q in range(3):
        A0, Ai, Bp, Bm = acc[("A0", q)], acc[("Ai", q)], acc[("Bp", q)], acc[("Bm", q)]
        P[3 * q] = add(A0, acc[("Ai", q - 1)]) if q > 0 else A0
        P[3 * q + 1] = add(add(Bp, Bm), Ai)  # Bp - Bm - Ai: same bounds as adds
        P[3 * q + 2] = add(add(Bp, Bm), A0)
    P[9] = acc[("Ai", 2)]
    # a5[0] = P[1] + sum_d P[2d+1] (lanes s+d); a5[1] = P[0] + sum_d P[2d]
    a50, a51 = P[1], P[0]
    for d in range(1, 5):
        a50 = add(a50, P[2 * d + 1])
        a51 = add(a51, P[2 * d])
    a5 = V(max(a50.m, a51.m), max(a50.e, a51.e))
    lo = cmul(a5, LIT[0])
    hi = cmul(a5, ghigh(0))
    for j in range(1, 10):
        lo = fma(a5, LIT[j], lo)
        hi = fma(a5, ghigh(j), hi)
    return lo, hi


def fma_toom6():
    """dwt8.h dwt8_toom6_core (the 3-channel window kernel, 4 lanes per signal): per group of four
    samples the six evaluations X(0) = x3, X(inf) = x0, X(+-1) = (x3 + x1) +- (x2 + x0),
    X(+-2) = fma(+-2, fma(4, x0, x2), fma(4, x1, x3)), 6 x 3 accumulators over 32 groups, the
    interpolation (toom6_finish, in its operation order), three partials per a5 and level 6 as
    fir10 with fma."""
    H = gen_taps.combined_taps()
    hh = lambda m: H[m] if m < len(H) else Fraction(0)
    x = V(1.0)
    E1, O1 = add(x, x), add(x, x)
    X1 = add(E1, O1)
    Xm1 = add(E1, O1)
    E2, O2 = fma(x, Fraction(4), x), fma(x, Fraction(4), x)
    X2 = fma(O2, Fraction(2), E2)
    Xm2 = fma(O2, Fraction(-2), E2)
    acc = {}
    for n in range(32):
        for q in range(3):
            b0, b1, b2 = (Fraction(hh(n + 32 * (3 * q + r))) for r in range(3))
            terms = (("V0", x, b0), ("Vi", x, b2), ("V1", X1, (b0 + b1 + b2) / 2),
                     ("Vm1", Xm1, (b0 - b1 + b2) / 2), ("V2", X2, (b0 + 2 * b1 + 4 * b2) / 24),
                     ("Vm2", Xm2, (b0 - 2 * b1 + 4 * b2) / 24))
            for name, src, c in terms:
                if name == "Vi" and n + 32 * (3 * q + 2) >= 280:
                    continue
                k = (name, q)
                acc[k] = cmul(src, c) if k not in acc else fma(src, c, acc[k])
    third = Fraction(-1, 3)
    C = [[None] * 3 for _ in range(6)]
    for q in range(3):
        g = lambda k: acc[(k, q)]
        c0, c5 = g("V0"), g("Vi")
        S1, D1 = add(g("V1"), g("Vm1")), add(g("V1"), g("Vm1"))
        T2, U2 = add(g("V2"), g("Vm2")), add(g("V2"), g("Vm2"))
        c4 = fma(S1, third, fma(c0, Fraction(1, 4), T2))
        c2 = add(add(S1, c0), c4)
        c3 = fma(U2, Fraction(2), fma(D1, third, cmul(c5, Fraction(-5))))
        c1 = add(add(D1, c3), c5)
        for r, v in enumerate((c0, c1, c2, c3, c4, c5)):
            C[r][q] = v
    P = []
    for m in range(12):
        q, r = divmod(m, 3)
        if q == 0:
            P.append(C[r][0])
        elif q == 3:
            P.append(C[r + 3][2])
        else:
            P.append(add(C[r][q], C[r + 3][q - 1]))
    a5 = V(0.0)
    for i in range(4):  # a5[4s + i] = (P_s[3 - i] + P_s+1[7 - i]) + P_s+2[11 - i]
        t = add(add(P[3 - i], P[7 - i]), P[11 - i])
        a5 = V(max(a5.m, t.m), max(a5.e, t.e))
    lo = cmul(a5, LIT[0])
    hi = cmul(a5, ghigh(0))
    for j in range(1, 10):
        lo = fma(a5, LIT[j], lo)
        hi = fma(a5, ghigh(j), hi)
    return lo, hi


def fma_cascade():
    """dwt8_cascade<true> (features_small_kernel under fma): level-by-level fir10 with fma; the
    partial-sum halos of levels 2-5 split a chain between two lanes without adding roundings, and
    level 5 adds the second lane's partial with one more add (modelled on every output)."""
    a = V(1.0)
    for level in range(5):
        acc = cmul(a, LIT[0])
        for j in range(1, 10):
            acc = fma(a, LIT[j], acc)
        if level == 4:
            acc = add(acc, V(0.0))
        a = acc
    lo = cmul(a, LIT[0])
    hi = cmul(a, ghigh(0))
    for j in range(1, 10):
        lo = fma(a, LIT[j], lo)
        hi = fma(a, ghigh(j), hi)
    return lo, hi


def constants(tol=0.5e-9, safety=1.25):
    """Guard constants for both fma forms: K2 = (2/TOL)^2 * 8 * (E_a6^2 + E_d6^2) * SAFETY with
    E = e_fma + e_exact of the form ('collapsed': the fused and batch kernels; 'cascade':
    features_small_kernel)."""
    ex_lo, ex_hi = exact_cascade()
    out = dict(exact_a6=ex_lo.e, exact_d6=ex_hi.e, tol=tol, safety=safety)
    for name, (lo, hi) in (("collapsed", fma_collapsed()), ("cascade", fma_cascade()),
                           ("toom6", fma_toom6())):
        Ea, Ed = ex_lo.e + lo.e, ex_hi.e + hi.e
        out[name + "_a6"], out[name + "_d6"] = lo.e, hi.e
        out[name + "_E_a6"], out[name + "_E_d6"] = Ea, Ed
        out[name + "_k2"] = (2.0 / tol) ** 2 * 8 * (Ea * Ea + Ed * Ed) * safety
    return out


if __name__ == "__main__":
    c = constants()
    for k, v in c.items():
        print("%-16s %.6e" % (k, v))
    for name in ("collapsed", "cascade", "toom6"):
        k2 = c[name + "_k2"]
        print("%-9s per-row threshold: |f|^2 >= %.6e * sum_c X_c^2  (|f| >= %.4e * sqrt(sum X_c^2))"
              % (name, k2, k2 ** 0.5))
