"""Generates dwt8_taps.h: the five-level db5 low-pass (levels 1-5 of the fe=dwt-8 pyramid) as one
280-tap filter applied at stride 32, for the collapsed FMA cascade in dwt8.h.

The eegdsp transform (WaveletTransform.java:126-137) runs the 10-tap
low-pass h at stride 2 with periodic extension five times, 512 -> 16.  Because each level's
signal is periodic with a period that divides the previous one, the five levels compose to

    a5[k] = sum_{m < 280} H5[m] x[(32 k + m) mod 512],
    H1 = h,  Hj[m] = sum_t h[t] H(j-1)[m - 2^(j-1) t]   (lengths 10, 28, 64, 136, 280).

H5 is computed here exactly, in rational arithmetic from the 12-decimal literals, and rounded once
to the nearest double.  The kernel takes a lane's samples in pairs (n, n + 32), which meet taps
H5[n + 32 j], j = 0..8, and updates its partial sums in a four-point (Toom) form (dwt8.h): with the
nine taps of row n in three blocks by j mod 3, B0[q] = H5[n + 96 q], B1[q] = H5[n + 96 q + 32],
B2[q] = H5[n + 96 q + 64] (0 past tap 279), row n of the table holds B0[0..2], B2[0..2],
(B0 + B1 + B2)[0..2] / 2 and (B0 - B1 + B2)[0..2] / 2: 12 doubles, 96 bytes, each an exact rational
sum rounded once.  The direct form (A/B builds) follows: rows n < 32 of H5[n + 32 j], j < 8 (one
64-byte scalar load), then the j = 8 column H5[256 + n] as a tail of 32 entries (zero past 279).

The six-point form (dwt8.h dwt8_toom6_core, 4 lanes per signal) takes a lane's samples in groups
of four (n, n + 32, n + 64, n + 96), the same nine taps of row n: with B(w) = B0 + w B1 + w^2 B2 it
accumulates the products at w = 0, infinity, 1, -1, 2, -2; row n of its table holds B0[0..2],
B2[0..2], B(1)[0..2] / 2, B(-1)[0..2] / 2, B(2)[0..2] / 24 and B(-2)[0..2] / 24 (18 doubles, 144
bytes), each exact and rounded once.

Run from anywhere:  python3 eeg_dataanalysispackage_amd/csrc/gen_taps.py  (rewrites the header;
tests/test_taps.py checks the committed header against this generator).
"""
from fractions import Fraction
import functools
import os

# Low-pass taps (the same literals as dwt8.h EEGFX_H0..H9)
H_LITERALS = ["0.160102397974", "0.603829269797", "0.724308528438", "0.138428145901",
              "-0.242294887066", "-0.032244869585", "0.077571493840", "-0.006241490213",
              "-0.012580751999", "0.003335725285"]

LEVELS = 5
STRIDE = 1 << LEVELS      # 32
ROWS = 32                 # sample offsets n of a pair (n, n + 32)
COLS = 8                  # j = 0..7 per row; j = 8 in the tail
TOOM = 12                 # B0[3], B2[3], (B0 + B1 + B2)/2 [3], (B0 - B1 + B2)/2 [3]
TOOM6 = 18                # B0[3], B2[3], B(1)/2 [3], B(-1)/2 [3], B(2)/24 [3], B(-2)/24 [3]


@functools.lru_cache(maxsize=None)
def combined_taps(levels=LEVELS):
    """Exact rational taps of `levels` composed low-pass stages."""
    h = [Fraction(v) for v in H_LITERALS]
    H = list(h)
    for j in range(2, levels + 1):
        step = 1 << (j - 1)
        out = [Fraction(0)] * (len(H) + step * (len(h) - 1))
        for t, ht in enumerate(h):
            for m, Hm in enumerate(H):
                out[m + step * t] += ht * Hm
        H = out
    return H


@functools.lru_cache(maxsize=None)
def table():
    """Rows n < 32 of H5[n + 32 j], j < 8, then the tail H5[256 + n], n < 32 (0 past 279)."""
    H = [float(v) for v in combined_taps()]  # float(Fraction) rounds to nearest
    assert len(H) == 280
    rows = [[H[n + STRIDE * j] for j in range(COLS)] for n in range(ROWS)]
    tail = [H[256 + n] if 256 + n < len(H) else 0.0 for n in range(ROWS)]
    return tuple(tuple(r) for r in rows), tuple(tail)


@functools.lru_cache(maxsize=None)
def toom_rows():
    """Rows n < 32 of the four-point form's constants (see the module docstring)."""
    H = combined_taps()
    h = lambda m: H[m] if m < len(H) else 0
    rows = []
    for n in range(ROWS):
        b = [[h(n + STRIDE * (3 * q + r)) for q in range(3)] for r in range(3)]  # b[r][q]
        row = [b[0][q] for q in range(3)] + [b[2][q] for q in range(3)]
        row += [(b[0][q] + b[1][q] + b[2][q]) / 2 for q in range(3)]
        row += [(b[0][q] - b[1][q] + b[2][q]) / 2 for q in range(3)]
        rows.append(tuple(float(v) for v in row))
    return tuple(rows)


@functools.lru_cache(maxsize=None)
def toom6_rows():
    """Rows n < 32 of the six-point form's constants (see the module docstring)."""
    H = combined_taps()
    h = lambda m: H[m] if m < len(H) else 0
    rows = []
    for n in range(ROWS):
        b = [[Fraction(h(n + STRIDE * (3 * q + r))) for q in range(3)] for r in range(3)]
        B = lambda w, q: b[0][q] + w * b[1][q] + w * w * b[2][q]
        row = [b[0][q] for q in range(3)] + [b[2][q] for q in range(3)]
        row += [B(1, q) / 2 for q in range(3)] + [B(-1, q) / 2 for q in range(3)]
        row += [B(2, q) / 24 for q in range(3)] + [B(-2, q) / 24 for q in range(3)]
        rows.append(tuple(float(v) for v in row))
    return tuple(rows)


def tap(n, j):
    """H5[n + 32 j] as the kernel reads it from the table (0 past 279)."""
    rows, tail = table()
    return rows[n][j] if j < COLS else tail[n]


def header_text():
    lines = [
        "// dwt8_taps.h -- GENERATED by gen_taps.py; do not edit.",
        "// Levels 1-5 of the fe=dwt-8 low-pass pyramid as one 280-tap filter at stride 32",
        "// (WaveletTransform.java:126-137; exact rational composition of the 12-decimal taps, rounded",
        "// once).  Rows n < 32 of the four-point form's 12 constants (gen_taps.py), then the direct",
        "// form's rows n < 32 of H5[n + 32 j], j < 8, and its tail H5[256 + n] (0 past tap 279).",
        "// EEGFX_T6_TABLE: rows n < 32 of the six-point form's 18 constants (gen_taps.py).",
        "#pragma once",
        "",
        "namespace eegfx {",
        "namespace dev {",
        "",
        "constexpr int kH5Rows = %d, kH5Cols = %d;" % (ROWS, TOOM),
        "constexpr int kH5Direct = kH5Rows * kH5Cols, kH5DirectCols = %d;" % COLS,
        "constexpr int kH5Tail = kH5Direct + kH5Rows * kH5DirectCols;",
        "constexpr int kH5Size = kH5Tail + kH5Rows;",
        "constexpr int kT6Rows = %d, kT6Cols = %d;" % (ROWS, TOOM6),
        "#define EEGFX_H5_TABLE \\",
    ]
    rows, tail = table()
    body = ["    " + ", ".join(float.hex(v) for v in row) for row in toom_rows()]
    body += ["    " + ", ".join(float.hex(v) for v in row) for row in rows]
    body += ["    " + ", ".join(float.hex(v) for v in tail[i:i + 8]) for i in range(0, ROWS, 8)]
    lines.append("  { \\")
    lines.append(", \\\n".join(body) + " \\")
    lines.append("  }")
    lines.append("#define EEGFX_T6_TABLE \\")
    body = ["    " + ", ".join(float.hex(v) for v in row) for row in toom6_rows()]
    lines.append("  { \\")
    lines.append(", \\\n".join(body) + " \\")
    lines.append("  }")
    lines += ["", "}  // namespace dev", "}  // namespace eegfx", ""]
    return "\n".join(lines)


def main():
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dwt8_taps.h")
    with open(path, "w") as f:
        f.write(header_text())


if __name__ == "__main__":
    main()
