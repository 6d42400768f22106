#!/usr/bin/env python3
"""Regenerates tools/probes/ablations/*.patch against the current product sources.

Each ablation is a list of exact text replacements in fused.hip / wide.hip / dwt8.h.  When the
product changes, rerun this script; a replacement whose text no longer exists fails loudly.
build_probes.sh applies the patches to copies of the sources and builds window_probe_<name>;
tools/ablation_study.sh measures them.

  python3 tools/probes/make_ablations.py
"""
import difflib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "..", "eeg_dataanalysispackage_amd", "csrc")
FILES = ("fused.hip", "wide.hip", "dwt8.h")

DMA_ISSUE = """    if (dma_issue<CT, C, NT>(raw, nbytes, wb, e0, ne, win, w, lane, rows))
      dma_fixup<CT, C>(raw, nbytes, wb, e0, ne, win, w, lane, rows);"""

FMA_BODY = """#pragma unroll
  for (int q = 0; q < 3; ++q) {
    A0[q] = n == 0 ? x1 * R[q] : __builtin_fma(x1, R[q], A0[q]);
    if (n + 32 * (3 * q + 2) < 280)
      Ai[q] = n == 0 ? x0 * R[3 + q] : __builtin_fma(x0, R[3 + q], Ai[q]);
    Bp[q] = n == 0 ? xp * R[6 + q] : __builtin_fma(xp, R[6 + q], Bp[q]);
    Bm[q] = n == 0 ? xm * R[9 + q] : __builtin_fma(xm, R[9 + q], Bm[q]);
  }"""

BASELINE_T32 = [
    ("fused.hip", "  const dim3 g((unsigned)((n + 63) / 64));",
     "  const dim3 g((unsigned)((n + 31) / 32));  // ablation: 32-epoch tiles"),
    ("fused.hip", """    hipLaunchKernelGGL((dev::baseline_kernel<3, 3, 64, true>), g, dim3(192), 0, st,""",
     """    hipLaunchKernelGGL((dev::baseline_kernel<3, 3, 32, true>), g, dim3(128), 0, st,"""),
    ("fused.hip", """    hipLaunchKernelGGL((dev::baseline_kernel<3, 3, 64>), g, dim3(192), 0, st, (const uint8_t*)raw,""",
     """    hipLaunchKernelGGL((dev::baseline_kernel<3, 3, 32>), g, dim3(128), 0, st, (const uint8_t*)raw,"""),
]

ABLATIONS = {
    "baseline32": (
        "baseline_kernel on 32-epoch tiles (the reference point of baseline128: same LDS "
        "occupancy class)",
        BASELINE_T32),
    "baseline128": (
        "baseline_kernel staging whole 128-byte lines: each epoch's quads start at floor128 of its "
        "600-byte run and cover only the lines the run touches (VERDICT r03 item 5), 32-epoch tiles",
        BASELINE_T32 + [
            ("fused.hip",
             "  static constexpr int BASEQ = (kPre * FB + 15) / 16 + 1;    // 39 quads (600 B + misalignment)",
             "  static constexpr int BASEQ = (kPre * FB + 127) / 128 * 8 + 8;  // ablation: whole lines"),
            ("fused.hip",
             "    A[k] = want[k] ? (tB[e] & ~(int64_t)15) + 16 * q : 0;",
             "    want[k] = want[k] && 16 * q < (int)(((tB[e] & 127) + kPre * G::FB + 127) & ~127);\n"
             "    A[k] = want[k] ? (tB[e] & ~(int64_t)127) + 16 * q : 0;"),
            ("fused.hip",
             "  const int16_t* src = (const int16_t*)((const uint8_t*)(stage + e * G::BSTR) + (tB[e] & 15)) +",
             "  const int16_t* src = (const int16_t*)((const uint8_t*)(stage + e * G::BSTR) + (tB[e] & 127)) +"),
        ]),
    "noguard": (
        "the fma conditioning guard compiled out of the window kernels (no per-signal X^2, no "
        "per-row check, no rare path): A/B of its cost (round 4)",
        [("dwt8.h", "#define EEGFX_GUARD 1", "#define EEGFX_GUARD 0")]),
    "cascade": (
        "fma filter bank as the round-2 level-by-level cascade with partial-sum halos "
        "(A/B against the collapsed filter)",
        [("dwt8.h", "#define EEGFX_COLLAPSED 1", "#define EEGFX_COLLAPSED 0")]),
    "direct": (
        "each pair's update in the direct form (18 multiply-adds) instead of the four-point Toom "
        "form (12 + two adds): A/B of the change",
        [("dwt8.h", "#define EEGFX_TOOM 1", "#define EEGFX_TOOM 0")]),
    "nodma": (
        "no window DMA: removes the HBM window reads and the LDS writes; LDS reads, decode and "
        "fp64 kept (wrong results)",
        [("fused.hip", DMA_ISSUE,
          "    (void)rows;  // ablation: no window DMA (no HBM window reads, no LDS writes)")]),
    "l2src": (
        "window DMA from a 2 MB L2-resident region (same addresses mod 2 MB): removes HBM reads "
        "only (wrong results)",
        [("fused.hip", "    const uint8_t* sb = raw + Bq;",
          "    const uint8_t* sb = raw + (Bq & 0x1FFFF0);  // ablation: L2-resident source")]),
    "regdirect": (
        "no LDS staging: each lane loads its 64 samples (128 B, L2-resident region) into VGPRs; "
        "no window DMA, no LDS sample reads (wrong results)",
        [("fused.hip", DMA_ISSUE,
          "    (void)rows;  // ablation: no LDS staging; the lane's 64 samples come from VGPRs"),
         ("fused.hip", """    cascade_lds<CT, FAST, TRACKABLE>(own, nxt, r, b, lane & ~7, s, a6, d6, &ymax);""",
          """    (void)own; (void)nxt;
    u32x4_a4 q[8];
    {
      const int64_t wv = mine ? wb[e0 + el] : 0;
      const u32x4_a16* src = (const u32x4_a16*)(raw + ((wv + 384 * s + 128 * w) & 0x1FFFF0));
#pragma unroll
      for (int i = 0; i < 8; ++i) q[i] = src[i];
    }
    dwt8_collapsed_cascade([&](int k) {
      const uint32_t v = q[k >> 3][(k >> 1) & 3];
      return (float)(int16_t)((k & 1) ? (v >> 16) : (v & 0xffffu));
    }, r, b, lane & ~7, s, a6, d6);""")]),
    "noldsread": (
        "no LDS sample reads: each sample is an opaque per-lane float plus its index (one fp32 "
        "add in place of the int16 conversion); window DMA, decode and fp64 kept (wrong results)",
        [("fused.hip",
          "      dwt8_collapsed_cascade([&](int k) { return (float)own[k * CT]; }, r, b, gbase, s, a6, d6);",
          "      float q = (float)((int)(uintptr_t)own & 1023);  // ablation: no LDS sample reads\n"
          "      asm volatile(\"\" : \"+v\"(q));\n"
          "      dwt8_collapsed_cascade([&](int k) { return q + (float)k; }, r, b, gbase, s, a6, d6);")]),
    "nofp64": (
        "fp64 filter bank removed: the 440 multiply-adds and adds per lane become 64 fp64 adds; "
        "DMA, LDS reads and decode kept (wrong results)",
        [("dwt8.h", FMA_BODY, """  (void)R;  // ablation: no fp64 filter work, the decoded samples are summed
  if (n == 0) {
    for (int q = 0; q < 3; ++q) { A0[q] = x1; Ai[q] = x0; Bp[q] = xp; Bm[q] = xm; }
  } else { A0[n % 3] += x1; Ai[n % 3] += x0; }""")]),
}


def main():
    src = {f: open(os.path.join(CSRC, f)).read() for f in FILES}
    out_dir = os.path.join(HERE, "ablations")
    os.makedirs(out_dir, exist_ok=True)
    for old in os.listdir(out_dir):
        if old.endswith(".patch"):
            os.remove(os.path.join(out_dir, old))
    for name, (what, edits) in ABLATIONS.items():
        new = dict(src)
        for f, a, b in edits:
            if a not in new[f]:
                sys.exit(f"ablation {name}: text not found in {f}:\n{a}")
            new[f] = new[f].replace(a, b, 1)
        lines = [f"# ablation: {what}\n"]
        for f in FILES:
            if new[f] != src[f]:
                lines += difflib.unified_diff(src[f].splitlines(True), new[f].splitlines(True),
                                              f"a/{f}", f"b/{f}")
        with open(os.path.join(out_dir, name + ".patch"), "w") as fh:
            fh.writelines(lines)
        print(name)


if __name__ == "__main__":
    main()
