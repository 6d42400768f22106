#!/usr/bin/env python3
"""Long randomised parity sweep of every compute entry point against the oracle (the seeded
`tests/test_gpu_fuzz*.py` cases run 40 per file; this runs thousands, as round evidence).

Per case: a random recording (int16 / float32, 1-64 channels per frame, any selection and order of
1-64 channels, per-channel resolutions, random-walk or noise samples), a random marker set with the
legal edges (pos = 100, windows past the end, pos - 100 = n_frames), then
  * eegfx_process_recording (host and device buffers), both numerics,
  * eegfx_process_recording_epochs (epochs + features in one pass), both numerics,
  * eegfx_extract_features_f64 on the oracle's epochs with a random feature size and skip,
    on device epochs and (C <= 16) on host epochs through the per-epoch kernel: up to 4 epochs,
    one epoch under fma, one epoch served by a context's resident server (eegfx_ctx_set_mailbox),
  * every fifth case, eegfx_process_recording_streamed with a random chunk size (EXACT).
EXACT must equal the oracle value for value (epochs always); fma within 1e-9 per feature.

`--flat` overwrites the spans [pos-100, pos+750) of about a third of each case's markers with
held samples (flat, the value at pos-100) or zeros (silent): the rows the fma guard's first
stage flags and its second stage certifies (the guard counters are added to the summary).

  python tools/parity_sweep.py [--cases 2000] [--seed0 0] [--flat] [--out summary.json]
                               [--max-seconds S]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def case(seed, flat=False):
    rng = np.random.default_rng(50_000 + seed)
    ct = int(rng.choice([1, 2, 3, 3, 3, 4, 5, 7, 8, 16, 32, 32, 40, 63, 64]))
    C = int(rng.integers(1, ct + 1)) if seed % 4 else ct
    cols = [int(c) for c in rng.permutation(ct)[:C]]
    res = [float(np.float32(r)) for r in rng.choice([0.1, 0.5, 1.0, 0.0488281, 2.5, 0.01], size=C)]
    nf = int(rng.integers(800, 8000))
    if seed % 3 == 0:
        raw = (rng.standard_normal((nf, ct)) * rng.choice([1.0, 50.0, 3000.0])).astype(np.float32)
    else:
        base = rng.integers(-30000, 30000, size=(1, ct))
        raw = np.clip(base + np.cumsum(rng.integers(-60, 61, size=(nf, ct)), axis=0), -32768,
                      32767).astype(np.int16)
    n = int(rng.integers(1, 70))
    pos = rng.integers(100, nf + 101, size=n).astype(np.int64)
    pos[0] = 100
    if n > 1:
        pos[-1] = nf + 100
    nfeat = int(rng.integers(1, 17))
    skip = int(rng.integers(0, 750 - 512 + 1))
    if flat:  # a separate stream, so the unplanted cases stay those of earlier sweeps
        prng = np.random.default_rng(90_000 + seed)
        raw = raw.copy()
        for p in pos[prng.random(n) < 0.35]:
            lo, hi = max(0, int(p) - 100), min(nf, int(p) + 750)
            if lo < hi:
                raw[lo:hi] = raw[lo] if prng.integers(0, 2) else 0
    return raw, ct, cols, res, pos, nfeat, skip


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=2000)
    ap.add_argument("--seed0", type=int, default=0)
    ap.add_argument("--flat", action="store_true")
    ap.add_argument("--out", default=None)
    ap.add_argument("--max-seconds", type=float, default=0.0,
                    help="stop after this long (the summary counts the cases run)")
    a = ap.parse_args()
    import torch
    import eeg_dataanalysispackage_amd as fx
    from oracle import oracle
    ex, fm = fx.Context(0, numerics="exact"), fx.Context(0, numerics="fma")
    mb = fx.Context(0)  # host calls only: the per-epoch resident server
    mb.set_mailbox(True)
    fm.guard_detail(reset=True)
    stats = {"cases": 0, "epochs": 0, "checks": 0, "mismatches": [], "max_fma_err": 0.0,
             "by_channels": {}}
    t0 = time.time()
    last = t0

    def fma_ok(got, want):
        fin = np.isfinite(want)
        if not np.array_equal(np.isfinite(got), fin):
            return False, float("inf")
        err = float(np.max(np.abs(got[fin] - want[fin]), initial=0.0))
        return err <= 1e-9, err

    for seed in range(a.seed0, a.seed0 + a.cases):
        if a.max_seconds and time.time() - t0 > a.max_seconds:
            break
        raw, ct, cols, res, pos, nfeat, skip = case(seed, a.flat)
        want = oracle.process_recording(raw, cols, res, pos)
        want_ep = oracle.decode_epochs(raw, cols, res, pos)
        want_x = oracle.extract_features(want_ep, nfeat=nfeat, skip=skip)
        draw, dpos = torch.from_numpy(raw).cuda(), torch.from_numpy(pos).cuda()
        results = []
        results.append(("process_recording exact host",
                        np.array_equal(ex.process_recording(raw, ct, cols, res, pos), want,
                                       equal_nan=True), 0.0))
        got = ex.process_recording(draw, ct, cols, res, dpos)
        ex.synchronize()
        results.append(("process_recording exact device",
                        np.array_equal(got.cpu().numpy(), want, equal_nan=True), 0.0))
        ok, err = fma_ok(fm.process_recording(raw, ct, cols, res, pos), want)
        results.append(("process_recording fma host", ok, err))
        f, ep = ex.process_recording_epochs(raw, ct, cols, res, pos)
        results.append(("process_recording_epochs exact",
                        np.array_equal(f, want, equal_nan=True) and
                        np.array_equal(ep, want_ep, equal_nan=True), 0.0))
        f, ep = fm.process_recording_epochs(raw, ct, cols, res, pos)
        ok, err2 = fma_ok(f, want)
        results.append(("process_recording_epochs fma",
                        ok and np.array_equal(ep, want_ep, equal_nan=True), err2))
        if seed % 5 == 0:  # the streamed ingest (configs[4]) with a random chunk size
            cf = int(np.random.default_rng(seed).integers(787, max(788, raw.shape[0] + 1)))
            results.append(("process_recording_streamed exact",
                            np.array_equal(ex.process_recording_streamed(raw, ct, cols, res, pos,
                                                                         chunk_frames=cf),
                                           want, equal_nan=True), 0.0))
        dep = torch.from_numpy(want_ep).cuda()
        got = ex.extract_features(dep, feature_size=nfeat, skip=skip)
        results.append(("extract_features exact device",
                        np.array_equal(got.cpu().numpy(), want_x, equal_nan=True), 0.0))
        ok, err3 = fma_ok(fm.extract_features(dep, feature_size=nfeat, skip=skip).cpu().numpy(),
                          want_x)
        results.append(("extract_features fma device", ok, err3))
        if len(cols) <= 16:  # host epochs: the per-epoch kernel (features_small_kernel)
            k = min(len(pos), 4)
            results.append(("extract_features exact host small",
                            np.array_equal(ex.extract_features(want_ep[:k], feature_size=nfeat,
                                                               skip=skip),
                                           want_x[:k], equal_nan=True), 0.0))
            ok, err4 = fma_ok(fm.extract_features(want_ep[:1], feature_size=nfeat, skip=skip),
                              want_x[:1])
            results.append(("extract_features fma host single", ok, err4))
            results.append(("extract_features resident server",
                            np.array_equal(mb.extract_features(want_ep[-1:], feature_size=nfeat,
                                                               skip=skip),
                                           want_x[-1:], equal_nan=True), 0.0))
        stats["cases"] += 1
        stats["epochs"] += len(pos)
        key = str(len(cols))
        stats["by_channels"][key] = stats["by_channels"].get(key, 0) + 1
        for name, ok, err in results:
            stats["checks"] += 1
            stats["max_fma_err"] = max(stats["max_fma_err"], err)
            if not ok:
                stats["mismatches"].append({"seed": seed, "check": name, "ct": ct, "cols": cols,
                                            "fmt": str(raw.dtype), "err": err})
        if time.time() - last > 30:
            last = time.time()
            print(f"{stats['cases']} cases, {len(stats['mismatches'])} mismatches, "
                  f"{last - t0:.0f} s", flush=True)
    checked, rechecked, recomputed = fm.guard_detail()
    stats["guard"] = {"rows_checked": checked, "rows_rechecked": rechecked,
                      "rows_recomputed": recomputed, "flat": a.flat}
    ex.close()
    fm.close()
    mb.set_mailbox(False)
    mb.close()
    stats["seconds"] = round(time.time() - t0, 1)
    stats["mismatches"] = stats["mismatches"][:20]
    line = json.dumps(stats)
    print(line)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(line + "\n")
    return 1 if stats["mismatches"] else 0


if __name__ == "__main__":
    sys.exit(main())
