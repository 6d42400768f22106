#!/usr/bin/env python3
"""Times eegfx_extract_features_f64 on device-resident epochs (the batched
WaveletTransform.extractFeatures over double[n][C][750], features_from_epochs_kernel).

  python3 tools/epochs_bench.py [--lib path/to/libeegfx.so] [--epochs N] [--steps K]

The epochs are cut from a synthetic recording on the device (eegfx_cut_epochs_f64), so the timed
region holds only the extraction.  Prints one JSON line per numerics mode: epochs/s, the kernel's
GB/s over its algorithmic bytes (C x 512 window doubles in + C x 16 features out per epoch), and a
hash of the EXACT features (equal across library builds when they agree value for value) plus the
largest |fma - exact| difference."""
import argparse
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None, help="libeegfx.so to load (default: the package's)")
    ap.add_argument("--epochs", type=int, default=1_000_000)
    ap.add_argument("--channels", type=int, default=3)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--tag", default="")
    ap.add_argument("--cut", action="store_true", help="also time eegfx_cut_epochs_f64")
    ap.add_argument("--onepass", action="store_true",
                    help="also time eegfx_process_recording_epochs (epochs + features in one pass) "
                         "against the cut alone and the two passes (cut, then extract)")
    args = ap.parse_args()
    import torch

    import eeg_dataanalysispackage_amd as fx
    from eeg_dataanalysispackage_amd import _lib
    if args.lib:
        _lib.LIB_PATH = os.path.abspath(args.lib)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n, C = args.epochs, args.channels
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx = fx.Context(0, numerics="exact")
    ctx.set_stream(stream.cuda_stream)
    raw = torch.empty((1000 * n + 2000, C), dtype=torch.int16, device=dev)
    ctx.synth_recording(raw, C, 7)
    pos = torch.arange(1000, 1000 * (n + 1), 1000, dtype=torch.int64, device=dev)
    ep = ctx.cut_epochs(raw, C, list(range(C)), [0.1] * C, pos)
    if args.cut:  # getData(): the materialised epochs themselves (a3 + a5..a7)
        for _ in range(args.warmup):
            ctx.cut_epochs(raw, C, list(range(C)), [0.1] * C, pos, out=ep)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.steps):
            ctx.cut_epochs(raw, C, list(range(C)), [0.1] * C, pos, out=ep)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / args.steps
        bpe = 850 * C * 2 + 8 + 750 * C * 8  # frames read (as the reference cuts them) + rows out
        f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        f0.record(stream)
        for _ in range(args.steps):
            ep.fill_(0.5)  # the write-bandwidth reference: the same rows, written only
        f1.record(stream)
        torch.cuda.synchronize(dev)
        fill_ms = f0.elapsed_time(f1) / args.steps
        ctx.cut_epochs(raw, C, list(range(C)), [0.1] * C, pos, out=ep)
        torch.cuda.synchronize(dev)
        print(json.dumps({"tool": "epochs_bench", "tag": args.tag, "op": "cut_epochs",
                          "fill_ms": round(fill_ms, 4),
                          "fill_GBps": round(ep.numel() * 8 / (fill_ms * 1e-3) / 1e9, 1),
                          "epochs": n, "channels": C, "ms_per_call": round(ms, 4),
                          "epochs_per_s": round(n / (ms * 1e-3), 1),
                          "GBps_algorithmic": round(n * bpe / (ms * 1e-3) / 1e9, 1),
                          "sha256_16": hashlib.sha256(ep.cpu().numpy().tobytes()).hexdigest()[:16]}),
              flush=True)
    if args.onepass:
        cols, res = list(range(C)), [0.1] * C
        feats = torch.empty((n, 16 * C), dtype=torch.float64, device=dev)

        def timed(fn):
            for _ in range(args.warmup):
                fn()
            torch.cuda.synchronize(dev)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for _ in range(args.steps):
                fn()
            b.record(stream)
            torch.cuda.synchronize(dev)
            return a.elapsed_time(b) / args.steps

        ctx.set_numerics("exact")
        cut_ms = timed(lambda: ctx.cut_epochs(raw, C, cols, res, pos, out=ep))
        ep_hash = hashlib.sha256(ep.cpu().numpy().tobytes()).hexdigest()[:16]
        for numerics in ("fma", "exact"):
            ctx.set_numerics(numerics)
            two_ms = timed(lambda: (ctx.cut_epochs(raw, C, cols, res, pos, out=ep),
                                    ctx.extract_features(ep, out=feats)))
            f_two = feats.clone()
            one_ms = timed(lambda: ctx.process_recording_epochs(raw, C, cols, res, pos, out=feats,
                                                                epochs_out=ep))
            ctx.synchronize()
            print(json.dumps({
                "tool": "epochs_bench", "tag": args.tag, "op": "epochs+features",
                "numerics": numerics, "epochs": n, "channels": C,
                "cut_only_ms": round(cut_ms, 4), "two_pass_ms": round(two_ms, 4),
                "one_pass_ms": round(one_ms, 4),
                "one_pass_over_cut": round(one_ms / cut_ms, 4),
                "one_pass_over_two_pass": round(one_ms / two_ms, 4),
                "epochs_equal_cut": hashlib.sha256(ep.cpu().numpy().tobytes()).hexdigest()[:16]
                == ep_hash,
                "features_max_abs_vs_two_pass": float((feats - f_two).abs().max())}), flush=True)
        ctx.set_numerics("exact")
    del raw
    out = torch.empty((n, 16 * C), dtype=torch.float64, device=dev)
    results = {}
    for numerics in ("fma", "exact"):
        ctx.set_numerics(numerics)
        for _ in range(args.warmup):
            ctx.extract_features(ep, out=out)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(args.steps):
            ctx.extract_features(ep, out=out)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        ms = e0.elapsed_time(e1) / args.steps
        results[numerics] = out.clone()
        bpe = C * 512 * 8 + C * 16 * 8
        maps = open("/proc/self/maps").read().split()
        loaded = sorted({os.path.basename(m) for m in maps if "libeegfx" in m})
        line = {"tool": "epochs_bench", "tag": args.tag, "lib_loaded": loaded,
                "numerics": numerics, "epochs": n, "channels": C, "ms_per_call": round(ms, 4),
                "epochs_per_s": round(n / (ms * 1e-3), 1),
                "wall_epochs_per_s": round(n * args.steps / wall, 1),
                "GBps_algorithmic": round(n * bpe / (ms * 1e-3) / 1e9, 1)}
        if numerics == "exact":
            line["exact_sha256_16"] = hashlib.sha256(
                results["exact"].cpu().numpy().tobytes()).hexdigest()[:16]
            line["max_abs_fma_minus_exact"] = float(
                (results["fma"] - results["exact"]).abs().max())
        print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
