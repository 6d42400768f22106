"""configs[2]'s 8M-epoch rank shard in one process_recording call against the same shard as k
calls over consecutive position slices (each a baseline pass + a window pass).  The 1M-epoch step
runs ~5 % faster per epoch than the 8M one (profiles/r04z: 0.757 vs 0.795 ms per 1M in the window
kernel): this times whether slicing recovers it.
  python tools/chunk_probe.py [--epochs 8000000] [--reps 10] [--rounds 2]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=8_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--slices", default="1,2,4,8,16")
    ap.add_argument("--numerics", default="fma")
    a = ap.parse_args()
    import torch
    import eeg_dataanalysispackage_amd as fx
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = fx.Context(0, numerics=a.numerics)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    n, sp, ct = a.epochs, 1000, 3
    raw = torch.empty((sp * n + 2000, ct), dtype=torch.int16, device=dev)
    ctx.synth_recording(raw, ct, 1234)
    pos = torch.arange(sp, sp * (n + 1), sp, dtype=torch.int64, device=dev)
    out = torch.empty((n, 48), dtype=torch.float64, device=dev)
    ref = torch.empty_like(out)
    cols, res = [0, 1, 2], [0.1] * 3

    def step(k):
        b = [n * i // k for i in range(k + 1)]
        for i in range(k):
            ctx.process_recording(raw, ct, cols, res, pos[b[i]:b[i + 1]], out=out[b[i]:b[i + 1]])

    step(1)
    torch.cuda.synchronize()
    ref.copy_(out)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:  # settle (power-cap clock transient)
        step(1)
        torch.cuda.synchronize()
    res_ms = {}
    for r in range(a.rounds):
        for k in [int(x) for x in a.slices.split(",")]:
            step(k)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.reps):
                step(k)
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            same = bool(torch.equal(out, ref))
            res_ms.setdefault(k, []).append(round(ms, 4))
            print(f"round {r} slices {k:2d}: {ms:.4f} ms per {n} epochs "
                  f"({ms * 1e6 / n:.4f} ms per 1M), rows identical {same}", flush=True)
    print(json.dumps({"epochs": n, "numerics": a.numerics, "ms": res_ms}))
    ctx.close()


if __name__ == "__main__":
    main()
