"""Stability: 1M-epoch fused path repeated 200 times in both numerics; every output bit-identical
to the first (deterministic kernels, no atomics), and a sample checked against the oracle."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import eeg_dataanalysispackage_amd as fx  # noqa: E402
from oracle import oracle  # noqa: E402

n = 1_000_000
for numerics in ("fma", "exact"):
    ctx = fx.Context(0, numerics=numerics)
    raw = torch.empty((1000 * n + 2000, 3), dtype=torch.int16, device="cuda")
    ctx.synth_recording(raw, 3, 99)
    pos = torch.arange(1000, 1000 * (n + 1), 1000, dtype=torch.int64, device="cuda")
    first = ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos)
    ctx.synchronize()
    ref = first.clone()
    bad = 0
    for _ in range(200):
        out = ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos, out=first)
        ctx.synchronize()
        bad += int(not torch.equal(out, ref))
    k = 20000
    want = oracle.process_recording(raw[: 1000 * k + 2000].cpu().numpy(), [0, 1, 2], [0.1] * 3,
                                    np.arange(1000, 1000 * (k + 1), 1000))
    got = ref[:k].cpu().numpy()
    err = np.max(np.abs(got - want)) if numerics == "fma" else float(not np.array_equal(got, want))
    print(f"{numerics}: 200 repeats, {bad} differing; sample vs oracle max |diff| / mismatch = {err}")
    ctx.close()
    del raw
