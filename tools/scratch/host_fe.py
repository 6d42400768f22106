"""IFeatureExtraction drop-in with host (JVM-side) epochs: eegfx_extract_features_f64 on a numpy
double[n][3][750] (pageable) and on a pinned buffer; epochs/s including the host link."""
import time

import numpy as np
import torch

import eeg_dataanalysispackage_amd as fx

n = 100_000
ctx = fx.Context(0, numerics="fma")
raw = torch.empty((1000 * n + 2000, 3), dtype=torch.int16, device="cuda")
ctx.synth_recording(raw, 3, 7)
pos = torch.arange(1000, 1000 * (n + 1), 1000, dtype=torch.int64, device="cuda")
ep_dev = ctx.cut_epochs(raw, 3, [0, 1, 2], [0.1] * 3, pos)
ctx.synchronize()
ep = ep_dev.cpu().numpy()
pinned = torch.empty(ep.shape, dtype=torch.float64, pin_memory=True)
pinned.copy_(torch.from_numpy(ep))
out = np.empty((n, 48))
ref = ctx.extract_features(ep_dev).cpu().numpy()
for name, src in (("pageable", ep), ("pinned", pinned.numpy())):
    ctx.extract_features(src, out=out)
    t = time.perf_counter()
    for _ in range(5):
        ctx.extract_features(src, out=out)
    dt = (time.perf_counter() - t) / 5
    print(f"{name}: {n/dt:.3e} epochs/s ({dt*1e3:.1f} ms per {n}), equal={np.array_equal(out, ref)}")
