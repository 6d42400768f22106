"""Times the two-step getData() path on the device: cut_epochs (materialised double[n][3][750]) and
extract_features on those epochs, 200k epochs, against their algorithmic bytes."""
import time

import torch

import eeg_dataanalysispackage_amd as fx

n = 200_000
ctx = fx.Context(0, numerics="fma")
raw = torch.empty((1000 * n + 2000, 3), dtype=torch.int16, device="cuda")
ctx.synth_recording(raw, 3, 7)
pos = torch.arange(1000, 1000 * (n + 1), 1000, dtype=torch.int64, device="cuda")
ep = torch.empty((n, 3, 750), dtype=torch.float64, device="cuda")
out = torch.empty((n, 48), dtype=torch.float64, device="cuda")
for _ in range(20):
    ctx.cut_epochs(raw, 3, [0, 1, 2], [0.1] * 3, pos, out=ep)
    ctx.extract_features(ep, out=out)
ctx.synchronize()
R = 50
t = time.perf_counter()
for _ in range(R):
    ctx.cut_epochs(raw, 3, [0, 1, 2], [0.1] * 3, pos, out=ep)
ctx.synchronize()
tc = (time.perf_counter() - t) / R
t = time.perf_counter()
for _ in range(R):
    ctx.extract_features(ep, out=out)
ctx.synchronize()
te = (time.perf_counter() - t) / R
bc = n * (850 * 6 + 8 + 18000)
be = n * (18000 + 384)
print(f"cut_epochs {tc*1e3:.3f} ms  {bc/tc/1e12:.2f} TB/s   extract_features {te*1e3:.3f} ms  "
      f"{be/te/1e12:.2f} TB/s  ({n/te:.3e} epochs/s)")
