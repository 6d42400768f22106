"""configs[2]-size marker planning: 64M markers, device scan vs the sequential host planner."""
import ctypes
import time

import numpy as np
import torch

import eeg_dataanalysispackage_amd as fx
from eeg_dataanalysispackage_amd import _lib

n = 64_000_000
rng = np.random.default_rng(0)
pos = (1000 + 1000 * np.arange(n)).astype(np.int64)
stim = rng.integers(0, 2, size=n).astype(np.int32)
nf = 1000 * n + 2000
ctx = fx.Context(0)
dpos, dstim = torch.from_numpy(pos).cuda(), torch.from_numpy(stim).cuda()
ctx.plan_markers(dpos, dstim, nf, 1)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(5):
    p, l, b = ctx.plan_markers(dpos, dstim, nf, 1)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / 5
print(f"device scan: {dt*1e3:.2f} ms for {n} markers ({n/dt:.3e} markers/s), selected {len(p)}")
# the sequential C planner (eegfx_plan_markers) on 4M marker structs
m = 4_000_000
arr = (_lib.Marker * m)()
for i in range(m):
    arr[i].position = int(pos[i]); arr[i].stimulus_index = int(stim[i])
po = np.empty(m, dtype=np.int64); lo = np.empty(m); bal = ctypes.c_int64(0); cnt = ctypes.c_int64()
t = time.perf_counter()
_lib.check(fx.lib().eegfx_plan_markers(arr, m, nf, 1, ctypes.byref(bal), ctypes.c_void_p(po.ctypes.data),
                                       ctypes.c_void_p(lo.ctypes.data), ctypes.byref(cnt)))
ht = time.perf_counter() - t
print(f"host sequential C planner: {ht*1e3:.2f} ms for {m} markers ({m/ht:.3e} markers/s)")
