"""Which engine serves a device-to-host copy into pinned memory (SDMA vs rocclr's blit kernel)?
Run under rocprofv3 --kernel-trace --memory-copy-trace: blit copies show up as
__amd_rocclr_copyBuffer kernels, SDMA copies as MEMORY_COPY_DEVICE_TO_HOST records."""
import ctypes
import time

import torch

dev = torch.device("cuda:0")
hip = ctypes.CDLL("libamdhip64.so")
n = 80_000 * 48  # one 8M-frame chunk's rows (doubles)
d = torch.empty(4 * n, dtype=torch.float64, device=dev)
h = torch.empty(4 * n, dtype=torch.float64, pin_memory=True)
s = torch.cuda.Stream(dev)
torch.cuda.synchronize()


def copy(dst, src, nbytes, stream):
    rc = hip.hipMemcpyAsync(ctypes.c_void_p(dst), ctypes.c_void_p(src), ctypes.c_size_t(nbytes),
                            ctypes.c_int(2), ctypes.c_void_p(stream))
    assert rc == 0, rc


for label, off, nbytes in (("aligned 30.7 MB", 0, n * 8), ("offset 384 B", 384, n * 8),
                           ("offset 3 rows", 3 * 384, n * 8 - 384), ("small 1 MB", 0, 1 << 20)):
    for _ in range(3):
        t0 = time.perf_counter()
        copy(h.data_ptr() + off, d.data_ptr() + off, nbytes, s.cuda_stream)
        s.synchronize()
        dt = time.perf_counter() - t0
    print(f"{label}: {nbytes / dt / 1e9:.1f} GB/s")
# torch's own copy of the same buffers
t0 = time.perf_counter()
with torch.cuda.stream(s):
    h.copy_(d, non_blocking=True)
s.synchronize()
print(f"torch copy_ {h.numel() * 8 / (time.perf_counter() - t0) / 1e9:.1f} GB/s")
