"""Host-to-device copy rate by copy size, alone and beside a device-to-host copy (configs[4]'s
chunked uploads run at ~48 GB/s, the bound leg's single 346 MB copy at ~57 GB/s)."""
import ctypes
import time

import torch

dev = torch.device("cuda:0")
hip = ctypes.CDLL("libamdhip64.so")
TOT = 345_600_000
h_in = torch.empty(TOT, dtype=torch.uint8, pin_memory=True)
d_in = torch.empty(TOT, dtype=torch.uint8, device=dev)
h_out = torch.empty(221_180_544, dtype=torch.uint8, pin_memory=True)
d_out = torch.empty(221_180_544, dtype=torch.uint8, device=dev)
up, down = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def cp(dst, src, n, kind, st):
    assert hip.hipMemcpyAsync(ctypes.c_void_p(dst), ctypes.c_void_p(src), ctypes.c_size_t(n),
                              ctypes.c_int(kind), ctypes.c_void_p(st.cuda_stream)) == 0


def run(chunk, with_down):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if with_down:
        cp(h_out.data_ptr(), d_out.data_ptr(), h_out.numel(), 2, down)
    off = 0
    while off < TOT:
        n = min(chunk, TOT - off)
        cp(d_in.data_ptr() + off, h_in.data_ptr() + off, n, 1, up)
        off += n
    up.synchronize()
    t_up = time.perf_counter() - t0
    down.synchronize()
    return TOT / t_up / 1e9


for chunk in (12_582_912, 25_165_824, 50_331_648, 100_663_296, TOT):
    for wd in (False, True):
        r = [run(chunk, wd) for _ in range(4)][1:]
        print(f"chunk {chunk / 1e6:7.1f} MB {'with D2H' if wd else 'alone   '}: "
              f"{max(r):5.1f} GB/s (median {sorted(r)[1]:5.1f})")
