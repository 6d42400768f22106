"""Host-link duplex: one 346 MB upload (or 50 MB chunks) and one 221 MB download on two streams,
issued in either order; prints when each direction finished (configs[4]'s uploads run at ~48 GB/s
beside row downloads, the bound leg's at ~57)."""
import ctypes
import time

import torch

dev = torch.device("cuda:0")
hip = ctypes.CDLL("libamdhip64.so")
UP, DOWN, CH = 345_600_000, 221_180_544, 50_331_648
h_in = torch.empty(UP, dtype=torch.uint8, pin_memory=True)
d_in = torch.empty(UP, dtype=torch.uint8, device=dev)
h_out = torch.empty(DOWN, dtype=torch.uint8, pin_memory=True)
d_out = torch.empty(DOWN, dtype=torch.uint8, device=dev)
su, sd = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
eu, ed, e0 = (torch.cuda.Event(enable_timing=True) for _ in range(3))


def cp(dst, src, n, kind, st):
    assert hip.hipMemcpyAsync(ctypes.c_void_p(dst), ctypes.c_void_p(src), ctypes.c_size_t(n),
                              ctypes.c_int(kind), ctypes.c_void_p(st.cuda_stream)) == 0


def up(chunk):
    off = 0
    while off < UP:
        n = min(chunk, UP - off)
        cp(d_in.data_ptr() + off, h_in.data_ptr() + off, n, 1, su)
        off += n
    eu.record(su)


def down():
    cp(h_out.data_ptr(), d_out.data_ptr(), DOWN, 2, sd)
    ed.record(sd)


for label, order, chunk in (("up first, one copy", "ud", UP), ("up first, 50 MB chunks", "ud", CH),
                            ("down first, one copy", "du", UP), ("up alone", "u", UP),
                            ("down alone", "d", UP)):
    res = []
    for _ in range(4):
        torch.cuda.synchronize()
        e0.record(torch.cuda.current_stream())
        su.wait_event(e0)
        sd.wait_event(e0)
        for c in order:
            up(chunk) if c == "u" else down()
        torch.cuda.synchronize()
        tu = e0.elapsed_time(eu) if "u" in order else 0.0
        td = e0.elapsed_time(ed) if "d" in order else 0.0
        res.append((tu, td))
    tu, td = sorted(res[1:])[1]
    print(f"{label:24s} up done {tu:6.3f} ms ({UP / tu / 1e6 if tu else 0:5.1f} GB/s)  "
          f"down done {td:6.3f} ms ({DOWN / td / 1e6 if td else 0:5.1f} GB/s)")
