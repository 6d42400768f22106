"""configs[4]'s host-link bound leg (bench.py bench_stream: two plain concurrent copies of the same
bytes) under variants, to see what its 6.07 ms per pair measures: the row buffer as bench.py
passes it (a numpy view of a pinned tensor) or as a pinned tensor, 5 pairs queued or 1 pair, and
the download's rate when each direction runs alone."""
import time

import numpy as np
import torch

dev = torch.device("cuda:0")
nf, n = 4 * 4 * 3600 * 1000, 576_000 - 9
host = torch.empty((nf, 3), dtype=torch.int16, pin_memory=True)
flat = host.view(-1)
out_np = torch.empty((n, 48), dtype=torch.float64, pin_memory=True).numpy()
h_np = torch.from_numpy(out_np)
h_pin = torch.empty((n, 48), dtype=torch.float64, pin_memory=True)
d_in = torch.empty(nf * 3, dtype=torch.int16, device=dev)
d_out = torch.empty((n, 48), dtype=torch.float64, device=dev)
s_in, s_out = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
print("numpy view is_pinned:", h_np.is_pinned(), " tensor is_pinned:", h_pin.is_pinned())


def run(label, reps, up=True, down=True, h_out=h_np, order="ud"):
    def pair():
        for c in order:
            if c == "u" and up:
                with torch.cuda.stream(s_in):
                    d_in.copy_(flat, non_blocking=True)
            if c == "d" and down:
                with torch.cuda.stream(s_out):
                    h_out.copy_(d_out, non_blocking=True)
    pair()
    torch.cuda.synchronize(dev)
    res = []
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(reps):
            pair()
        t_issue = time.perf_counter() - t0
        torch.cuda.synchronize(dev)
        res.append(((time.perf_counter() - t0) / reps * 1e3, t_issue / reps * 1e3))
    ms, iss = sorted(res)[1]
    print(f"{label:44s} {ms:7.3f} ms per pair (host issue {iss:7.3f} ms)")


def chunked(label, up_chunk, down_chunk, down_delay_chunks=0):
    """both directions as chunked copies queued at once (downloads optionally behind the first
    `down_delay_chunks` uploads, as the pipeline's rows follow their chunk's kernels)"""
    fu, fd = flat.view(torch.uint8), h_pin.view(-1).view(torch.uint8)
    du, dd = d_in.view(torch.uint8), d_out.view(-1).view(torch.uint8)
    ev = [torch.cuda.Event() for _ in range(64)]

    def go():
        k = 0
        for off in range(0, fu.numel(), up_chunk):
            with torch.cuda.stream(s_in):
                du[off:off + up_chunk].copy_(fu[off:off + up_chunk], non_blocking=True)
                ev[k].record(s_in)
            k += 1
        for i, off in enumerate(range(0, fd.numel(), down_chunk)):
            with torch.cuda.stream(s_out):
                if down_delay_chunks:
                    s_out.wait_event(ev[min(i + down_delay_chunks, k - 1)])
                fd[off:off + down_chunk].copy_(dd[off:off + down_chunk], non_blocking=True)
    go()
    torch.cuda.synchronize(dev)
    res = []
    for _ in range(3):
        t0 = time.perf_counter()
        go()
        torch.cuda.synchronize(dev)
        res.append((time.perf_counter() - t0) * 1e3)
    print(f"{label:44s} {sorted(res)[1]:7.3f} ms")


run("bench leg: numpy view, 5 pairs", 5)
run("pinned tensor, 5 pairs", 5, h_out=h_pin)
run("numpy view, 1 pair", 1)
run("pinned tensor, 1 pair", 1, h_out=h_pin)
run("pinned tensor, download issued first, 1 pair", 1, h_out=h_pin, order="du")
run("upload alone", 1, down=False)
run("download alone (numpy view)", 1, up=False)
run("download alone (pinned tensor)", 1, up=False, h_out=h_pin)
chunked("chunked 48 MB up / 30 MB down, at once", 48 << 20, 30 << 20)
chunked("chunked, each download behind its upload", 48 << 20, 30 << 20, 1)
chunked("chunked, each download two uploads behind", 48 << 20, 30 << 20, 2)
