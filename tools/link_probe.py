#!/usr/bin/env python3
"""Host-link probe for the configs[4] streamed path: pinned host -> device copy
rates for the bench's 346 MB recording moved whole, in chunks on one stream, in chunks alternating
over two streams, and with every chunk split over two streams; each with and without the
221 MB of feature rows going device -> host at the same time.

  python3 tools/link_probe.py [--reps 5]
"""
import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    nbytes = 4 * 4 * 3600 * 1000 * 6          # bench_stream's recording
    dbytes = 576_000 * 48 * 8                 # its feature rows
    host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    host.fill_(1)
    d_in = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d_out = torch.empty(dbytes, dtype=torch.uint8, device=dev)
    h_out = torch.empty(dbytes, dtype=torch.uint8, pin_memory=True)
    ss = [torch.cuda.Stream(dev) for _ in range(3)]

    def run(chunk, mode, down):
        if down:
            with torch.cuda.stream(ss[2]):
                h_out.copy_(d_out, non_blocking=True)
        k = 0
        for o in range(0, nbytes, chunk):
            e = min(nbytes, o + chunk)
            if mode == "split":
                m = (o + e) // 2
                with torch.cuda.stream(ss[0]):
                    d_in[o:m].copy_(host[o:m], non_blocking=True)
                with torch.cuda.stream(ss[1]):
                    d_in[m:e].copy_(host[m:e], non_blocking=True)
            else:
                s = ss[k % 2] if mode == "alt" else ss[0]
                with torch.cuda.stream(s):
                    d_in[o:e].copy_(host[o:e], non_blocking=True)
            k += 1

    out = []
    for down in (False, True):
        for chunk, mode in ((nbytes, "one"), (12 << 20, "one"), (48 << 20, "one"),
                            (96 << 20, "one"), (48 << 20, "alt"), (48 << 20, "split"),
                            (nbytes, "split")):
            run(chunk, mode, down)
            torch.cuda.synchronize(dev)
            t = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                run(chunk, mode, down)
                torch.cuda.synchronize(dev)
                t.append(time.perf_counter() - t0)
            ms = sorted(t)[len(t) // 2] * 1e3
            r = {"chunk_MB": round(chunk / 2**20, 1), "mode": mode, "with_d2h": down,
                 "ms": round(ms, 3), "h2d_GBps": round(nbytes / ms / 1e6, 2)}
            out.append(r)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
