#!/usr/bin/env python3
"""Other contexts' work beside a resident per-epoch server (eegfx_ctx_set_mailbox), for one build
of the library: streamed calls (pinned staging reused) and an 11-epoch host batch on a second
context, timed with the server resident and without; prints one JSON line (medians, ms).
  python tools/probes/server_stall.py [path/to/libeegfx.so]"""
import json
import os
import statistics
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    from eeg_dataanalysispackage_amd import _lib
    if len(sys.argv) > 1:
        _lib.LIB_PATH = os.path.abspath(sys.argv[1])
    import eeg_dataanalysispackage_amd as fx
    rng = np.random.default_rng(1)
    nf = 40_000
    raw = np.clip(-25000 + np.cumsum(rng.integers(-40, 41, size=(nf, 3)), axis=0), -32768,
                  32767).astype(np.int16)
    pos = np.arange(1000, nf - 1000, 997, dtype=np.int64)
    ep = rng.standard_normal((11, 3, 750))
    server, work = fx.Context(0), fx.Context(0)
    out = {"lib": _lib.LIB_PATH}
    try:
        for resident in (False, True):
            server.set_mailbox(resident)
            server.extract_features(ep[:1])
            st, b11, one = [], [], []
            for _ in range(20):
                t = time.perf_counter()
                work.process_recording_streamed(raw, 3, [0, 1, 2], [0.1] * 3, pos,
                                                chunk_frames=5000)
                st.append(time.perf_counter() - t)
                t = time.perf_counter()
                work.extract_features(ep)
                b11.append(time.perf_counter() - t)
                t = time.perf_counter()
                server.extract_features(ep[:1])
                one.append(time.perf_counter() - t)
            key = "resident" if resident else "launched"
            out[key] = {"streamed_ms": round(statistics.median(st) * 1e3, 3),
                        "streamed_max_ms": round(max(st) * 1e3, 3),
                        "batch11_ms": round(statistics.median(b11) * 1e3, 4),
                        "batch11_max_ms": round(max(b11) * 1e3, 3),
                        "server_epoch_ms": round(statistics.median(one) * 1e3, 4)}
    finally:
        server.set_mailbox(False)
        server.close()
        work.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
