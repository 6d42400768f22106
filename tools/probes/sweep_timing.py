#!/usr/bin/env python3
"""Where a parity-sweep case spends its time with a resident per-epoch server on another context:
times each call of tools/parity_sweep.py's case loop over a few cases, with the server on and off."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))


def main():
    import torch
    import eeg_dataanalysispackage_amd as fx
    from parity_sweep import case
    ex, fm = fx.Context(0, numerics="exact"), fx.Context(0, numerics="fma")
    mb = fx.Context(0)
    for server in (False, True, False):
        mb.set_mailbox(server)
        tot = {}
        for seed in range(400000, 400030):
            raw, ct, cols, res, pos, nfeat, skip = case(seed)
            if len(cols) > 16:
                continue
            ep = np.zeros((len(pos), len(cols), 750))
            steps = [
                ("to_device", lambda: (torch.from_numpy(raw).cuda(), torch.from_numpy(pos).cuda())),
                ("pr_exact_host", lambda: ex.process_recording(raw, ct, cols, res, pos)),
                ("pr_fma_host", lambda: fm.process_recording(raw, ct, cols, res, pos)),
                ("epochs_exact", lambda: ex.process_recording_epochs(raw, ct, cols, res, pos)),
                ("small_exact", lambda: ex.extract_features(ep[:4], feature_size=nfeat, skip=skip)),
                ("small_fma", lambda: fm.extract_features(ep[:1], feature_size=nfeat, skip=skip)),
                ("server", lambda: mb.extract_features(ep[-1:], feature_size=nfeat, skip=skip)),
                ("dev_extract", lambda: ex.extract_features(torch.from_numpy(ep).cuda(),
                                                            feature_size=nfeat,
                                                            skip=skip).cpu()),
            ]
            for name, fn in steps:
                t = time.perf_counter()
                fn()
                tot[name] = tot.get(name, 0.0) + time.perf_counter() - t
        print("server" if server else "no server",
              {k: round(v * 1e3, 1) for k, v in tot.items()}, "ms", flush=True)
    mb.set_mailbox(False)
    for c in (ex, fm, mb):
        c.close()


if __name__ == "__main__":
    main()
