"""Quick parity check of the fused path under the current EEGFX_FUSED_IMPL (perf experiments)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import eeg_dataanalysispackage_amd as fx  # noqa: E402
from oracle import oracle  # noqa: E402

rng = np.random.default_rng(5)
n = 1000
nf = 1100 * n + 2000
raw = np.clip(rng.integers(-26000, -24000, size=(1, 3)) +
              np.cumsum(rng.integers(-40, 41, size=(nf, 3)), axis=0), -32768, 32767).astype(np.int16)
pos = np.sort(rng.integers(100, nf + 100, size=n))
for numerics in ("exact", "fma"):
    ctx = fx.Context(0, numerics=numerics)
    got = ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos)
    want = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos)
    if numerics == "exact":
        ok = np.array_equal(got, want, equal_nan=True)
    else:
        ok = np.nanmax(np.abs(got - want)) <= 1e-9
    print(os.environ.get("EEGFX_FUSED_IMPL", "default"), numerics, "parity", "OK" if ok else "FAIL")
    ctx.close()
    if not ok:
        sys.exit(1)
