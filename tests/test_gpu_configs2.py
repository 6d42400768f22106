"""configs[2] on one GPU: the 8M-epoch shard one rank of the 64M-epoch / 8 x MI355X job runs.

BASELINE.json configs[2] ("Synthetic 64M epochs from multiplexed int16 BrainVision recordings,
epoch-sharded over 8xMI355X") gives every rank 8,000,000 epochs (eegfx_shard_range of 64M over 8)
of its own recording: 8,000,000 markers 1,000 frames apart, 8.0e9 frames x 3 channels of int16
= 48 GB generated on the device (synth_kernel), resident in HBM.  The fused path runs over the
whole shard; parity with the oracle is exact (EXACT numerics) on a spread sample of epochs, and
the size-independent properties are checked on every row: unit L2 norm (SignalProcessing.
normalize), finiteness, determinism (two launches, identical bytes) and the fma numerics within
1e-9 of the exact rows.  Row order is the shard's getData() order (OffLineDataProvider.java:
370-372): row i belongs to marker i."""
import numpy as np
import pytest
import torch

import eeg_dataanalysispackage_amd as fx
from eeg_dataanalysispackage_amd.sharding import shard_range
from oracle import oracle

pytestmark = pytest.mark.gpu
TOTAL = 64_000_000
WORLD = 8
SPACING = 1000
SEED = 0x5EED


def test_configs2_rank_shard_8m_epochs():
    s, e = shard_range(TOTAL, 3, WORLD)
    n = e - s
    assert n == 8_000_000
    dev = torch.device("cuda", 0)
    nf = SPACING * n + 2000
    ctx = fx.Context(0)
    try:
        raw = torch.empty((nf, 3), dtype=torch.int16, device=dev)  # 48 GB
        ctx.synth_recording(raw, 3, SEED + 3)
        pos = torch.arange(SPACING, SPACING * (n + 1), SPACING, dtype=torch.int64, device=dev)
        out = torch.empty((n, 48), dtype=torch.float64, device=dev)
        ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos, out=out)
        ctx.synchronize()
        norms = torch.linalg.vector_norm(out, dim=1)
        assert bool(torch.all(torch.isfinite(out)))
        assert float(torch.max(torch.abs(norms - 1.0))) < 1e-12
        # exact parity on a spread sample: the oracle on a host copy of the frames epoch i reads
        idx = np.unique(np.concatenate([np.arange(0, n, 4001), [1, n - 2, n - 1]]))
        starts = torch.as_tensor(SPACING + SPACING * idx - 100, device=dev)
        frames = starts[:, None] + torch.arange(850, device=dev)[None, :]
        windows = raw[frames].cpu().numpy()  # [k][850][3]
        got = out[torch.as_tensor(idx, device=dev)].cpu().numpy()
        for j, i in enumerate(idx):
            want = oracle.process_recording(np.ascontiguousarray(windows[j]), [0, 1, 2],
                                            [0.1] * 3, [100])
            assert np.array_equal(got[j:j + 1], want, equal_nan=True), i
        # determinism
        out2 = torch.empty_like(out)
        ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos, out=out2)
        ctx.synchronize()
        assert torch.equal(out, out2)
        # fma numerics over the whole shard: within the north_star's 1e-9
        ctx.set_numerics("fma")
        ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos, out=out2)
        ctx.synchronize()
        assert float(torch.max(torch.abs(out2 - out))) <= 1e-9
    finally:
        ctx.close()
