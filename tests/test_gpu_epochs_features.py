"""getData() and extractFeatures in one pass (eegfx_process_recording_epochs, SURVEY §8b's
`epochs_out`), and the provider built on it (OffLineDataProvider.loadData keeps the rows, so
getFeatures() is a copy).

Bar: epochs bit-identical to the oracle's decode (OffLineDataProvider.java:216-233) in every
numerics mode; features bit-identical to the oracle under EXACT and within 1e-9 under fma
(WaveletTransform.java:107-141); rows the fma guard cannot certify value-identical.  Layouts: the
3-channel packed frames, other packed and whole-dword int16 frames, float32, the 32-channel
montage, and wide files whose epoch span does not fit one workgroup (the two-pass fallback; the
staged cut's multi-chunk passes).
"""
import numpy as np
import pytest

import eeg_dataanalysispackage_amd as fx
from conftest import DOD01, DOD02, INFO_TRAIN, hexrows
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = fx.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def ctx_fma():
    c = fx.Context(0, numerics="fma")
    yield c
    c.close()


def eq(a, b):
    return np.array_equal(a, b, equal_nan=True)


def within(a, b, tol=1e-9):
    return a.shape == b.shape and bool(np.all(np.abs(a - b) <= tol))


def synth(rng, nf, ct, dtype=np.int16):
    walk = np.cumsum(rng.integers(-30, 31, size=(nf, ct)), axis=0) % 4000
    raw = -25000 + walk + rng.integers(-300, 300, size=(nf, ct))
    if dtype == np.float32:
        return (raw * 0.25).astype(np.float32)
    return np.clip(raw, -32768, 32767).astype(np.int16)


@pytest.mark.parametrize("base,guessed", [(DOD01, 1), (DOD02, 4)])
def test_recordings_one_pass(ctx, ctx_fma, base, guessed):
    raw = fx.read_raw(base + ".vhdr", base + ".eeg")
    allpos = [m.position for m in fx.read_markers(base + ".vmrk") if m.position >= 100]
    want_ep = oracle.decode_epochs(raw, [0, 1, 2], [0.1] * 3, allpos)
    want_f = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, allpos)
    f, ep = ctx.process_recording_epochs(raw, 3, [0, 1, 2], [0.1] * 3, allpos)
    assert eq(ep, want_ep) and eq(f, want_f)
    f, ep = ctx_fma.process_recording_epochs(raw, 3, [0, 1, 2], [0.1] * 3, allpos)
    assert eq(ep, want_ep) and within(f, want_f)


@pytest.mark.parametrize("numerics", ["exact", "fma"])
def test_unaligned_device_features_take_the_two_pass_route(ctx, ctx_fma, numerics):
    """A device `features` view offset by one double (8-byte aligned): the 3-channel one-pass
    kernel stores 16-byte row pairs, so such a pointer takes the cut + batch-extract route
     -- same rows, no misaligned vector stores."""
    import torch
    raw = fx.read_raw(DOD02 + ".vhdr", DOD02 + ".eeg")
    allpos = [m.position for m in fx.read_markers(DOD02 + ".vmrk") if m.position >= 100]
    n = len(allpos)
    c = ctx if numerics == "exact" else ctx_fma
    want_f = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, allpos)
    want_ep = oracle.decode_epochs(raw, [0, 1, 2], [0.1] * 3, allpos)
    buf = torch.full((n * 48 + 1,), float("nan"), dtype=torch.float64, device="cuda")
    feats = buf[1:].view(n, 48)
    assert feats.data_ptr() % 16 == 8
    ep = torch.empty((n, 3, 750), dtype=torch.float64, device="cuda")
    c.process_recording_epochs(torch.from_numpy(raw).cuda(), 3, [0, 1, 2], [0.1] * 3,
                               torch.from_numpy(np.asarray(allpos, dtype=np.int64)).cuda(),
                               out=feats, epochs_out=ep)
    c.synchronize()
    assert eq(ep.cpu().numpy(), want_ep)
    got = feats.cpu().numpy()
    assert eq(got, want_f) if numerics == "exact" else within(got, want_f)
    assert torch.isnan(buf[0])


LAYOUTS = [  # (ct, cols, fmt)
    (3, [0, 1, 2], np.int16),          # the reference's Fz/Cz/Pz file: 6-byte packed frames
    (5, [4, 1], np.int16),             # packed, 2 of 5 channels
    (4, [3, 0, 1, 2], np.int16),       # whole-dword frames
    (32, list(range(32)), np.int16),   # configs[3]'s montage: 64-byte frames
    (40, list(range(39, -1, -1)), np.int16),  # 40 signals: two passes of the 4 waves
    (3, [2, 0, 1], np.float32),        # IEEE_FLOAT_32
    (7, [6, 5, 4, 3, 2], np.float32),
]


@pytest.mark.parametrize("ct,cols,dtype", LAYOUTS)
@pytest.mark.parametrize("numerics", ["exact", "fma"])
def test_layouts_one_pass(ct, cols, dtype, numerics):
    c = fx.Context(0, numerics=numerics)
    rng = np.random.default_rng(ct * 7 + len(cols))
    n, sp = 37, 900
    nf = sp * n + 1200
    raw = synth(rng, nf, ct, dtype)
    pos = np.arange(200, 200 + sp * n, sp, dtype=np.int64)
    pos[-1] = nf - 300                     # the last epoch runs past the end: zero padding
    res = [0.1 + 0.05 * i for i in range(len(cols))]
    want_ep = oracle.decode_epochs(raw, cols, res, pos)
    want_f = oracle.process_recording(raw, cols, res, pos)
    f, ep = c.process_recording_epochs(raw, ct, cols, res, pos)
    assert eq(ep, want_ep)
    assert eq(f, want_f) if numerics == "exact" else within(f, want_f)
    # device buffers, and the same outputs as the separate calls
    import torch
    dr, dp = torch.from_numpy(raw).cuda(), torch.from_numpy(pos).cuda()
    fd, epd = c.process_recording_epochs(dr, ct, cols, res, dp)
    c.synchronize()
    assert eq(epd.cpu().numpy(), ep) and eq(fd.cpu().numpy(), f)
    assert eq(c.cut_epochs(raw, ct, cols, res, pos), ep)
    c.close()


WIDE = [  # epoch spans beyond one workgroup's LDS: the staged cut in chunks + the batch extract
    (63, [62, 0, 31, 5, 17, 40, 8, 55], np.int16),   # 126-byte packed frames, 2 chunks
    (60, list(range(0, 60, 6)), np.int16),           # 120-byte (124 staged) frames, 93 KB, 2 chunks
    (40, list(range(0, 40, 4)), np.float32),         # 160-byte frames
]


@pytest.mark.parametrize("ct,cols,dtype", WIDE)
def test_wide_files_two_pass(ctx, ctx_fma, ct, cols, dtype):
    rng = np.random.default_rng(ct)
    n, sp = 11, 800
    nf = sp * n + 1101                                 # odd frame count
    raw = synth(rng, nf, ct, dtype)
    pos = np.arange(150, 150 + sp * n, sp, dtype=np.int64)
    pos[-1] = nf - 5
    res = [0.1] * len(cols)
    want_ep = oracle.decode_epochs(raw, cols, res, pos)
    want_f = oracle.process_recording(raw, cols, res, pos)
    assert eq(ctx.cut_epochs(raw, ct, cols, res, pos), want_ep)
    f, ep = ctx.process_recording_epochs(raw, ct, cols, res, pos)
    assert eq(ep, want_ep) and eq(f, want_f)
    f, ep = ctx_fma.process_recording_epochs(raw, ct, cols, res, pos)
    assert eq(ep, want_ep) and within(f, want_f)


def test_null_space_rows_one_pass(ctx_fma):
    """The fma guard in the one-pass kernels: Nyquist-alternating windows come back EXACT."""
    n = 20
    t = np.arange(1000 * n + 2000)[:, None]
    for ct, cols, dt in ((3, [0, 1, 2], np.int16), (4, [0, 1, 2, 3], np.int16),
                         (3, [0, 1, 2], np.float32)):
        raw = (np.where(t % 2 == 0, 1, -1) * 700 * np.ones((1, ct))).astype(dt)
        pos = np.arange(1000, 1000 * (n + 1), 1000) + np.arange(n) % 2
        res = [0.1] * len(cols)
        ctx_fma.guard_stats(reset=True)
        f, ep = ctx_fma.process_recording_epochs(raw, ct, cols, res, pos)
        assert eq(ep, oracle.decode_epochs(raw, cols, res, pos))
        assert eq(f, oracle.process_recording(raw, cols, res, pos))
        assert ctx_fma.guard_stats()[1] == n


def test_provider_keeps_rows_from_load(ctx, ctx_fma, golden_vectors):
    for c in (ctx, ctx_fma):
        odp = fx.OffLineDataProvider([INFO_TRAIN], context=c)
        odp.loadData()
        feats = odp.getFeatures()
        g = hexrows(golden_vectors["infoTrain"]["features_hex"])
        assert eq(feats, g) if c is ctx else within(feats, g)
        # other parameters recompute from the resident epochs
        f12 = odp.getFeatures(feature_size=12)
        assert eq(f12, oracle.extract_features(odp.getData(), nfeat=12)) if c is ctx else \
            within(f12, oracle.extract_features(odp.getData(), nfeat=12))
    # numerics switched after loadData: recomputed under the current numerics
    odp = fx.OffLineDataProvider([DOD02 + ".eeg", "4"], context=ctx_fma)
    odp.loadData()
    ctx_fma.set_numerics("exact")
    try:
        assert eq(odp.getFeatures(), hexrows(golden_vectors["DoD_2015_02_g4"]["features_hex"]))
    finally:
        ctx_fma.set_numerics("fma")
