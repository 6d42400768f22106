"""Boundary robustness on the GPU: device-resident marker positions the reference would not cut,
buffer dtypes, stream ordering with torch, concurrent contexts, and the small-batch (per-epoch)
IFeatureExtraction path.

References: OffLineDataProvider.java:220-225,262-264 (copyOfRange's AIOOBE for pos-100 outside
[0, len]: the epoch is not cut), include/eegfx.h threading rules (one context per Spark executor
thread, LogisticRegressionClassifier.java:50,90), FeatureExtractionTest.java:62-67 (one
extractFeatures call per epoch)."""
import threading

import numpy as np
import pytest
import torch

import eeg_dataanalysispackage_amd as fx
from eeg_dataanalysispackage_amd import classification as clf
from oracle import oracle

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def ctx():
    c = fx.Context(0)
    yield c
    c.close()


def synth_raw(rng, n_frames, ct):
    walk = np.cumsum(rng.integers(-40, 41, size=(n_frames, ct)), axis=0)
    return np.clip(-25000 + walk + rng.integers(-300, 300, size=(n_frames, ct)), -32768,
                   32767).astype(np.int16)


def eq(a, b):
    return np.array_equal(a, b, equal_nan=True)


# ---- device-resident positions are validated ----------------------------------------------------
BAD = [99, 0, -1, -(10 ** 15), 10 ** 15, 2 ** 62, -(2 ** 63), 2 ** 63 - 1]


@pytest.mark.parametrize("ct,cols", [(3, [0, 1, 2]), (32, list(range(32))), (5, [4, 0, 2])])
def test_invalid_device_positions_raise_at_synchronize(ctx, ct, cols):
    """Any position with pos-100 outside [0, n_frames] -- including values whose byte offsets
    would overflow -- is reported as ERANGE (IndexError) by the next synchronize, the kernels
    never touch memory outside the recording, and the valid epochs of the same call are exact."""
    rng = np.random.default_rng(ct)
    nf = 40_000
    raw = synth_raw(rng, nf, ct)
    good = rng.integers(100, nf - 900, size=40).astype(np.int64)
    for bad in BAD + [nf + 101]:
        pos = good.copy()
        pos[17] = bad
        d_raw = torch.from_numpy(raw).to(DEV)
        d_pos = torch.from_numpy(pos).to(DEV)
        out = ctx.process_recording(d_raw, ct, cols, [0.1] * len(cols), d_pos)
        with pytest.raises(IndexError):
            ctx.synchronize()
        ctx.synchronize()  # the flag was cleared
        got = out.cpu().numpy()
        keep = np.arange(len(pos)) != 17
        want = oracle.process_recording(raw, cols, [0.1] * len(cols), good[keep])
        assert eq(got[keep], want), bad
    # the boundary values the reference does cut are accepted
    for edge in (100, nf + 100):
        d_pos = torch.tensor([edge], dtype=torch.int64, device=DEV)
        out = ctx.process_recording(torch.from_numpy(raw).to(DEV), ct, cols, [0.1] * len(cols),
                                    d_pos)
        ctx.synchronize()
        assert eq(out.cpu().numpy(), oracle.process_recording(raw, cols, [0.1] * len(cols), [edge]))


def test_invalid_device_position_surfaces_at_next_synchronising_call(ctx):
    """A caller that never calls synchronize() still sees the refused position: the next API call
    that synchronises the context (here a host-memory call) raises IndexError (ERANGE), clears
    the flag, and the call after it is exact again."""
    rng = np.random.default_rng(8)
    nf = 30_000
    raw = synth_raw(rng, nf, 3)
    good = rng.integers(100, nf - 900, size=20).astype(np.int64)
    bad = good.copy()
    bad[3] = 42
    ctx.process_recording(torch.from_numpy(raw).to(DEV), 3, [0, 1, 2], [0.1] * 3,
                          torch.from_numpy(bad).to(DEV))
    with pytest.raises(IndexError) as e:
        ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, good)
    assert e.value.code == -6
    got = ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, good)
    assert eq(got, oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, good))
    ctx.synchronize()


def test_invalid_device_positions_in_cut_epochs(ctx):
    rng = np.random.default_rng(5)
    raw = synth_raw(rng, 20_000, 3)
    pos = np.array([500, 50, 1200, 10 ** 14], dtype=np.int64)
    ep = ctx.cut_epochs(torch.from_numpy(raw).to(DEV), 3, [0, 1, 2], [0.1] * 3,
                        torch.from_numpy(pos).to(DEV))
    with pytest.raises(IndexError):
        ctx.synchronize()
    want = oracle.decode_epochs(raw, [0, 1, 2], [0.1] * 3, pos[[0, 2]])
    assert eq(ep.cpu().numpy()[[0, 2]], want)


# ---- dtypes of device buffers -------------------------------------------------------------------
def test_wrong_dtype_device_tensors_are_refused(ctx):
    raw = torch.zeros((10_000, 3), dtype=torch.int16, device=DEV)
    pos32 = torch.tensor([500, 600], dtype=torch.int32, device=DEV)
    with pytest.raises(ValueError):
        ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos32)
    pos = pos32.to(torch.int64)
    with pytest.raises(ValueError):
        ctx.process_recording(raw.to(torch.int32), 3, [0, 1, 2], [0.1] * 3, pos)
    with pytest.raises(ValueError):
        ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos,
                              out=torch.empty((2, 48), dtype=torch.float32, device=DEV))
    with pytest.raises(ValueError):
        ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos,
                              out=torch.empty((3, 48), dtype=torch.float64, device=DEV))
    with pytest.raises(ValueError):
        ctx.extract_features(torch.zeros((2, 3, 750), dtype=torch.float32, device=DEV))
    with pytest.raises(ValueError):
        ctx.process_recording(raw[:, :2], 2, [0, 1], [0.1] * 2, pos)  # non-contiguous
    X = torch.zeros((10, 48), dtype=torch.float32, device=DEV)
    y = torch.zeros(10, dtype=torch.float64, device=DEV)
    with pytest.raises(ValueError):
        clf.sgd_train(ctx, X, y, 2)


# ---- ordering with torch's stream, no manual synchronisation ----------------------------------
def test_device_calls_order_with_torch_stream():
    """Inputs produced by torch kernels still in flight, outputs consumed by torch right after the
    call, and a fresh context (own non-blocking stream): no torch.cuda.synchronize() and no
    ctx.synchronize() anywhere."""
    ctx = fx.Context(0)
    rng = np.random.default_rng(11)
    nf, n = 400_000, 300
    raw_h = synth_raw(rng, nf, 3)
    pos_h = np.sort(rng.integers(100, nf - 800, size=n)).astype(np.int64)
    want = oracle.process_recording(raw_h, [0, 1, 2], [0.1] * 3, pos_h)
    for it in range(4):
        big = torch.randn((4096, 4096), device=DEV)  # keep torch's stream busy
        for _ in range(3):
            big = big @ big
            big = big / big.abs().max()
        raw32 = torch.from_numpy(raw_h.astype(np.int32)).to(DEV) + big[:1, :1].round().to(torch.int32) * 0
        raw = raw32.to(torch.int16)  # produced by a kernel queued behind the matmuls
        pos = torch.from_numpy(pos_h).to(DEV) + 0
        out = ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos)
        got = (out * 1.0).cpu().numpy()  # consumed by torch right away
        del raw, raw32, pos, out
        assert eq(got, want), it
    ctx.close()


# ---- concurrent contexts (Spark local[*]: one context per executor thread) --------------------
def test_two_contexts_two_threads():
    rng = np.random.default_rng(21)
    jobs = []
    for t in range(2):
        nf = 150_000 + 50_000 * t
        raw = synth_raw(rng, nf, 3)
        pos = rng.integers(100, nf - 800, size=2000).astype(np.int64)
        jobs.append((raw, pos, oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos),
                     oracle.decode_epochs(raw, [0, 1, 2], [0.1] * 3, pos[:200])))
    errors = []

    def worker(t):
        try:
            c = fx.Context(0)
            raw, pos, want, ep = jobs[t]
            wf = oracle.extract_features(ep)
            for it in range(6):
                k = 200 * (it + 1)  # growing batches: every buffer grows while the other thread runs
                got = c.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos[:k] if it < 5 else pos)
                assert eq(got, want[:len(got)]), (t, it)
                f = c.extract_features(ep[: 40 * (it + 1)])
                assert eq(f, wf[: 40 * (it + 1)]), (t, it)
            c.close()
        except Exception as e:  # noqa: BLE001 - reported in the main thread
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not any(x.is_alive() for x in th)
    assert not errors, errors


# ---- the per-epoch drop-in (IFeatureExtraction called once per epoch) ---------------------------
def test_small_batches_zero_copy_path(ctx):
    """extractFeatures on host epochs for every batch size around the zero-copy threshold
    (768 KB of window rows = 64 epochs of 3 channels), one epoch at a time included."""
    rng = np.random.default_rng(3)
    raw = synth_raw(rng, 200_000, 3)
    pos = rng.integers(100, 199_000, size=80).astype(np.int64)
    ep = oracle.decode_epochs(raw, [0, 1, 2], [0.1] * 3, pos)
    want = oracle.extract_features(ep)
    for n in (1, 2, 11, 63, 64, 65, 80):
        assert eq(ctx.extract_features(ep[:n]), want[:n]), n
    for i in range(10):  # one call per epoch, as the Spark map closure makes them
        assert eq(ctx.extract_features(ep[i:i + 1]), want[i:i + 1]), i
    fe = fx.WaveletTransform(context=ctx)
    assert eq(fe.extractFeatures(ep[0]), want[0])


@pytest.mark.parametrize("C", [3, 5, 9, 16])
def test_small_batches_every_channel_count_both_numerics(C):
    """The zero-copy small-batch kernel (features_small_kernel) for channel counts that use one
    wave (C <= 8) and two waves (C = 9..16), under EXACT (value-exact) and FMA numerics (its
    dwt8_cascade<true, true> partial-sum halos; <= 1e-9 per normalised feature)."""
    rng = np.random.default_rng(100 + C)
    raw = synth_raw(rng, 60_000, C)
    cols = list(range(C))
    pos = rng.integers(100, 59_000, size=9).astype(np.int64)
    ep = oracle.decode_epochs(raw, cols, [0.1] * C, pos)
    want = oracle.extract_features(ep)
    for numerics in ("exact", "fma"):
        c = fx.Context(0, numerics=numerics)
        try:
            for n in (1, 2, 9):
                got = c.extract_features(ep[:n])
                if numerics == "exact":
                    assert eq(got, want[:n]), (C, n)
                else:
                    assert np.max(np.abs(got - want[:n])) <= 1e-9, (C, n)
        finally:
            c.close()
