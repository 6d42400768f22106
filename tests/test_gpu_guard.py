"""The fma numerics on the reference's own data, and the conditioning guard.

north_star: "Output must match the reference Java DWT on the same inputs within 1e-9 relative in
fp64".  Under EEGFX_FMA every row is either certified by the guard (guard.h: its rounding
difference from the EXACT row is provably below 0.5e-9 after normalisation) or recomputed under
EXACT on the device.  These tests run the fma path

  * through the reference's own flows and recordings -- OffLineDataProvider(infoTrain.txt) and the
    DoD_2015_02 g=4 file (OfflineDataProviderTest.java:53-134, FeatureExtractionTest.java:70-112),
    process_recording on both recordings -- against the golden hex rows and the oracle, within
    1e-9, and the feature sum within 1e-9 * 528 of FeatureExtractionTest.java:106;
  * on windows in the filters' null space (Nyquist-alternating +-A, with and without DC, 1-3
    channels, several amplitudes and resolutions) and near it, where the fma rows are rounding
    noise: these rows must come back value-identical to the oracle (the EXACT recomputation),
    through every fma kernel family (3-channel fused, any-layout, 32-channel, float32, batch and
    per-epoch extract, streamed);
  * and check the guard's counters (eegfx_ctx_guard_stats).
"""
import numpy as np
import pytest

import eeg_dataanalysispackage_amd as fx
from conftest import DOD01, DOD02, FEATURE_SUM_GOLDEN, INFO_TRAIN, hexrows
from oracle import oracle

pytestmark = pytest.mark.gpu
TOL = 1e-9


@pytest.fixture(scope="module")
def ctx():
    c = fx.Context(0, numerics="fma")
    yield c
    c.close()


def within(a, b, tol=TOL):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and bool(np.all(np.abs(a - b) <= tol))


def eq(a, b):
    return np.array_equal(a, b, equal_nan=True)


# ---- the reference's flows and recordings under fma ----------------------------------------------
def test_info_train_flow_fma(ctx, golden_vectors):
    ctx.guard_stats(reset=True)
    odp = fx.OffLineDataProvider([INFO_TRAIN], context=ctx)
    odp.loadData()
    assert odp.last_error == ""
    feats = odp.getFeatures()
    g = golden_vectors["infoTrain"]
    assert feats.shape == (11, 48)
    assert within(feats, hexrows(g["features_hex"]))
    assert abs(oracle.java_feature_sum(feats) - FEATURE_SUM_GOLDEN) <= TOL * 528
    # IFeatureExtraction per epoch (the per-epoch drop-in kernel) and the device batch
    wt = fx.WaveletTransform(8, 512, 175, 16, context=ctx)
    ep = odp.getData()
    for i in range(len(ep)):
        assert within(wt.extractFeatures(ep[i]), feats[i])
    import torch
    dev = ctx.extract_features(torch.from_numpy(ep).cuda())
    ctx.synchronize()
    assert within(dev.cpu().numpy(), hexrows(g["features_hex"]))
    checked, redone = ctx.guard_stats()
    # every selected epoch certified (the per-epoch kernel computes EXACT rows: not counted)
    assert checked >= 11 + 11 and redone == 0


def test_dod_2015_02_g4_flow_fma(ctx, golden_vectors):
    odp = fx.OffLineDataProvider([DOD02 + ".eeg", "4"], context=ctx)
    odp.loadData()
    g = golden_vectors["DoD_2015_02_g4"]
    feats = odp.getFeatures()
    assert feats.shape == (27, 48)
    assert within(feats, hexrows(g["features_hex"]))
    assert abs(oracle.java_feature_sum(feats) - float.fromhex(g["feature_sum"])) <= TOL * 27 * 48


@pytest.mark.parametrize("base,guessed", [(DOD01, 1), (DOD02, 4)])
def test_process_recording_fma_on_recordings(ctx, base, guessed):
    raw = fx.read_raw(base + ".vhdr", base + ".eeg")
    pos, _, _ = fx.plan_markers(fx.read_markers(base + ".vmrk"), raw.shape[0], guessed)
    assert within(ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos),
                  oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos))
    # every marker with a window, the balanced selection's rejects included
    allpos = [m.position for m in fx.read_markers(base + ".vmrk") if m.position >= 100]
    ctx.guard_detail(reset=True)
    got = ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, allpos)
    want = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, allpos)
    assert within(got, want)
    checked, rechecked, redone = ctx.guard_detail()
    assert checked == len(allpos)
    print(f"{base.split('/')[-1]}: guard rechecked {rechecked}, recomputed {redone} of {checked}")
    assert redone == 0
    if base == DOD01:
        # the recording ends in a flat stretch (constant samples): those windows decode to one
        # fp32 rounding residue, far below the a-priori bound, so they go to the second stage,
        # whose measured max |x| certifies them (tests/test_guard_bound.py checks the ratio)
        flat = [i for i, p in enumerate(allpos) if np.ptp(raw[p + 175:p + 687], axis=0).max() == 0]
        assert flat and rechecked >= len(flat)
        assert within(got[flat], want[flat])


# ---- windows in (and near) the filters' null space ------------------------------------------------
def alternating(nf, ct, amp, dc, phase=0):
    t = np.arange(nf)[:, None]
    sign = np.where((t + phase) % 2 == 0, 1, -1)
    return np.clip(dc + amp * sign * np.ones((1, ct), dtype=np.int64), -32768, 32767).astype(np.int16)


NULL_CASES = [  # (amplitude, DC, resolution)
    (1, 0, 1.0), (100, 0, 1.0), (20000, 0, 1.0), (7, -25000, 1.0),
    (1, 0, 0.1), (300, -20000, 0.1), (32767, 0, 0.1), (5000, 1000, 0.5),
]


@pytest.mark.parametrize("amp,dc,res", NULL_CASES)
@pytest.mark.parametrize("C", [1, 2, 3])
def test_null_space_windows_equal_oracle(ctx, amp, dc, res, C):
    nf, n = 40 * 1000 + 2000, 40
    raw = alternating(nf, 3, amp, dc)
    pos = np.arange(1000, 1000 * (n + 1), 1000, dtype=np.int64) + np.arange(n) % 2  # both phases
    cols = list(range(C))
    want = oracle.process_recording(raw, cols, [res] * C, pos)
    ctx.guard_stats(reset=True)
    got = ctx.process_recording(raw, 3, cols, [res] * C, pos)
    assert eq(got, want)
    _, redone = ctx.guard_stats()
    assert redone == n


def test_dc_plus_alternating_and_near_null(ctx):
    """A DC offset in the window (not cancelled: the baseline comes from a different level) keeps
    the features far above rounding: certified, within 1e-9.  An alternating window with a single
    perturbed sample, or a tiny step, is near the null space: recomputed, value-identical."""
    nf, n = 30 * 1000 + 2000, 30
    raw = alternating(nf, 3, 500, -1000).astype(np.int64)
    pos = np.arange(1000, 1000 * (n + 1), 1000, dtype=np.int64)
    for k, p in enumerate(pos):
        if k % 3 == 0:
            raw[p:p + 750] += 40                       # DC step after the stimulus
        elif k % 3 == 1:
            raw[p + 175 + 17 * k % 512, k % 3] += 1    # one sample off the null space
    raw = raw.astype(np.int16)
    want = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos)
    got = ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos)
    assert within(got, want)
    near = [k for k in range(n) if k % 3 == 2]          # pure alternating windows
    assert eq(got[near], want[near])


def test_null_space_every_fma_kernel_family(ctx):
    """The guard in each fma kernel: any-layout (ct=5), the 32-channel montage, float32
    recordings (measured X), device batch extract (rows in LDS and, at C = 32, through the
    output), per-epoch host extract, streamed."""
    import torch
    n = 24
    pos = np.arange(1000, 1000 * (n + 1), 1000, dtype=np.int64) + np.arange(n) % 2
    for ct, cols in ((5, [4, 0, 2]), (32, list(range(32)))):
        raw = alternating(1000 * n + 2000, ct, 1234, -300)
        res = [0.1] * len(cols)
        want = oracle.process_recording(raw, cols, res, pos)
        assert eq(ctx.process_recording(raw, ct, cols, res, pos), want)
        assert eq(ctx.process_recording(torch.from_numpy(raw).cuda(), ct, cols, res,
                                         torch.from_numpy(pos).cuda()).cpu().numpy(), want)
    raw32 = alternating(1000 * n + 2000, 3, 250, 0).astype(np.float32) * np.float32(0.37)
    want = oracle.process_recording(raw32, [0, 1, 2], [1.0] * 3, pos)
    assert eq(ctx.process_recording(raw32, 3, [0, 1, 2], [1.0] * 3, pos), want)
    m = 100  # > 64 host epochs: the chunked-copy batch path; fewer: the per-epoch kernel
    posm = np.arange(1000, 1000 * (m + 1), 1000, dtype=np.int64) + np.arange(m) % 2
    raw = alternating(1000 * m + 2000, 3, 999, 0)
    ep = oracle.decode_epochs(raw, [0, 1, 2], [0.1] * 3, posm)
    want = oracle.extract_features(ep)
    assert eq(ctx.extract_features(torch.from_numpy(ep).cuda()).cpu().numpy(), want)
    assert eq(ctx.extract_features(ep), want)                # host batch (chunked copies)
    assert eq(ctx.extract_features(ep[:5]), want[:5])        # per-epoch drop-in kernel
    # wide rows (C = 32: the batch extract's rows go through `out`), flagged rows mixed with
    # ordinary ones in one tile
    wide = alternating(1000 * 20 + 2000, 32, 700, 0)
    ep32 = oracle.decode_epochs(wide, list(range(32)), [0.1] * 32, posm[:20])
    ep32[1::3] += np.random.default_rng(3).standard_normal((7, 32, 750))
    want32 = oracle.extract_features(ep32)
    ctx.guard_stats(reset=True)
    got32 = ctx.extract_features(torch.from_numpy(ep32).cuda()).cpu().numpy()
    flagged = [i for i in range(20) if i % 3 != 1]
    assert eq(got32[flagged], want32[flagged])
    assert np.max(np.abs(got32 - want32)) <= 1e-9
    assert ctx.guard_stats()[1] == len(flagged)
    wt = fx.WaveletTransform(8, 512, 175, 16, context=ctx)
    assert eq(wt.extractFeatures(ep[3]), want[3])
    want = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos)
    assert eq(ctx.process_recording_streamed(raw, 3, [0, 1, 2], [0.1] * 3, pos,
                                             chunk_frames=5000), want)


def test_guard_mixed_batch_and_counters(ctx):
    """Flagged rows scattered through a large ordinary batch: exactly those are recomputed (the
    counter matches), the others stay certified fma rows within 1e-9 of the oracle."""
    rng = np.random.default_rng(7)
    n, sp = 5000, 1000
    nf = sp * n + 2000
    t = np.arange(nf)[:, None]
    # a 3 Hz rhythm of 2,000 counts: features far above the guard's threshold
    raw = (-5000 + 2000 * np.sin(2 * np.pi * 3 * t / 1000 + np.arange(3)[None, :])
           + rng.integers(-300, 300, size=(nf, 3))).astype(np.int64)
    pos = np.arange(sp, sp * (n + 1), sp, dtype=np.int64)
    null = rng.choice(n, size=37, replace=False)
    alt = np.where(np.arange(-100, 750) % 2 == 0, 1, -1)[:, None] * 60 - 5000
    for k in null:
        raw[pos[k] - 100:pos[k] + 750] = alt
    raw = raw.astype(np.int16)
    want = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos)
    ctx.guard_stats(reset=True)
    got = ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos)
    assert within(got, want)
    assert eq(got[np.sort(null)], want[np.sort(null)])
    checked, redone = ctx.guard_stats(reset=True)
    assert (checked, redone) == (n, len(null))
    assert ctx.guard_stats() == (0, 0)


def flat_recording(n, sp, ct, flat_every, seed=11):
    """A 3 Hz rhythm on a DC level with every flat_every-th marker's span [pos-100, pos+750) held
    at the DC level (the flat stretch of DoD2015_01): the a-priori test fails those rows, the
    second stage certifies them."""
    rng = np.random.default_rng(seed)
    nf = sp * n + 2000
    t = np.arange(nf)[:, None]
    raw = (-25000 + 2000 * np.sin(2 * np.pi * 3 * t / 1000 + np.arange(ct)[None, :])
           + rng.integers(-300, 300, size=(nf, ct))).astype(np.int64)
    pos = np.arange(sp, sp * (n + 1), sp, dtype=np.int64)
    flat = np.arange(0, n, flat_every)
    for k in flat:
        raw[pos[k] - 100:pos[k] + 750] = raw[pos[k] - 100]
    return raw.astype(np.int16), pos, flat


def test_flat_windows_certified_by_second_stage_every_int16_kernel(ctx):
    """Flat windows through every int16 fma kernel: the 3-channel fused kernel (flat rows at every
    sub-tile slot, epoch 0's read back from the recording), the one-pass epochs + features, the
    any-layout and 32-channel kernels and the streamed path: all rechecked, none recomputed, every
    row within 1e-9 of the oracle."""
    import torch
    n = 67
    raw, pos, flat = flat_recording(n, 1000, 3, 3)
    want = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos)
    runs = {
        "fused": lambda: ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos),
        "fused_device": lambda: ctx.process_recording(
            torch.from_numpy(raw).cuda(), 3, [0, 1, 2], [0.1] * 3,
            torch.from_numpy(pos).cuda()).cpu().numpy(),
        "one_pass": lambda: ctx.process_recording_epochs(raw, 3, [0, 1, 2], [0.1] * 3, pos)[0],
        "streamed": lambda: ctx.process_recording_streamed(raw, 3, [0, 1, 2], [0.1] * 3, pos,
                                                           chunk_frames=7000),
    }
    for name, run in runs.items():
        ctx.guard_detail(reset=True)
        got = run()
        checked, rechecked, redone = ctx.guard_detail()
        assert within(got, want), name
        assert redone == 0 and rechecked >= len(flat), (name, rechecked, redone)
    for ct, cols in ((5, [4, 0, 2]), (32, list(range(32)))):
        raw, pos, flat = flat_recording(n, 1000, ct, 4)
        res = [0.1] * len(cols)
        want = oracle.process_recording(raw, cols, res, pos)
        ctx.guard_detail(reset=True)
        got = ctx.process_recording(raw, ct, cols, res, pos)
        checked, rechecked, redone = ctx.guard_detail()
        assert within(got, want), ct
        assert redone == 0 and rechecked >= len(flat), (ct, rechecked, redone)


def test_flat_window_past_the_recording_end_rechecked_from_the_recording(ctx):
    """A silent stretch (raw 0, so x = 0 after the baseline) running into the end of the recording:
    the last marker's window is zero-padded past the end (copyOfRange) and is the first epoch of
    its sub-tile, so its second stage reads the recording with the per-frame end test (the window
    kernel's rows lie over that epoch's staged window).  Certified, not recomputed; the row equals
    the oracle (0/0 -> NaN)."""
    n = 9
    raw, pos, _ = flat_recording(n, 1000, 3, n + 1)
    raw = raw[:pos[8] + 400].copy()
    raw[pos[8] - 100:] = 0
    want = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos)
    for name, run in (("fused", lambda: ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos)),
                      ("one_pass", lambda: ctx.process_recording_epochs(raw, 3, [0, 1, 2],
                                                                        [0.1] * 3, pos)[0])):
        ctx.guard_detail(reset=True)
        got = run()
        checked, rechecked, redone = ctx.guard_detail()
        assert np.isnan(want[8]).all() and np.isnan(got[8]).all(), name
        assert within(got[:8], want[:8]), name
        assert rechecked >= 1 and redone == 0, (name, rechecked, redone)


def test_flat_and_null_windows_mixed(ctx):
    """Flat windows (certified by the second stage) and null-space windows (recomputed) in one
    sub-tile: the counters separate them and the null rows equal the oracle value for value."""
    n = 40
    raw, pos, flat = flat_recording(n, 1000, 3, 2)
    raw = raw.astype(np.int64)
    null = np.arange(1, n, 4)
    alt = np.where(np.arange(-100, 750) % 2 == 0, 1, -1)[:, None] * 90 - 3000
    for k in null:
        raw[pos[k] - 100:pos[k] + 750] = alt
    raw = raw.astype(np.int16)
    want = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos)
    ctx.guard_detail(reset=True)
    got = ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos)
    checked, rechecked, redone = ctx.guard_detail()
    assert within(got, want)
    assert eq(got[null], want[null])
    assert redone == len(null) and rechecked == len(null) + len(flat)


def test_guard_strategies_agree():
    """The 3-channel window kernel's two second-stage strategies (fused.hip EEGFX_TRACK_X): a
    context's first launch scans the staged windows of the rows it flags; a launch after one that
    flagged more than 1/16 of its rows tracks max |x| while decoding instead.  Flat rows (certified)
    and null-space rows (recomputed) mixed: both launches give the same rows, counters and oracle
    values, and the strategy survives a counter reset."""
    c = fx.Context(0, numerics="fma")
    n = 48
    raw, pos, flat = flat_recording(n, 1000, 3, 2)
    raw = raw.astype(np.int64)
    null = np.arange(1, n, 4)
    alt = np.where(np.arange(-100, 750) % 2 == 0, 1, -1)[:, None] * 90 - 3000
    for k in null:
        raw[pos[k] - 100:pos[k] + 750] = alt
    raw = raw.astype(np.int16)
    want = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos)
    runs = []
    for _ in range(3):  # scan, then track (and track again after the reset)
        c.guard_detail(reset=True)
        got = c.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos)
        runs.append((got, c.guard_detail()))
    for got, (checked, rechecked, redone) in runs:
        assert within(got, want)
        assert eq(got[null], want[null])
        assert checked == n and redone == len(null) and rechecked == len(null) + len(flat)
    assert eq(runs[0][0], runs[1][0]) and eq(runs[1][0], runs[2][0])
    c.close()


def test_guard_strategies_agree_c32():
    """The same for the 32-channel kernel (wide.hip window_c32_kernel): its first launch tests the
    flagged rows against the staged window in one wave, later launches after a heavily flagged one
    use the X_c every lane tracked while decoding; same rows, counters and oracle values."""
    c = fx.Context(0, numerics="fma")
    n = 40
    raw, pos, flat = flat_recording(n, 1000, 32, 2)
    cols, res = list(range(32)), [0.1] * 32
    want = oracle.process_recording(raw, cols, res, pos)
    runs = []
    for _ in range(3):
        c.guard_detail(reset=True)
        got = c.process_recording(raw, 32, cols, res, pos)
        runs.append((got, c.guard_detail()))
    for got, (checked, rechecked, redone) in runs:
        assert within(got, want)
        assert checked == n and redone == 0 and rechecked >= len(flat)
    assert runs[0][1] == runs[1][1] == runs[2][1]
    assert eq(runs[0][0], runs[1][0]) and eq(runs[1][0], runs[2][0])
    c.close()


def test_exact_numerics_not_guarded():
    c = fx.Context(0)  # EXACT
    raw = alternating(12000, 3, 5, 0)
    pos = [1000, 2001, 3000]
    assert eq(c.process_recording(raw, 3, [0, 1, 2], [1.0] * 3, pos),
              oracle.process_recording(raw, [0, 1, 2], [1.0] * 3, pos))
    assert c.guard_stats() == (0, 0)
    c.close()
