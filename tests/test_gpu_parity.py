"""GPU parity: libeegfx kernels (through the C ABI) against the CPU oracle and the reference goldens.

Bar (BASELINE.json north_star):
  * marker offsets, labels, epoch counts: bit-exact;
  * EXACT numerics: epochs and features equal to the oracle value for value (np.array_equal with
    NaN == NaN; the only representable difference is the sign of an exactly-zero coefficient);
  * FMA numerics: |gpu - oracle| <= 1e-9 per feature; each feature row has unit L2 norm, so this
    is 1e-9 relative to the feature vector (the north_star tolerance).
"""
import os

import numpy as np
import pytest

import eeg_dataanalysispackage_amd as fx
from conftest import (DOD01, DOD02, EPOCH_SUM_GOLDEN, FEATURE_SUM_GOLDEN, INFO_TRAIN, DATA,
                      hexrows)
from oracle import oracle

pytestmark = pytest.mark.gpu
FMA_TOL = 1e-9


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


def synth_raw(rng, n_frames, ct, lo=-32768, hi=32767):
    base = rng.integers(-26000, -24000, size=(1, ct))
    walk = np.cumsum(rng.integers(-40, 41, size=(n_frames, ct)), axis=0)
    raw = np.clip(base + walk + rng.integers(-300, 300, size=(n_frames, ct)), lo, hi)
    return raw.astype(np.int16)


# ---- reference goldens through the GPU path ---------------------------------------------------
def test_offline_data_provider_info_txt(ctx, epochs_csv, golden_vectors):
    odp = fx.OffLineDataProvider([INFO_TRAIN], context=ctx)
    odp.loadData()
    assert odp.last_error == ""
    ep = odp.getData()
    assert ep.shape == (11, 3, 750)                           # OfflineDataProviderTest :65-67
    assert oracle.java_epoch_sum(ep) == EPOCH_SUM_GOLDEN      # :81
    assert int(sum(odp.getDataLabels())) == 5                 # :88
    for i, row in enumerate(epochs_csv):                      # Epochs.csv, per value
        assert np.array_equal(ep[i, 2], np.array(row))
    oep, olab, opos, _ = oracle.data_provider([INFO_TRAIN])
    assert np.array_equal(ep, oep)
    pos, fid = odp.getPositions()
    assert list(pos) == opos == golden_vectors["infoTrain"]["positions"]


def test_feature_extraction_golden(ctx, golden_vectors):
    odp = fx.OffLineDataProvider([INFO_TRAIN], context=ctx)
    odp.loadData()
    feats = odp.getFeatures()
    assert feats.shape == (11, 48)                               # FeatureExtractionTest :88-90
    assert oracle.java_feature_sum(feats) == FEATURE_SUM_GOLDEN  # :106, exact ==
    assert eq(feats, hexrows(golden_vectors["infoTrain"]["features_hex"]))
    # per-epoch IFeatureExtraction.extractFeatures, as the Spark map closure calls it
    wt = fx.WaveletTransform(8, 512, 175, 16, context=ctx)
    assert wt.getFeatureDimension() == 48
    ep = odp.getData()
    for i in range(len(ep)):
        assert eq(wt.extractFeatures(ep[i]), feats[i])


def test_loading_file_dod_2015_02(ctx, golden_vectors):
    odp = fx.OffLineDataProvider([DOD02 + ".eeg", "4"], context=ctx)
    odp.loadData()
    ep = odp.getData()
    assert ep.shape == (27, 3, 750)
    assert int(sum(odp.getDataLabels())) == 13
    g = golden_vectors["DoD_2015_02_g4"]
    assert oracle.java_epoch_sum(ep) == float.fromhex(g["epoch_sum"])
    assert eq(odp.getFeatures(), hexrows(g["features_hex"]))


@pytest.mark.parametrize("base,guessed", [(DOD01, 1), (DOD02, 4)])
def test_fused_path_on_recordings(ctx, base, guessed):
    raw = fx.read_raw(base + ".vhdr", base + ".eeg")
    pos, lab, _ = fx.plan_markers(fx.read_markers(base + ".vmrk"), raw.shape[0], guessed)
    got = ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos)
    want = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos)
    assert eq(got, want)
    # every marker that has a full window, not only the balanced selection
    allpos = [m.position for m in fx.read_markers(base + ".vmrk") if m.position >= 100]
    assert eq(ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, allpos),
              oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, allpos))


# ---- synthetic recordings: sizes, tails, padding, layouts ----------------------------------------
@pytest.mark.parametrize("n", [1, 7, 8, 9, 63, 64, 65, 130, 1000])
def test_fused_exact_ragged_tiles(ctx, n):
    rng = np.random.default_rng(n)
    nf = 1100 * n + 2000
    raw = synth_raw(rng, nf, 3)
    pos = np.sort(rng.integers(100, nf + 100, size=n))  # includes zero-padded tails past the end
    pos[-1] = nf + 100                                  # pos-100 == n_frames: all-zero epoch
    got = ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos)
    want = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos)
    assert eq(got, want)
    assert np.all(np.isnan(got[-1]))
    two = ctx.extract_features(ctx.cut_epochs(raw, 3, [0, 1, 2], [0.1] * 3, pos))
    assert eq(two, want)


def test_cut_epochs_exact(ctx):
    rng = np.random.default_rng(3)
    raw = synth_raw(rng, 40000, 3)
    pos = rng.integers(100, 40100, size=300)
    assert eq(ctx.cut_epochs(raw, 3, [2, 0, 1], [0.1, 0.25, 0.5], pos),
              oracle.decode_epochs(raw, [2, 0, 1], [0.1, 0.25, 0.5], pos))


def test_extract_features_host_chunks(ctx):
    """Host epochs (the IFeatureExtraction drop-in) go through window-only pinned staging in
    8,192-epoch chunks: equal to the device-resident path and to the oracle."""
    import torch
    rng = np.random.default_rng(17)
    n = 20001
    raw = synth_raw(rng, 1000 * n + 2000, 3)
    pos = np.arange(1000, 1000 * (n + 1), 1000)
    dep = ctx.cut_epochs(torch.from_numpy(raw).cuda(), 3, [0, 1, 2], [0.1] * 3,
                         torch.from_numpy(pos).cuda())
    ctx.synchronize()
    host = dep.cpu().numpy()
    got = ctx.extract_features(host)
    dev = ctx.extract_features(dep)
    ctx.synchronize()
    assert eq(got, dev.cpu().numpy())
    sel = np.r_[0:50, 8180:8200, n - 30:n]
    assert eq(got[sel], oracle.extract_features(host[sel]))
    for nf, sk in ((5, 175), (16, 238)):
        assert eq(ctx.extract_features(host[:9000], feature_size=nf, skip=sk),
                  oracle.extract_features(host[:9000], nfeat=nf, skip=sk))


def test_cut_epochs_device_paths(ctx):
    """Device-resident cut: the two-pass kernels (staged baselines + 16-byte row writes) and the
    single-kernel fallback taken for an output that is only 8-byte aligned."""
    import torch
    rng = np.random.default_rng(13)
    raw = synth_raw(rng, 30000, 3)
    pos = np.concatenate([[100], rng.integers(100, 30100, size=60), [30100]])
    want = oracle.decode_epochs(raw, [0, 1, 2], [0.1] * 3, pos)
    draw, dpos = torch.from_numpy(raw).cuda(), torch.from_numpy(pos).cuda()
    got = ctx.cut_epochs(draw, 3, [0, 1, 2], [0.1] * 3, dpos)
    ctx.synchronize()
    assert eq(got.cpu().numpy(), want)
    flat = torch.empty(len(pos) * 3 * 750 + 1, dtype=torch.float64, device="cuda")
    odd = flat[1:].view(len(pos), 3, 750)          # 8-byte aligned only
    ctx.cut_epochs(draw, 3, [0, 1, 2], [0.1] * 3, dpos, out=odd)
    ctx.synchronize()
    assert eq(odd.cpu().numpy(), want)
    raw5 = synth_raw(rng, 20000, 5)                # generic layout: baseline_any + write pass
    pos5 = rng.integers(100, 20100, size=40)
    assert eq(ctx.cut_epochs(raw5, 5, [4, 1], [0.1, 0.3], pos5),
              oracle.decode_epochs(raw5, [4, 1], [0.1, 0.3], pos5))


def test_saturated_and_odd_positions(ctx):
    rng = np.random.default_rng(5)
    raw = synth_raw(rng, 20000, 3)
    raw[rng.integers(0, 20000, size=300), rng.integers(0, 3, size=300)] = -32768
    raw[rng.integers(0, 20000, size=300), rng.integers(0, 3, size=300)] = 32767
    pos = np.arange(101, 19000, 977)  # odd and even frame offsets -> both 4-byte alignments
    assert eq(ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos),
              oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos))


@pytest.mark.parametrize("ct,cols", [(5, [4, 0, 2]), (32, [16, 17, 18]), (1, [0]), (2, [1, 0])])
def test_generic_layouts_exact(ctx, ct, cols):
    rng = np.random.default_rng(ct)
    raw = synth_raw(rng, 30000, ct)
    res = [0.1 + 0.05 * i for i in range(len(cols))]
    pos = rng.integers(100, 30100, size=77)
    assert eq(ctx.process_recording(raw, ct, cols, res, pos),
              oracle.process_recording(raw, cols, res, pos))


def test_full_32_channel_montage(ctx):
    rng = np.random.default_rng(32)
    raw = synth_raw(rng, 20000, 32)
    cols = list(range(32))
    pos = rng.integers(100, 19000, size=40)
    got = ctx.process_recording(raw, 32, cols, [0.1] * 32, pos)
    assert got.shape == (40, 512)
    assert eq(got, oracle.process_recording(raw, cols, [0.1] * 32, pos))


@pytest.mark.parametrize("ct,C", [(32, 32), (17, 5), (64, 2)])
def test_wide_recording_edges_exact(ctx, ct, C):
    """Any-layout kernels at the recording edges: the first legal marker (pos = 100: baseline from
    frame 0), windows straddling the end (zero padding, partially staged quads) and an all-zero
    epoch (pos - 100 == n_frames)."""
    rng = np.random.default_rng(ct * 100 + C)
    nf = 9000 + ct
    raw = synth_raw(rng, nf, ct)
    cols = list(rng.permutation(ct)[:C])
    res = [0.1 + 0.01 * i for i in range(C)]
    pos = np.concatenate([[100, 101, 102, 103], rng.integers(100, nf, size=30),
                          np.arange(nf - 700, nf + 101, 37), [nf + 100]])
    got = ctx.process_recording(raw, ct, cols, res, pos)
    assert eq(got, oracle.process_recording(raw, cols, res, pos))
    assert np.all(np.isnan(got[-1]))


def test_ieee_float32_recording(ctx):
    rng = np.random.default_rng(11)
    raw = (rng.standard_normal((15000, 3)) * 50).astype(np.float32)
    pos = rng.integers(100, 15000, size=50)
    assert eq(ctx.process_recording(raw, 3, [0, 1, 2], [1.0] * 3, pos),
              oracle.process_recording(raw, [0, 1, 2], [1.0] * 3, pos))
    avg = fx.read_raw(os.path.join(DATA, "DoD", "DoD_2015_02-1.vhdr"),
                      os.path.join(DATA, "DoD", "DoD_2015_02-1.avg"))
    assert eq(ctx.cut_epochs(avg, 3, [0, 1, 2], [1.0] * 3, [101]),
              oracle.decode_epochs(avg, [0, 1, 2], [1.0] * 3, [101]))


def test_feature_size_below_16(ctx):
    rng = np.random.default_rng(9)
    ep = oracle.decode_epochs(synth_raw(rng, 9000, 3), [0, 1, 2], [0.1] * 3,
                              rng.integers(100, 8000, size=20))
    for nf in (1, 5, 8, 12):
        assert eq(ctx.extract_features(ep, feature_size=nf, skip=175),
                  oracle.extract_features(ep, nfeat=nf))
    assert eq(ctx.extract_features(ep, skip=238), oracle.extract_features(ep, skip=238))


def test_fma_numerics_within_tolerance(ctx_fma):
    rng = np.random.default_rng(21)
    raw = synth_raw(rng, 300000, 3)
    pos = rng.integers(100, 299000, size=2000)
    got = ctx_fma.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos)
    want = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos)
    assert np.max(np.abs(got - want)) <= FMA_TOL
    fmafeat = ctx_fma.extract_features(oracle.decode_epochs(raw, [0, 1, 2], [0.1] * 3, pos[:100]))
    assert np.max(np.abs(fmafeat - want[:100])) <= FMA_TOL


# ---- device memory, full-size properties ----------------------------------------------------------
def test_device_memory_full_size_properties(ctx):
    import torch
    n = 1_000_000
    nf = 1000 * n + 2000
    dev = torch.device("cuda", 0)
    raw = torch.empty((nf, 3), dtype=torch.int16, device=dev)
    ctx.synth_recording(raw, 3, 0x5EED)
    pos = torch.arange(1000, 1000 + 1000 * n, 1000, dtype=torch.int64, device=dev)
    out = ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos)
    ctx.synchronize()
    feats = out.cpu().numpy()
    assert feats.shape == (n, 48)
    assert np.all(np.isfinite(feats))
    assert np.max(np.abs(np.linalg.norm(feats, axis=1) - 1.0)) < 1e-12  # unit rows
    # exact parity on a spread sample (oracle on a host copy of the touched frames)
    idx = np.unique(np.concatenate([np.arange(0, n, 9973), [n - 1]]))
    starts = torch.as_tensor(1000 + 1000 * idx - 100, device=dev)
    frames = starts[:, None] + torch.arange(850, device=dev)[None, :]
    windows = raw[frames].cpu().numpy()  # [k][850][3]: everything epoch i reads
    for j, i in enumerate(idx):
        want = oracle.process_recording(np.ascontiguousarray(windows[j]), [0, 1, 2], [0.1] * 3,
                                        [100])
        assert eq(feats[i:i + 1], want), i
    # determinism: a second launch gives identical bytes
    out2 = ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos)
    ctx.synchronize()
    assert torch.equal(out, out2)


def test_errors_are_raised(ctx):
    raw = np.zeros((5000, 3), dtype=np.int16)
    with pytest.raises(fx.EegfxError) as e:
        ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, [50])
    assert e.value.code == -6  # ERANGE: copyOfRange AIOOBE
    with pytest.raises(fx.EegfxError) as e:
        ctx.process_recording(raw, 3, [0, 1, 3], [0.1] * 3, [500])
    assert e.value.code == -1
    with pytest.raises(fx.EegfxError) as e:
        ctx.extract_features(np.zeros((2, 3, 750)), epoch_size=256)
    assert e.value.code == -7
    assert ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, []).shape == (0, 48)


# ---- any-layout fused kernels (wide.hip): configs[3] 32-channel montage, fma numerics ---------
@pytest.mark.parametrize("ct,cols", [(32, list(range(32))), (7, [6, 0, 3, 5]), (3, [2, 1])])
def test_wide_fma_within_tolerance(ctx_fma, ct, cols):
    rng = np.random.default_rng(40 + ct)
    raw = synth_raw(rng, 25000, ct)
    pos = rng.integers(100, 25100, size=61)  # includes zero-padded tails past the end
    got = ctx_fma.process_recording(raw, ct, cols, [0.1] * len(cols), pos)
    want = oracle.process_recording(raw, cols, [0.1] * len(cols), pos)
    assert got.shape == (61, 16 * len(cols))
    nan = np.isnan(want)
    assert np.array_equal(np.isnan(got), nan)
    assert np.max(np.abs(got[~nan] - want[~nan])) <= FMA_TOL


# ---- configs[4]: long recordings streamed from host memory in chunks -------------------------
@pytest.mark.parametrize("chunk,ordered", [(787, False), (1000, False), (4099, False),
                                           (1 << 20, False), (1600, True), (8192, True)])
def test_streamed_equals_resident(ctx, chunk, ordered):
    rng = np.random.default_rng(chunk)
    nf = 60000
    raw = synth_raw(rng, nf, 3)
    pos = rng.integers(100, nf + 100, size=400)  # unsorted, overlapping, tails past the end
    pos[:3] = [100, nf + 100, nf - 50]
    if ordered:  # the in-order fast path (rows leave per chunk) with ramped chunk sizes
        pos = np.sort(pos)
    got = ctx.process_recording_streamed(raw, 3, [0, 1, 2], [0.1] * 3, pos, chunk_frames=chunk)
    assert eq(got, ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos))
    assert eq(got, oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos))


@pytest.mark.parametrize("chunk", [787, 1600, 8192, 1 << 20])
def test_streamed_rows_into_pinned_output(ctx, chunk):
    """In position order into a pinned output (the bench's case): the same rows as the pageable
    output and the oracle, the buffer's other bytes untouched."""
    import torch
    rng = np.random.default_rng(chunk + 5)
    nf = 60000
    raw = synth_raw(rng, nf, 3)
    pos = np.sort(rng.integers(100, nf + 100, size=400))
    pos[-1] = nf + 100
    pinned = torch.full((pos.size + 2, 48), -7.0, dtype=torch.float64, pin_memory=True).numpy()
    out = pinned[1:-1]
    got = ctx.process_recording_streamed(raw, 3, [0, 1, 2], [0.1] * 3, pos, chunk_frames=chunk,
                                         out=out)
    assert eq(got, oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos))
    assert eq(got, ctx.process_recording_streamed(raw, 3, [0, 1, 2], [0.1] * 3, pos,
                                                  chunk_frames=chunk))
    assert np.all(pinned[0] == -7.0) and np.all(pinned[-1] == -7.0)


def test_streamed_pinned_source_and_wide_layout(ctx_fma):
    import torch
    rng = np.random.default_rng(77)
    nf, ct = 40000, 8
    pinned = torch.empty((nf, ct), dtype=torch.int16, pin_memory=True)
    pinned.numpy()[:] = synth_raw(rng, nf, ct)
    raw = pinned.numpy()
    pos = np.sort(rng.integers(100, nf, size=300))
    cols = [7, 1, 4, 0, 2]
    got = ctx_fma.process_recording_streamed(raw, ct, cols, [0.1] * 5, pos, chunk_frames=3000)
    want = oracle.process_recording(raw, cols, [0.1] * 5, pos)
    assert np.max(np.abs(got - want)) <= FMA_TOL
    with pytest.raises(fx.EegfxError):
        ctx_fma.process_recording_streamed(raw, ct, cols, [0.1] * 5, pos, chunk_frames=500)


def test_streamed_float32_recording(ctx):
    # IEEE_FLOAT_32 samples (4-byte frames per channel) through the streamed path: chunk byte
    # offsets scale with the frame size; unsorted positions take the reorder path.
    rng = np.random.default_rng(31)
    nf, ct = 30000, 4
    raw = (rng.standard_normal((nf, ct)) * 40).astype(np.float32)
    pos = rng.integers(100, nf + 100, size=200)
    pos[:2] = [100, nf + 100]
    cols, res = [3, 0], [0.5, 1.0]
    got = ctx.process_recording_streamed(raw, ct, cols, res, pos, chunk_frames=2500)
    assert eq(got, oracle.process_recording(raw, cols, res, pos))


def test_vectorized_recording_through_the_provider(ctx, tmp_path):
    """OffLineDataProvider over a DataOrientation=VECTORIZED copy of DoD2015_01 gives the
    multiplexed original's epochs and features (parity unpinned against eegloader: the reference's
    test data holds no VECTORIZED file, so the copy is synthesised)."""
    raw = fx.read_raw(DOD01 + ".vhdr", DOD01 + ".eeg")
    vhdr = open(DOD01 + ".vhdr", encoding="utf-8").read()
    (tmp_path / "DoD2015_01.vhdr").write_text(
        vhdr.replace("DataOrientation=MULTIPLEXED", "DataOrientation=VECTORIZED"), encoding="utf-8")
    np.ascontiguousarray(raw.T).tofile(str(tmp_path / "DoD2015_01.eeg"))
    with open(DOD01 + ".vmrk", "rb") as f:
        (tmp_path / "DoD2015_01.vmrk").write_bytes(f.read())
    runs = []
    for path in (DOD01 + ".eeg", str(tmp_path / "DoD2015_01.eeg")):
        odp = fx.OffLineDataProvider([path, "1"], context=ctx)
        odp.loadData()
        assert odp.last_error == ""
        runs.append((odp.getData(), odp.getFeatures(), list(odp.getDataLabels())))
    assert runs[0][0].shape == (11, 3, 750)
    assert np.array_equal(runs[0][0], runs[1][0]) and eq(runs[0][1], runs[1][1])
    assert runs[0][2] == runs[1][2]
