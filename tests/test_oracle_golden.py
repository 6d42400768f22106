"""Pins the CPU oracle to the reference's own goldens.

The reference cannot run here (no JVM, un-vendored jars, HDFS), so these asserts are the
reference's test assertions applied to the oracle:
  OfflineDataProviderTest.java:65-67,81,88  11 epochs, 3x750, sum == -253772.18676757812, 5 targets
  OfflineDataProviderTest.java:107-109,129  27 epochs, 3x750, 13 targets
  FeatureExtractionTest.java:88-90,106      11 x 48 features, sum == -24.861844096031625
  /Epochs.csv                               Pz samples of the 11 epochs, per value
"""
import numpy as np
import pytest

from conftest import (DOD02, EPOCH_SUM_GOLDEN, FEATURE_SUM_GOLDEN, INFO_TRAIN, hexrows)
from oracle import oracle


@pytest.fixture(scope="module")
def info_train():
    return oracle.data_provider([INFO_TRAIN])


def test_loading_info_txt_file(info_train):
    ep, lab, pos, err = info_train
    assert err == ""
    assert ep.shape == (11, 3, 750)
    assert oracle.java_epoch_sum(ep) == EPOCH_SUM_GOLDEN
    assert int(sum(lab)) == 5


def test_epochs_csv_pz_bit_exact(info_train, epochs_csv):
    ep = info_train[0]
    assert len(epochs_csv) == 11
    for i, row in enumerate(epochs_csv):
        assert len(row) == 750
        assert np.array_equal(ep[i, 2], np.array(row)), f"Pz row {i}"


def test_selected_markers_dod2015_01(info_train):
    # DoD2015_01 with guessed 1 selects Mk2,8..17
    assert info_train[2] == [12016, 21014, 22517, 24019, 25522, 27024, 28527, 30029, 31531,
                             33034, 34536]
    # Mk2 S2 nt, Mk8 S1 t, Mk9 S1 t, Mk10 S3, Mk11 S5, Mk12 S1 t, Mk13 S1 t, Mk14 S5, Mk15 S1 t,
    # Mk16 S3, Mk17 S3 (balance D = targets - non-targets gates each acceptance)
    assert info_train[1] == [0.0, 1.0, 1.0, 0.0, 0.0, 1.0, 1.0, 0.0, 1.0, 0.0, 0.0]


def test_feature_sum_golden(info_train):
    f = oracle.extract_features(info_train[0])
    assert f.shape == (11, 48)
    assert oracle.java_feature_sum(f) == FEATURE_SUM_GOLDEN


def test_minimal_cascade_equals_full_pyramid(info_train):
    full = oracle.extract_features(info_train[0], faithful=True)
    mini = oracle.extract_features(info_train[0], faithful=False)
    assert np.array_equal(full, mini)


def test_feature_vectors_unit_norm(info_train):
    f = oracle.extract_features(info_train[0])
    assert np.allclose(np.linalg.norm(f, axis=1), 1.0, rtol=0, atol=1e-14)


def test_loading_file_dod_2015_02():
    ep, lab, pos, err = oracle.data_provider([DOD02 + ".eeg", "4"])
    assert err == ""
    assert ep.shape == (27, 3, 750)
    assert int(sum(lab)) == 13


def test_fused_equals_two_stage(info_train):
    raw = np.fromfile(DOD02.replace("DoD_2015_02", "DoD2015_01") + ".eeg", dtype="<i2").reshape(-1, 3)
    fused = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, info_train[2])
    two = oracle.extract_features(info_train[0])
    assert np.array_equal(fused, two)
    mt = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, info_train[2], nthreads=4)
    assert np.array_equal(mt, two)


def test_committed_fixtures_match_oracle(golden_vectors, info_train):
    g = golden_vectors["infoTrain"]
    assert g["positions"] == info_train[2]
    assert g["labels"] == info_train[1]
    assert float.fromhex(g["epoch_sum"]) == EPOCH_SUM_GOLDEN
    assert float.fromhex(g["feature_sum"]) == FEATURE_SUM_GOLDEN
    assert np.array_equal(hexrows(g["features_hex"]), oracle.extract_features(info_train[0]))
    g2 = golden_vectors["DoD_2015_02_g4"]
    ep, lab, pos, _ = oracle.data_provider([DOD02 + ".eeg", "4"])
    assert g2["positions"] == pos and g2["labels"] == lab
    assert np.array_equal(hexrows(g2["features_hex"]), oracle.extract_features(ep))


def test_zero_padded_epoch_past_end():
    # copyOfRange(ch, pos-100, pos+750) with pos+750 > len: zero padding, then baseline.
    rng = np.random.default_rng(1)
    raw = rng.integers(-30000, -20000, size=(2000, 3), dtype=np.int16)
    ep = oracle.decode_epochs(raw, [0, 1, 2], [0.1] * 3, [1500, 2100])
    seg = raw[1400:2000, 0].astype(np.float32) * np.float32(0.1)
    b = np.float32(0)
    for v in seg[:100]:
        b = np.float32(b + v)
    b = np.float32(b / np.float32(100))
    assert ep[0, 0, 499] == np.float64(np.float32(seg[599] - b))
    assert ep[0, 0, 500] == np.float64(np.float32(np.float32(0) - b))
    assert np.all(ep[1] == 0.0)  # pos-100 == len: all-zero epoch (baseline 0)
    f = oracle.extract_features(ep[1:])
    assert np.all(np.isnan(f))   # 0/0 in SignalProcessing.normalize


def test_optimised_cpu_baseline_bit_identical(info_train):
    # bench.py's optimised CPU leg must compute the same features bit for bit:
    # the reference recording, then ragged / zero-padded tails, other layouts, float32 data.
    raw = np.fromfile(DOD02.replace("DoD_2015_02", "DoD2015_01") + ".eeg", dtype="<i2").reshape(-1, 3)
    for nt in (1, 3):
        fast = oracle.process_recording_fast(raw, [0, 1, 2], [0.1] * 3, info_train[2], nthreads=nt)
        assert oracle.java_feature_sum(fast) == FEATURE_SUM_GOLDEN
        assert np.array_equal(fast.view(np.int64),
                              oracle.extract_features(info_train[0]).view(np.int64))
    rng = np.random.default_rng(7)
    for ct, cols, f32 in ((3, [0, 1, 2], False), (5, [4, 0, 2], False), (4, [1, 3], True)):
        k = 37
        raw = (rng.integers(-3000, 3000, size=(1000 * k + 500, ct)) - 20000).astype(np.int16)
        if f32:
            raw = (rng.standard_normal((1000 * k + 500, ct)) * 100).astype(np.float32)
        pos = np.arange(1000, 1000 * (k + 1), 1000, dtype=np.int64)
        pos[-1] = raw.shape[0] + 100      # pos - 100 == n_frames: all-zero epoch -> NaN row
        pos[-2] = raw.shape[0] - 300      # window runs past the end: zero padding
        res = [0.1, 0.25, 0.5][: len(cols)]
        want = oracle.process_recording(raw, cols, res, pos, faithful=True)
        for nt in (1, 4, 64):
            got = oracle.process_recording_fast(raw, cols, res, pos, nthreads=nt)
            assert np.array_equal(got.view(np.int64), want.view(np.int64)), (ct, nt)
    with pytest.raises(ValueError):
        oracle.process_recording_fast(raw, cols, res, pos, win=256)


def test_optimised_extract_features_bit_identical(info_train):
    ep = info_train[0]
    want = oracle.extract_features(ep)
    for i in range(len(ep)):  # one epoch per call, as the drop-in calls it
        got = oracle.extract_features_fast(ep[i:i + 1])
        assert np.array_equal(got.view(np.int64), want[i:i + 1].view(np.int64))
    rng = np.random.default_rng(11)
    for C in (1, 4, 5, 9):
        e = rng.standard_normal((6, C, 750)) * 30
        e[2] = 0.0  # all-zero epoch: NaN row like SignalProcessing.normalize
        a = oracle.extract_features(e)
        b = oracle.extract_features_fast(e)
        assert np.array_equal(a.view(np.int64), b.view(np.int64)), C
