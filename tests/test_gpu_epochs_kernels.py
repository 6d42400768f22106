"""The materialised-epoch kernels on the device (kernels.hip): features_from_epochs_kernel (batched
WaveletTransform.extractFeatures on double[n][C][750], WaveletTransform.java:107-141) and the
getData() write passes cut_write_small_kernel / cut_write_kernel (OffLineDataProvider.java:216-233).

The batch extractor stages eight windows per channel through LDS and, under fma numerics, runs the
collapsed four-point filter on the doubles; its feature rows sit in dynamic LDS (8 x 16C doubles)
while the workgroup still fits three times per CU (C <= 20), and go through the output rows beyond
(C = 21, 32, 64: rescaled in place at the end).  Ragged tiles (n not a multiple of 8) read the last epoch's windows and drop the
result.  EXACT must equal the oracle value for value; fma within 1e-9 per normalised feature (the
north_star tolerance).  Inputs are random doubles, not only decoded int16 epochs, since the API
takes any double rows."""
import numpy as np
import pytest

import eeg_dataanalysispackage_amd as fx
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctxs():
    a, b = fx.Context(0, numerics="exact"), fx.Context(0, numerics="fma")
    yield a, b
    a.close()
    b.close()


def eq(a, b):
    return np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("C", [1, 2, 5, 17, 20, 21, 32, 64])
@pytest.mark.parametrize("n", [1, 7, 9, 33])
def test_device_batch_extract(ctxs, C, n):
    import torch
    rng = np.random.default_rng(1000 * C + n)
    ep = rng.standard_normal((n, C, 750)) * rng.choice([1e-3, 1.0, 3e4])
    ep[0, 0, 175:687] += 250.0  # a DC step inside one window
    want = oracle.extract_features(ep)
    exact, fma = ctxs
    dep = torch.from_numpy(ep).cuda()
    got = exact.extract_features(dep).cpu().numpy()
    assert eq(got, want), (C, n)
    got_f = fma.extract_features(dep).cpu().numpy()
    assert np.max(np.abs(got_f - want)) <= 1e-9, (C, n)


@pytest.mark.parametrize("C", [3, 32])
@pytest.mark.parametrize("nf,skip", [(1, 0), (8, 100), (12, 5), (16, 238)])
def test_device_batch_extract_feature_size_and_skip(ctxs, nf, skip, C):
    import torch
    rng = np.random.default_rng(nf + skip + C)
    ep = rng.standard_normal((21, C, 750))
    want = oracle.extract_features(ep, nfeat=nf, skip=skip)
    exact, fma = ctxs
    dep = torch.from_numpy(ep).cuda()
    assert eq(exact.extract_features(dep, feature_size=nf, skip=skip).cpu().numpy(), want)
    got_f = fma.extract_features(dep, feature_size=nf, skip=skip).cpu().numpy()
    assert np.max(np.abs(got_f - want)) <= 1e-9


@pytest.mark.parametrize("C", [3, 32])
def test_device_batch_extract_zero_rows(ctxs, C):
    """An all-zero window normalises to NaN (0/0), as SignalProcessing.normalize does (rows in LDS
    at C = 3, rescaled in the output at C = 32)."""
    import torch
    ep = np.zeros((9, C, 750))
    ep[3] = np.random.default_rng(5).standard_normal((C, 750))
    want = oracle.extract_features(ep)
    for c in ctxs:
        got = c.extract_features(torch.from_numpy(ep).cuda()).cpu().numpy()
        assert np.array_equal(np.isnan(got), np.isnan(want))
        assert np.max(np.abs(got[3] - want[3])) <= 1e-9


@pytest.mark.parametrize("fmt", ["int16", "float32"])
@pytest.mark.parametrize("cols", [[0], [2, 0], [1, 2, 0], [3, 1, 4, 0]])
def test_device_cut_epochs_small_and_wide(ctxs, fmt, cols):
    """getData() on the device: C <= 3 takes cut_write_small_kernel, C = 4 the general write pass;
    markers at both legal ends (pos = 100, windows past the recording's end, zero-padded)."""
    import torch
    rng = np.random.default_rng(len(cols) + (7 if fmt == "int16" else 11))
    ct, nf = 5, 40_000
    if fmt == "int16":
        raw = np.clip(rng.integers(-26000, -24000, size=(1, ct)) +
                      np.cumsum(rng.integers(-40, 41, size=(nf, ct)), axis=0),
                      -32768, 32767).astype(np.int16)
    else:
        raw = (rng.standard_normal((nf, ct)) * 50.0).astype(np.float32)
    pos = np.concatenate([[100], rng.integers(100, nf, size=37), [nf - 200, nf + 100]])
    res = [0.1, 0.25, 1.0, 0.5][:len(cols)]
    want = oracle.decode_epochs(raw, cols, res, pos)
    exact, _ = ctxs
    got = exact.cut_epochs(torch.from_numpy(raw).cuda(), ct, cols, res,
                           torch.from_numpy(pos.astype(np.int64)).cuda())
    exact.synchronize()
    assert eq(got.cpu().numpy(), want)


@pytest.mark.parametrize("fmt,ct,cols", [
    ("int16", 32, list(range(32))),           # configs[3]'s montage: 16 dwords per frame
    ("int16", 32, [31, 0, 7, 16, 3]),         # a few of many channels, any order
    ("int16", 8, [7, 6, 5, 4, 3, 2, 1, 0]),   # 4 dwords per frame
    ("int16", 6, [0, 2, 4, 5]),               # odd dword count per frame (even LDS stride)
    ("int16", 3, [0, 1, 2]),                  # 6-byte frames: the packed staging (configs[1])
    ("int16", 3, [2, 0]),
    ("int16", 7, [3]),                        # 14-byte frames, one channel of seven
    ("float32", 32, list(range(0, 32, 2))),   # 33 staged dwords per frame: two chunks per epoch
    ("float32", 5, [4, 3, 2, 1, 0]),
])
def test_device_cut_epochs_lds_staged(ctxs, fmt, ct, cols):
    """getData() with the LDS-staged write passes (the epoch's frames at most twice the rows):
    cut_write_lds_kernel for whole-dword frames (padded per frame, in chunks),
    cut_write_lds_packed_kernel for int16 frames that are not (staged as they lie); rows written as
    16-byte pairs.  Value-equal to the oracle's decode (OffLineDataProvider.java:216-233), markers at
    pos = 100 and past the end of the recording (zero padding, Arrays.copyOfRange)."""
    import torch
    rng = np.random.default_rng(ct * 100 + len(cols))
    nf = 12_001  # odd: with an odd channel count the recording ends inside a dword
    if fmt == "int16":
        raw = np.clip(rng.integers(-26000, -24000, size=(1, ct)) +
                      np.cumsum(rng.integers(-40, 41, size=(nf, ct)), axis=0),
                      -32768, 32767).astype(np.int16)
    else:
        raw = (rng.standard_normal((nf, ct)) * 50.0).astype(np.float32)
    pos = np.concatenate([[100], rng.integers(100, nf, size=21), [nf - 749, nf - 400, nf, nf + 100]])
    res = list(rng.choice([0.1, 0.25, 1.0, 0.5, 0.048828125], size=len(cols)))
    want = oracle.decode_epochs(raw, cols, res, pos)
    exact, _ = ctxs
    got = exact.cut_epochs(torch.from_numpy(raw).cuda(), ct, cols, res,
                           torch.from_numpy(pos.astype(np.int64)).cuda())
    exact.synchronize()
    assert eq(got.cpu().numpy(), want)
