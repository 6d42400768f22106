"""The opt-in resident server of the per-epoch drop-in (eegfx_ctx_set_mailbox): small host
extract batches -- IFeatureExtraction.extractFeatures called once per epoch from the Spark map
closure (LogisticRegressionClassifier.java:55-61) -- served by a workgroup that stays on the
device.  Bar: the same rows as the launch path (the same kernel code), bit for bit, in both
numerics; the server survives buffer growth, its own idle exit, concurrent contexts and a
context destroyed with it running.  Every context here is host-only (no torch device sync while a
server is resident)."""
import threading
import time

import numpy as np
import pytest

import eeg_dataanalysispackage_amd as fx
from conftest import INFO_TRAIN, hexrows
from oracle import oracle

pytestmark = pytest.mark.gpu


def eq(a, b):
    return np.array_equal(a, b, equal_nan=True)


@pytest.fixture(scope="module")
def epochs():
    odp = fx.OffLineDataProvider([INFO_TRAIN])
    odp.loadData()
    return np.ascontiguousarray(odp.getData())


@pytest.mark.parametrize("numerics", ["exact", "fma"])
def test_mailbox_rows_equal_launch_path(epochs, golden_vectors, numerics):
    c = fx.Context(0, numerics=numerics)
    try:
        want = np.stack([c.extract_features(epochs[i:i + 1])[0] for i in range(len(epochs))])
        c.set_mailbox(True)
        got = np.stack([c.extract_features(epochs[i:i + 1])[0] for i in range(len(epochs))])
        assert eq(got, want)
        assert eq(c.extract_features(epochs), want)                 # the 11-epoch batch
        if numerics == "exact":
            assert eq(got, hexrows(golden_vectors["infoTrain"]["features_hex"]))
        # growth of the pinned staging (stops and restarts the server), then small again
        big = np.concatenate([epochs] * 6)                          # 66 epochs, 1.6 MB rows
        assert eq(c.extract_features(big[:64]), np.concatenate([want] * 6)[:64])
        assert eq(c.extract_features(epochs[3:4]), want[3:4])
        c.set_mailbox(False)
        assert eq(c.extract_features(epochs[5:6]), want[5:6])       # back on the launch path
    finally:
        c.set_mailbox(False)
        c.close()


def test_mailbox_idle_exit_and_restart(epochs):
    c = fx.Context(0)
    try:
        want = oracle.extract_features(epochs[:2])
        c.set_mailbox(True)
        assert eq(c.extract_features(epochs[:1]), want[:1])
        time.sleep(1.3)   # longer than the server's 1 s idle limit: it has returned
        assert eq(c.extract_features(epochs[1:2]), want[1:2])
        c.set_mailbox(True)   # idempotent
        assert eq(c.extract_features(epochs[:2]), want)
    finally:
        c.set_mailbox(False)
        c.close()


def test_mailbox_concurrent_contexts_and_destroy(epochs):
    """Four threads, a context and a resident server each (the Spark executor threads), all
    serving single epochs at once; every context destroyed with its server still running."""
    want = oracle.extract_features(epochs)
    errors = []

    def work(t):
        c = fx.Context(0)
        try:
            c.set_mailbox(True)
            for k in range(200):
                i = (t + k) % len(epochs)
                if not eq(c.extract_features(epochs[i:i + 1]), want[i:i + 1]):
                    errors.append((t, k))
        except Exception as exc:   # reported below
            errors.append(repr(exc))
        finally:
            c.close()              # destroys the context with the server resident

    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=90)
    assert not any(x.is_alive() for x in th)
    assert errors == []


@pytest.mark.parametrize("C,nfeat", [(1, 16), (5, 7), (16, 16)])
def test_per_epoch_kernel_any_channel_count(C, nfeat):
    """The per-epoch kernel beyond the 3-channel montage, launched and served resident: up to 16
    channels (rows of up to 256 features, so the lane-ordered sum of squares takes four passes of
    64) and feature sizes below 16, value-identical to the oracle under EXACT and within 1e-9
    under fma."""
    rng = np.random.default_rng(100 + C)
    nf = 6000
    raw = np.clip(rng.integers(-26000, -24000, size=(1, C)) +
                  np.cumsum(rng.integers(-40, 41, size=(nf, C)), axis=0), -32768, 32767)
    raw = raw.astype(np.int16)
    ep = oracle.decode_epochs(raw, list(range(C)), [0.1] * C, [500, 1800, 3100, 4400])
    want = oracle.extract_features(ep, nfeat=nfeat)
    for numerics in ("exact", "fma"):
        c = fx.Context(0, numerics=numerics)
        try:
            for mailbox in (False, True):
                c.set_mailbox(mailbox)
                got = np.concatenate([c.extract_features(ep[i:i + 1], feature_size=nfeat)
                                      for i in range(len(ep))])
                if numerics == "exact":
                    assert eq(got, want), (C, nfeat, mailbox)
                else:
                    assert np.max(np.abs(got - want)) <= 1e-9, (C, nfeat, mailbox)
                assert eq(c.extract_features(ep, feature_size=nfeat), got)  # the 4-epoch batch
        finally:
            c.set_mailbox(False)
            c.close()


def test_streamed_calls_beside_resident_servers(epochs):
    """The streamed ingest on a context whose server -- and another context's -- is resident: its
    pinned staging is grow-only, so a call neither frees host memory (hipHostFree synchronises the
    whole device, i.e. waits up to 1 s for every resident server's idle exit) nor returns wrong
    rows; growth stops the context's own server first."""
    rng = np.random.default_rng(5)
    nf = 40_000
    raw = np.clip(-25000 + np.cumsum(rng.integers(-40, 41, size=(nf, 3)), axis=0), -32768,
                  32767).astype(np.int16)
    pos = np.arange(1000, nf - 1000, 997, dtype=np.int64)
    want = oracle.process_recording(raw, [0, 1, 2], [0.1] * 3, pos)
    want_ep = oracle.extract_features(epochs[:1])
    c, other = fx.Context(0), fx.Context(0)
    try:
        for x in (c, other):
            x.set_mailbox(True)
            assert eq(x.extract_features(epochs[:1]), want_ep)
        times = []
        for chunk in (5000, 5000, 9000):   # first use, reuse, growth
            t = time.perf_counter()
            got = c.process_recording_streamed(raw, 3, [0, 1, 2], [0.1] * 3, pos,
                                               chunk_frames=chunk)
            times.append(time.perf_counter() - t)
            assert eq(got, want), chunk
            assert eq(other.extract_features(epochs[:1]), want_ep)   # other's server still serves
        print("streamed call times (first use, reuse, growth):", times)
        assert times[1] < 0.5, times   # reuse: no device-wide synchronisation behind the servers
        assert eq(c.extract_features(epochs[:1]), want_ep)   # c's server restarted after growth
    finally:
        for x in (c, other):
            x.set_mailbox(False)
            x.close()


def _build_mailbox_threads(tmp_path):
    import os
    import subprocess
    from eeg_dataanalysispackage_amd import _lib
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "mailbox_threads")
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Werror", "-pthread",
                    "-I", os.path.join(repo, "include"),
                    os.path.join(repo, "tests", "c_abi", "mailbox_threads.c"), "-L", libdir,
                    "-leegfx", f"-Wl,-rpath,{libdir}", "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("threads", [5, 16, 32])
def test_mailbox_server_slots_at_spark_thread_counts(tmp_path, threads):
    """Spark local[*] with -Deegfx.mailbox=true: one context per executor thread, every one asking
    for a resident server (tests/c_abi/mailbox_threads.c, native threads, 200 single-epoch calls
    each).  The high-priority queue pool holds 4 servers; a fifth used to share a queue with a
    busy server and wait for it to idle out (1 s) or fail after 30 s.  Now at most 4
    contexts are resident at once, the rest take the launch path, every row equals the launch
    path's, and no call stalls.  The small-call staging is allocated when the server is enabled, so
    no first call grows it and restarts the server (those calls took 3-4 ms at 32 threads); the
    slowest call measured 0.3-0.8 ms at 32 threads.  The bound here is 10 ms: the
    box's 16 host cores are shared, and descheduled threads have taken 1-3 ms."""
    import subprocess
    from conftest import DOD01
    exe = _build_mailbox_threads(tmp_path)
    r = subprocess.run([exe, DOD01 + ".vhdr", str(threads), "200"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    line = r.stdout.strip().splitlines()[-1]
    print(line)
    f = line.split()
    vals = dict(zip(f[0::2], f[1::2]))
    assert 1 <= int(vals["resident"]) <= 4
    assert float(vals["max_us"]) < 10_000
