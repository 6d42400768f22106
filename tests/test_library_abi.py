"""libeegfx.so loads here (no GPU) and exports exactly the C ABI of include/eegfx.h (the hot-path
drop-in contract) plus include/eegfx_ext.h (the out-of-scope SVM extension)."""
import os
import re
import subprocess

import numpy as np
import pytest

import eeg_dataanalysispackage_amd as fx
from eeg_dataanalysispackage_amd import _lib
from conftest import REPO

HEADER = os.path.join(REPO, "include", "eegfx.h")
EXT_HEADER = os.path.join(REPO, "include", "eegfx_ext.h")


def declared_functions(headers=(HEADER, EXT_HEADER)):
    found = set()
    for h in headers:
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        found |= set(re.findall(r"\b(eegfx_[a-z0-9_]+)\s*\(", text))
    return found


def test_svm_is_outside_the_drop_in_contract():
    # SVM is out of scope; its entry points live in the extension header only
    core, ext = declared_functions((HEADER,)), declared_functions((EXT_HEADER,))
    assert ext == {"eegfx_svm_sgd_train", "eegfx_svm_predict"}
    assert not any("svm" in f for f in core)


def exported_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], check=True,
                         capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_library_loads_and_reports_version():
    assert os.path.exists(_lib.LIB_PATH)
    assert fx.lib().eegfx_version().decode().startswith("eegfx")


def test_every_declared_function_is_exported_and_bound():
    decl = declared_functions()
    assert len(decl) >= 25
    missing = decl - exported_symbols()
    assert not missing, missing
    assert decl == set(_lib.SIGNATURES), decl ^ set(_lib.SIGNATURES)


def test_no_oracle_in_product_path():
    # The product must never link or import the CPU oracle.
    pkg = os.path.join(REPO, "eeg_dataanalysispackage_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                src = open(os.path.join(root, f), encoding="utf-8").read()
                assert "oracle" not in src.replace("oracle/", "").lower() or f == "_lib.py", f
    deps = subprocess.run(["ldd", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in deps


def test_status_mapping_without_gpu():
    # Host-only entry points report errors through status + eegfx_last_error().
    import ctypes
    info = _lib.HeaderInfo()
    rc = fx.lib().eegfx_read_header(b"/nonexistent.vhdr", ctypes.byref(info), None, 0)
    assert rc == _lib.EEGFX_EIO
    assert b"cannot open" in fx.lib().eegfx_last_error()


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    """No CPU fallback: with the shared object gone, every entry point raises."""
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "libeegfx.so"))
    import pytest
    with pytest.raises(ImportError, match="missing"):
        _lib.lib()
    with pytest.raises(ImportError):
        fx.Context(0)


def _build_c_consumer(tmp_path):
    exe = str(tmp_path / "abi_consumer")
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-O1", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "c_abi", "abi_consumer.c"), "-L", libdir, "-leegfx",
                    f"-Wl,-rpath,{libdir}", "-o", exe], check=True)
    return exe


def _build_shim_consumer(tmp_path):
    """tests/c_abi/shim_consumer.c + the JNI shim's core (integration/jni/eegfx_shim.c), plain C."""
    exe = str(tmp_path / "shim_consumer")
    libdir = os.path.dirname(_lib.LIB_PATH)
    jni = os.path.join(REPO, "integration", "jni")
    subprocess.run(["gcc", "-std=c99", "-O1", "-Wall", "-Werror", "-pthread",
                    "-I", os.path.join(REPO, "include"), "-I", jni,
                    os.path.join(REPO, "tests", "c_abi", "shim_consumer.c"),
                    os.path.join(jni, "eegfx_shim.c"), "-L", libdir, "-leegfx",
                    f"-Wl,-rpath,{libdir}", "-o", exe], check=True)
    return exe


def test_java_shim_core_host(tmp_path):
    """The Java drop-in's shim core from C without a device: exception mapping, the reference's
    confusion-matrix reading, and the planning-only provider on infoTrain.txt (11 epochs, 5
    targets, OfflineDataProviderTest.java:65-88)."""
    from conftest import INFO_TRAIN
    exe = _build_shim_consumer(tmp_path)
    r = subprocess.run([exe, INFO_TRAIN], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "shim_consumer ok (host)" in r.stdout


def test_plain_c_consumer(tmp_path):
    """The ABI from plain C (what the JNI shim is): header parsing, marker planning against the
    reference golden, error statuses -- no GPU needed."""
    exe = _build_c_consumer(tmp_path)
    from conftest import DOD01
    r = subprocess.run([exe, DOD01], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "abi_consumer ok" in r.stdout


def test_no_environment_knobs_in_the_product():
    """The kernel choice of every call is a function of its arguments only: no getenv in the
    library sources (the rejected perf-study variants live as patches under tools/probes/history/)."""
    csrc = os.path.join(REPO, "eeg_dataanalysispackage_amd", "csrc")
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".cpp", ".h")):
            assert "getenv(" not in open(os.path.join(csrc, f)).read(), f


def test_recording_frame_checks():
    # Context methods derive n_frames from the buffer and n_channels_total; a count that does not
    # divide the buffer, is not positive, or disagrees with a 2-D recording is refused before any
    # device call.
    from eeg_dataanalysispackage_amd.context import _frames
    raw = np.zeros((100, 3), dtype=np.int16)
    assert _frames(raw, 3) == 100
    assert _frames(raw.reshape(-1), 3) == 100
    assert _frames(raw.reshape(-1), 4) == 75
    for bad in (0, -3):
        with pytest.raises(ValueError):
            _frames(raw, bad)
    with pytest.raises(ValueError):
        _frames(raw, 4)              # 2-D with 3 channels per frame
    with pytest.raises(ValueError):
        _frames(raw.reshape(-1), 7)  # 300 samples are not frames of 7
