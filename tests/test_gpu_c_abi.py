"""The fused path driven from plain C through include/eegfx.h (the JNI shim's view of the
library): DoD2015_01 -> 11 x 48 features whose Java-order sum equals
FeatureExtractionTest.java:106's golden exactly."""
import subprocess

import pytest

from conftest import DOD01
from test_library_abi import _build_c_consumer

pytestmark = pytest.mark.gpu


def test_plain_c_consumer_gpu(tmp_path):
    exe = _build_c_consumer(tmp_path)
    r = subprocess.run([exe, DOD01, "gpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "golden sum matches" in r.stdout
