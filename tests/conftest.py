import json
import os
import sys

import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")
DATA = os.path.join(GOLDEN, "test-data")
INFO_TRAIN = os.path.join(DATA, "infoTrain.txt")
DOD01 = os.path.join(DATA, "DoD", "DoD2015_01")
DOD02 = os.path.join(DATA, "DoD", "DoD_2015_02")

# Reference goldens
EPOCH_SUM_GOLDEN = -253772.18676757812      # OfflineDataProviderTest.java:81
FEATURE_SUM_GOLDEN = -24.861844096031625    # FeatureExtractionTest.java:106


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libeegfx on the device)")


# Run order under `pytest -x`: the golden / oracle parity tests first, so that a failure in a
# heavy test (the 48 GB configs[2] shard, the multi-process rehearsals) can never leave them
# unreached; everything else keeps its collection order inside its rank.
_FIRST = ("test_oracle_golden", "test_library_abi", "test_gpu_parity", "test_gpu_c_abi",
          "test_gpu_fuzz", "test_gpu_fuzz_fused")
_LAST = ("test_gpu_distributed", "test_gpu_configs2")


def _rank(item):
    mod = os.path.splitext(os.path.basename(str(item.fspath)))[0]
    if mod in _FIRST:
        return _FIRST.index(mod)
    if mod in _LAST:
        return 100 + _LAST.index(mod)
    return 50


def pytest_collection_modifyitems(session, config, items):
    items.sort(key=_rank)  # stable: collection order is kept within a module and a rank


@pytest.fixture(scope="session")
def golden_vectors():
    with open(os.path.join(GOLDEN, "golden_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def epochs_csv():
    """/Epochs.csv of the reference: Pz rows of the 11 infoTrain epochs (Double.toString)."""
    rows = []
    with open(os.path.join(GOLDEN, "Epochs.csv")) as f:
        for line in f:
            line = line.strip()
            if line:
                rows.append([float(v) for v in line.rstrip(",").split(",")])
    return rows


def hexrows(rows):
    import numpy as np
    return np.array([[float.fromhex(v) for v in r] for r in rows], dtype=np.float64)
