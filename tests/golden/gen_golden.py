"""Generates tests/golden/golden_vectors.json from the CPU oracle.

The reference (Java + two un-vendored jars + HDFS) cannot run in this container (SURVEY.md
8c), so the chain of trust is:  reference goldens (OfflineDataProviderTest.java:81,88,107,129,
FeatureExtractionTest.java:106, Epochs.csv)  --pin-->  oracle (tests/test_oracle_golden.py)
--generates-->  these per-value fixtures (doubles as hex strings, bit-exact).

Run:  python tests/golden/gen_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

from oracle import oracle  # noqa: E402

DATA = os.path.join(HERE, "test-data")


def case(args):
    ep, lab, pos, err = oracle.data_provider(args)
    feats = oracle.extract_features(ep) if len(ep) else ep.reshape(0, 48)
    return {
        "args": [os.path.relpath(a, HERE) if a.endswith((".txt", ".eeg")) else a for a in args],
        "n_epochs": int(len(ep)),
        "positions": [int(p) for p in pos],
        "labels": lab,
        "error": err,
        "epoch_sum": oracle.java_epoch_sum(ep).hex(),
        "features_hex": [[float(v).hex() for v in row] for row in feats],
        "feature_sum": oracle.java_feature_sum(feats).hex(),
    }


def main():
    out = {
        "infoTrain": case([os.path.join(DATA, "infoTrain.txt")]),
        "DoD_2015_02_g4": case([os.path.join(DATA, "DoD", "DoD_2015_02.eeg"), "4"]),
    }
    with open(os.path.join(HERE, "golden_vectors.json"), "w") as f:
        json.dump(out, f, indent=1)
    print({k: (v["n_epochs"], sum(v["labels"])) for k, v in out.items()})


if __name__ == "__main__":
    main()
