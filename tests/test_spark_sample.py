"""MLlib 1.6.2's mini-batch sampler (GradientDescent: data.sample(false, f, 42 + i)), restated in
the product (csrc/spark_sample.h, eegfx_spark_sample) and in the oracle (oracle/mllib_logreg.py
sample_rows): the two must keep exactly the same rows.  The generators are pinned to their
published definitions (java.util.Random's known outputs); no reference fixture holds a Spark
sample, so the sampler's parity with Spark itself is unpinned."""
import numpy as np
import pytest

from eeg_dataanalysispackage_amd import classification as clf
from eeg_dataanalysispackage_amd._lib import EegfxError
from oracle import mllib_logreg as ref


def test_java_random_known_outputs():
    # new java.util.Random(42).nextLong(), new Random(0).nextLong() (JDK documentation examples)
    assert ref.JavaRandom(42).next_long() == -5025562857975149833
    assert ref.JavaRandom(0).next_long() == -4962768465676381896


def test_partition_bounds_are_parallel_collection_slices():
    assert ref.partition_bounds(10, 3) == [(0, 3), (3, 6), (6, 10)]
    assert ref.partition_bounds(2, 4) == [(0, 0), (0, 1), (1, 1), (1, 2)]


@pytest.mark.parametrize("n,f,parts", [(1000, 0.1, 4), (1000, 0.5, 4), (37, 0.3, 8),
                                       (5000, 0.05, 16), (5000, 0.9, 3), (100, 0.0, 2),
                                       (100, 1.0, 2), (12345, 0.4, 7), (12345, 0.41, 7),
                                       (3, 0.2, 16), (70000, 0.01, 256)])
def test_product_sampler_equals_oracle(n, f, parts):
    for i in (1, 2, 57, 100):   # GradientDescent's seed 42 + i
        got = clf.spark_sample(n, f, parts, 42 + i)
        want = np.array(ref.sample_rows(n, f, parts, 42 + i), dtype=np.int64)
        assert np.array_equal(got, want), (n, f, parts, i)


def test_sampler_rates():
    # Bernoulli(f): the kept fraction concentrates around f on both code paths (gap / filter)
    for f in (0.1, 0.4, 0.5, 0.8):
        k = np.mean([clf.spark_sample(20000, f, 8, 42 + i).size for i in range(1, 11)]) / 20000
        assert abs(k - f) < 0.01, (f, k)


def test_sampler_argument_checks():
    with pytest.raises(EegfxError):
        clf.spark_sample(10, 1.5, 2, 43)      # BernoulliSampler: fraction outside [0, 1]
    with pytest.raises(EegfxError):
        clf.spark_sample(10, 0.5, 0, 43)
