"""Classifier-flow glue around the hot path.

Reproduces what ``PipelineBuilder.execute`` does between ``OffLineDataProvider`` and
``IClassifier.train/test`` (Pipeline/PipelineBuilder.java:167-188) so that GPU features feed the
same train/test split the reference uses:

* ``Collections.shuffle(data, new Random(1))`` and ``Collections.shuffle(targets, new Random(1))``
  (:177-179) -- the same permutation for both lists, from java.util.Random's 48-bit LCG;
* ``subList(0, (int)(size*0.7))`` / ``subList((int)(size*0.7), size)`` (:182-187);
* ``featureExtractionFunc`` + ``zip`` into ``LabeledPoint(label, features)``
  (Classification/LogisticRegressionClassifier.java:55-68, :87-94), batched on the device.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

_MULT = 0x5DEECE66D
_MASK = (1 << 48) - 1


class JavaRandom:
    """java.util.Random (the 48-bit linear congruential generator of the JDK)."""

    def __init__(self, seed: int):
        self._seed = (seed ^ _MULT) & _MASK

    def _next(self, bits: int) -> int:
        self._seed = (self._seed * _MULT + 0xB) & _MASK
        v = self._seed >> (48 - bits)
        return v - (1 << bits) if v >= 1 << (bits - 1) and bits == 32 else v

    def nextInt(self, bound: int) -> int:
        if bound <= 0:
            raise ValueError("bound must be positive")
        if bound & (bound - 1) == 0:  # power of two
            return (bound * self._next(31)) >> 31
        while True:
            bits = self._next(31)
            val = bits % bound
            if bits - val + (bound - 1) < (1 << 31):  # no int overflow in Java
                return val


def java_shuffle_permutation(n: int, seed: int = 1) -> List[int]:
    """Index order after ``Collections.shuffle(list, new Random(seed))`` of a list of n items:
    ``for i = n..2: swap(list, i-1, rnd.nextInt(i))``."""
    idx = list(range(n))
    rnd = JavaRandom(seed)
    for i in range(n, 1, -1):
        j = rnd.nextInt(i)
        idx[i - 1], idx[j] = idx[j], idx[i - 1]
    return idx


def reference_split(n: int, seed: int = 1, train_fraction: float = 0.7
                    ) -> Tuple[List[int], List[int]]:
    """(train indices, test indices) into the provider's epoch list, as PipelineBuilder.java
    :177-187 slices the shuffled lists."""
    perm = java_shuffle_permutation(n, seed)
    cut = int(n * train_fraction)  # (int)(data.size()*0.7): truncation of a double
    return perm[:cut], perm[cut:]


def labeled_points(features, labels: Sequence[float]) -> List[Tuple[float, np.ndarray]]:
    """``new LabeledPoint(label, Vectors.dense(features))`` pairs (LogisticRegressionClassifier
    .java:63-68), in list order."""
    f = np.asarray(features)
    if len(f) != len(labels):
        raise ValueError("features and labels differ in length")
    return [(float(labels[i]), f[i]) for i in range(len(labels))]


def train_test_features(odp, fe) -> Tuple[np.ndarray, List[float], np.ndarray, List[float]]:
    """The reference's train/test data for a loaded provider: epochs shuffled and split like
    PipelineBuilder, features extracted in one batched device call per split (the Spark map of
    LogisticRegressionClassifier.java:90,126).  ``fe`` is a WaveletTransform."""
    data = odp.getData()
    labels = odp.getDataLabels()
    tr, te = reference_split(len(labels))
    ftr = fe.extractFeaturesBatch(np.ascontiguousarray(data[tr])) if tr else np.empty((0, 48))
    fte = fe.extractFeaturesBatch(np.ascontiguousarray(data[te])) if te else np.empty((0, 48))
    return ftr, [labels[i] for i in tr], fte, [labels[i] for i in te]
