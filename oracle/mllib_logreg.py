"""CPU restatement of the classifier the reference trains on the dwt-8 features -- TEST
INFRASTRUCTURE ONLY (tests/ and bench.py's cpu_baseline leg import it; the product never does).

The algorithm lives in an un-vendored dependency, ``org.apache.spark:spark-mllib_2.10:1.6.2``
(pom.xml:59-63), which is absent here; this file restates its published Spark 1.6.2 behaviour:

* ``LogisticRegressionClassifier.train`` (Classification/LogisticRegressionClassifier.java:85-114):
  with all of config_num_iterations / config_step_size / config_mini_batch_fraction set it calls
  the static ``LogisticRegressionWithSGD.train(rdd, iters, step, fraction)`` (regParam 0.0);
  otherwise ``new LogisticRegressionWithSGD().run(rdd)`` -- the default constructor's
  (stepSize 1.0, numIterations 100, regParam 0.01, miniBatchFraction 1.0).
* ``GeneralizedLinearAlgorithm.run``: binary-label validation, no intercept, no feature scaling
  (SGD), zero initial weights.
* ``GradientDescent.runMiniBatchSGD``: for i = 1..numIterations while not converged: gradient =
  sum over the (fraction 1.0 = whole) sample of ``LogisticGradient`` / sample size; weights =
  ``SquaredL2Updater``: w *= (1 - step/sqrt(i) * reg); w -= step/sqrt(i) * gradient; converged
  when i >= 2 and ||w_prev - w|| < convergenceTol (0.001) * max(||w||, 1).
* ``LogisticGradient`` (binary): multiplier = 1 / (1 + exp(-w.x)) - label; gradient += multiplier x.
* ``LogisticRegressionModel.predict``: 1.0 if 1 / (1 + exp(-(w.x + b))) > threshold (0.5).
* ``SVMClassifier.train`` (Classification/SVMClassifier.java:83-111): ``SVMWithSGD`` -- the same
  GradientDescent / SquaredL2Updater loop and defaults with ``HingeGradient``: s = 2 label - 1;
  a row with 1 > s * w.x adds -s x to the gradient, any other row adds nothing (the config_*
  path passes config_reg_param through).  ``SVMModel.predict`` (:71): 1.0 if w.x + b > threshold
  (0.0), the margin itself without a threshold.
* ``test`` (:117-141): MulticlassMetrics' 2x2 confusion matrix (rows = actual label, columns =
  predicted, labels ascending) read through ``toArray`` (column-major) as tn, fp, fn, tp =
  cm[0], cm[1], cm[2], cm[3] -- i.e. the reference's "fp" counts actual-1/predicted-0 and its
  "fn" actual-0/predicted-1.

* ``miniBatchFraction`` f < 1 (``config_mini_batch_fraction``, README.md:136): iteration i trains
  on ``data.sample(false, f, 42 + i)`` (GradientDescent 1.6.2), i.e. ``PartitionwiseSampledRDD``
  with a ``BernoulliSampler(f)``: a ``java.util.Random(42 + i)`` draws one ``nextLong`` seed per
  partition in partition order; each partition's sampler is an ``XORShiftRandom`` seeded with it
  (``hashSeed``: two scala ``MurmurHash3.bytesHash`` over ``ByteBuffer.allocate(Long.SIZE)`` --
  64 bytes, the long big-endian in the first 8); for f <= 0.4 a ``GapSamplingIterator`` (skip
  ``(int)(log(max(u, 5e-11)) / log1p(-f))`` rows before the first and after every kept row),
  otherwise keep a row when ``nextDouble() <= f``.  The partitions are ``ParallelCollectionRDD``
  slices of the ``parallelize``d lists (LogisticRegressionClassifier.java:87-94): partition p of
  N holds rows [p n / N, (p + 1) n / N), N = local[*]'s core count (SparkInitializer.java:44) --
  stated by the caller here.  The gradient is divided by the sample size; an empty sample skips
  the update (and the convergence test, which compares the last two updated weight vectors).

Spark sums the per-row gradients per partition and combines partitions in a tree, so its
floating-point order depends on the partitioning (local[*] = the host's core count): parity is a
tolerance on the weights, never bit equality.  Rows are summed here in index order (one
partition).  Parity unpinned: no fixture of the reference holds trained weights or statistics
(ClassifierTest.java's accuracy assertion is commented out), and no reference fixture pins the
sampler; the restated generators are checked against their published definitions only.
"""
from __future__ import annotations

import math

import numpy as np

DEFAULT_STEP = 1.0
DEFAULT_ITERS = 100
DEFAULT_REG = 0.01
DEFAULT_FRACTION = 1.0
CONVERGENCE_TOL = 0.001


M64 = (1 << 64) - 1
M32 = (1 << 32) - 1


def _s32(v):
    v &= M32
    return v - (1 << 32) if v >> 31 else v


def _s64(v):
    v &= M64
    return v - (1 << 64) if v >> 63 else v


class JavaRandom:
    """java.util.Random: 48-bit LCG (only what PartitionwiseSampledRDD uses: nextLong)."""

    def __init__(self, seed):
        self.seed = (seed ^ 0x5DEECE66D) & ((1 << 48) - 1)

    def next(self, bits):
        self.seed = (self.seed * 0x5DEECE66D + 0xB) & ((1 << 48) - 1)
        return _s32(self.seed >> (48 - bits))

    def next_long(self):
        return _s64((self.next(32) << 32) + self.next(32))


def _rotl32(x, r):
    x &= M32
    return ((x << r) | (x >> (32 - r))) & M32


def _mix_last(h, k):
    k = (k * 0xCC9E2D51) & M32
    k = _rotl32(k, 15)
    k = (k * 0x1B873593) & M32
    return (h ^ k) & M32


def _mix(h, k):
    h = _rotl32(_mix_last(h, k), 13)
    return (h * 5 + 0xE6546B64) & M32


def murmur3_bytes_hash(data, seed=0x3C074A61):
    """scala.util.hashing.MurmurHash3.bytesHash (Scala 2.10; default seed = arraySeed)."""
    h = seed & M32
    n = len(data)
    i = 0
    while n - i >= 4:
        k = data[i] | (data[i + 1] << 8) | (data[i + 2] << 16) | (data[i + 3] << 24)
        h = _mix(h, k)
        i += 4
    rem = n - i
    k = 0
    if rem == 3:
        k ^= data[i + 2] << 16
    if rem >= 2:
        k ^= data[i + 1] << 8
    if rem >= 1:
        k ^= data[i]
        h = _mix_last(h, k)
    h ^= n
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return _s32(h)


class XORShiftRandom:
    """org.apache.spark.util.random.XORShiftRandom (Spark 1.6): next(bits) on a 64-bit xorshift
    state, nextDouble as java.util.Random's."""

    def __init__(self, seed):
        buf = (seed & M64).to_bytes(8, "big") + bytes(56)   # ByteBuffer.allocate(Long.SIZE = 64)
        lo = murmur3_bytes_hash(buf)
        hi = murmur3_bytes_hash(buf, lo)
        self.s = ((hi << 32) | (lo & M32)) & M64

    def next(self, bits):
        s = self.s ^ ((self.s << 21) & M64)
        s ^= s >> 35
        s ^= (s << 4) & M64
        self.s = s
        return _s32(s & ((1 << bits) - 1))

    def next_double(self):
        return ((self.next(26) << 27) + self.next(27)) * 2.0 ** -53


def partition_bounds(n, num_partitions):
    """ParallelCollectionRDD.slice positions: partition p holds [p n / N, (p + 1) n / N)."""
    return [(p * n // num_partitions, (p + 1) * n // num_partitions) for p in range(num_partitions)]


def bernoulli_sample(start, end, fraction, seed):
    """BernoulliSampler(fraction) over the rows [start, end) of one partition, seeded `seed`."""
    if fraction <= 0.0:
        return []
    if fraction >= 1.0:
        return list(range(start, end))
    rng = XORShiftRandom(seed)
    if fraction <= 0.4:   # RandomSampler.defaultMaxGapSamplingFraction: GapSamplingIterator
        lnq = math.log1p(-fraction)
        out, r = [], start

        def skip():
            u = max(rng.next_double(), 5e-11)   # RandomSampler.rngEpsilon
            return int(math.log(u) / lnq)

        r += skip()
        while r < end:
            out.append(r)
            r += 1 + skip()
        return out
    return [r for r in range(start, end) if rng.next_double() <= fraction]


def sample_rows(n, fraction, num_partitions, seed):
    """RDD.sample(false, fraction, seed) of the n training rows in num_partitions slices."""
    rnd = JavaRandom(seed)
    rows = []
    for a, b in partition_bounds(n, num_partitions):
        rows.extend(bernoulli_sample(a, b, fraction, rnd.next_long()))
    return rows


def sgd_train(X, y, num_iterations=DEFAULT_ITERS, step_size=DEFAULT_STEP, reg_param=0.0,
              convergence_tol=CONVERGENCE_TOL, initial=None, gradient="logistic",
              mini_batch_fraction=1.0, num_partitions=1):
    """Returns (weights, iterations_run).  gradient: "logistic" (LogisticRegressionWithSGD) or
    "hinge" (SVMWithSGD).  mini_batch_fraction < 1: iteration i's sample as sample_rows(n, f,
    num_partitions, 42 + i)."""
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    n, d = X.shape
    if n == 0:
        raise ValueError("empty training set")
    if not np.all((y == 0.0) | (y == 1.0)):
        raise ValueError("Input validation failed.")
    w = np.zeros(d) if initial is None else np.array(initial, dtype=np.float64)
    prev = None
    i = 1
    done = 0
    while i <= num_iterations:
        Xs, ys = X, y
        if mini_batch_fraction < 1.0:
            rows = sample_rows(n, mini_batch_fraction, num_partitions, 42 + i)
            if not rows:   # "The size of sampled batch is zero": no update, no convergence test
                done = i
                i += 1
                continue
            Xs, ys = X[rows], y[rows]
        if gradient == "hinge":
            s_lab = 2.0 * ys - 1.0
            mult = np.where(1.0 > s_lab * (Xs @ w), -s_lab, 0.0)
        else:
            margin = -(Xs @ w)
            mult = 1.0 / (1.0 + np.exp(margin)) - ys
        grad = (mult[:, None] * Xs).sum(axis=0) / len(ys)
        step = step_size / math.sqrt(i)
        w = w * (1.0 - step * reg_param)
        w = w - step * grad
        done = i
        if prev is not None:
            diff = np.linalg.norm(prev - w)
            if diff < convergence_tol * max(np.linalg.norm(w), 1.0):
                break
        prev = w.copy()
        i += 1
    return w, done


def predict(X, w, intercept=0.0, threshold=0.5):
    score = 1.0 / (1.0 + np.exp(-(np.asarray(X, dtype=np.float64) @ w + intercept)))
    if threshold is None:
        return score
    return (score > threshold).astype(np.float64)


def svm_predict(X, w, intercept=0.0, threshold=0.0):
    margin = np.asarray(X, dtype=np.float64) @ w + intercept
    if threshold is None:
        return margin
    return (margin > threshold).astype(np.float64)


def reference_statistics(pred, labels):
    """(tp, tn, fp, fn) exactly as LogisticRegressionClassifier.test builds them
    (LogisticRegressionClassifier.java:129-137).  MulticlassMetrics (Spark 1.6.2) takes its
    ``labels`` from the actual labels only (tpByClass.keys); predicted classes outside them are
    not in confusionMatrix."""
    pred = np.asarray(pred, dtype=np.float64)
    labels = np.asarray(labels, dtype=np.float64)
    classes = sorted(set(labels.tolist()))
    k = len(classes)
    cm = np.zeros((k, k))
    for a, p in zip(labels, pred):
        if p in classes:
            cm[classes.index(a), classes.index(p)] += 1
    flat = cm.flatten(order="F")  # DenseMatrix.toArray: column-major
    tn, fp, fn, tp = (int(flat[0]), int(flat[1]), int(flat[2]), int(flat[3]))
    return tp, tn, fp, fn
