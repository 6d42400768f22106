"""The downstream classifiers of the train/test flow on the GPU.

Mirrors ``Classification/LogisticRegressionClassifier`` and ``Classification/SVMClassifier``
(IClassifier) and
``Utils/ClassificationStatistics`` of the reference: ``train(epochs, targets, fe)`` extracts the
features of the epochs (one batched device call instead of the Spark map of :90) and fits Spark
MLlib 1.6.2 ``LogisticRegressionWithSGD`` on the device (``eegfx_logreg_sgd_train``);
``test(epochs, targets)`` predicts on the device and builds the statistics exactly as :117-141 do,
including the reference's reading of the column-major confusion matrix (its "false positives"
count actual-1 / predicted-0).  ``SVMClassifier`` is the same flow with MLlib 1.6.2
``SVMWithSGD`` (HingeGradient, ``eegfx_svm_sgd_train``) and ``SVMModel.predict`` (margin > 0).
Model save/load (Spark model directories) is out of scope.
"""
from __future__ import annotations

import math
from ctypes import byref, c_int32, c_int64
from typing import Dict, Optional, Sequence

import numpy as np

from ._lib import EegfxError, lib, ptr
from .context import Context, _contig, _is_device, _mem

# LogisticRegressionWithSGD() defaults (MLlib 1.6.2) and GradientDescent's convergence tolerance
DEFAULT_STEP_SIZE = 1.0
DEFAULT_NUM_ITERATIONS = 100
DEFAULT_REG_PARAM = 0.01
DEFAULT_MINI_BATCH_FRACTION = 1.0
CONVERGENCE_TOL = 0.001


def _train(entry, ctx: Context, X, y, num_iterations, step_size, reg_param, mini_batch_fraction,
           convergence_tol, initial_weights, num_partitions=None):
    if _is_device(X) != _is_device(y):
        raise ValueError("X and y must both be host or both be device arrays")
    X = _contig(X, np.float64)
    y = _contig(y, np.float64)
    n, d = int(X.shape[0]), int(X.shape[1])
    if X.ndim != 2 or y.ndim != 1 or int(y.shape[0]) != n:
        raise ValueError(f"X must be [n][d] and y [n], got {tuple(X.shape)} and {tuple(y.shape)}")
    w = (np.zeros(d) if initial_weights is None
         else np.array(initial_weights, dtype=np.float64).copy())
    it = c_int32()
    mem = _mem(X, y)
    # ordered after the torch work that produced X / y (Context._call), like every device call
    head = (ctx.handle, ptr(X), ptr(y), n, d, int(num_iterations), float(step_size),
            float(reg_param), float(mini_batch_fraction), float(convergence_tol))
    if num_partitions is None:
        ctx._call(mem, X, getattr(lib(), entry), *head, ptr(w), byref(it), mem)
    else:
        ctx._call(mem, X, getattr(lib(), entry + "_partitioned"), *head, int(num_partitions),
                  ptr(w), byref(it), mem)
    return w, it.value


def _predict(entry, ctx: Context, X, weights, intercept, threshold):
    w = np.ascontiguousarray(weights, dtype=np.float64)
    X = _contig(X, np.float64)
    n, d = int(X.shape[0]), int(X.shape[1])
    if _is_device(X):
        import torch
        out = torch.empty(n, dtype=torch.float64, device=X.device)
    else:
        out = np.empty(n, dtype=np.float64)
    t = math.nan if threshold is None else float(threshold)
    mem = _mem(X, out)
    ctx._call(mem, X, getattr(lib(), entry), ctx.handle, ptr(X), n, d, ptr(w), float(intercept),
              t, ptr(out), mem)
    return out


def sgd_train(ctx: Context, X, y, num_iterations: int = DEFAULT_NUM_ITERATIONS,
              step_size: float = DEFAULT_STEP_SIZE, reg_param: float = 0.0,
              mini_batch_fraction: float = DEFAULT_MINI_BATCH_FRACTION,
              convergence_tol: float = CONVERGENCE_TOL, initial_weights=None,
              num_partitions: Optional[int] = None):
    """LogisticRegressionWithSGD on the device; returns (weights, iterations_run).  X (n x d
    float64, host numpy or device torch) and y (n labels 0/1) may live on either side.
    mini_batch_fraction < 1 samples iteration i's mini-batch as MLlib's data.sample(false, f,
    42 + i) over num_partitions Spark partitions (None: the processors available to the process,
    affinity and cgroup quota honoured, as Spark local[*]'s Runtime.availableProcessors();
    eegfx_logreg_sgd_train_partitioned)."""
    return _train("eegfx_logreg_sgd_train", ctx, X, y, num_iterations, step_size, reg_param,
                  mini_batch_fraction, convergence_tol, initial_weights, num_partitions)


def spark_sample(n: int, fraction: float, num_partitions: int, seed: int) -> np.ndarray:
    """RDD.sample(false, fraction, seed) of n rows in num_partitions slices (eegfx_spark_sample,
    host only): the kept row indices, ascending."""
    words = np.zeros((n + 31) // 32, dtype=np.uint32)
    kept = c_int64()
    from ._lib import check
    check(lib().eegfx_spark_sample(int(n), float(fraction), int(num_partitions), int(seed),
                                   ptr(words), byref(kept)))
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:n]
    rows = np.nonzero(bits)[0]
    assert rows.size == kept.value
    return rows


def predict(ctx: Context, X, weights, intercept: float = 0.0,
            threshold: Optional[float] = 0.5):
    """LogisticRegressionModel.predict on the device: 0/1 per row, or the score when
    ``threshold`` is None (clearThreshold)."""
    return _predict("eegfx_logreg_predict", ctx, X, weights, intercept, threshold)


def svm_sgd_train(ctx: Context, X, y, num_iterations: int = DEFAULT_NUM_ITERATIONS,
                  step_size: float = DEFAULT_STEP_SIZE, reg_param: float = DEFAULT_REG_PARAM,
                  mini_batch_fraction: float = DEFAULT_MINI_BATCH_FRACTION,
                  convergence_tol: float = CONVERGENCE_TOL, initial_weights=None):
    """Full-batch SVMWithSGD (HingeGradient) on the device; returns (weights, iterations_run)."""
    return _train("eegfx_svm_sgd_train", ctx, X, y, num_iterations, step_size, reg_param,
                  mini_batch_fraction, convergence_tol, initial_weights)


def svm_predict(ctx: Context, X, weights, intercept: float = 0.0,
                threshold: Optional[float] = 0.0):
    """SVMModel.predict on the device: margin w.x + b > threshold (0.0) -> 1 else 0, or the
    margin when ``threshold`` is None (clearThreshold)."""
    return _predict("eegfx_svm_predict", ctx, X, weights, intercept, threshold)


class ClassificationStatistics:
    """Utils/ClassificationStatistics.java (the counters the classifiers report)."""

    def __init__(self, truePositives: int = 0, trueNegatives: int = 0, falsePositives: int = 0,
                 falseNegatives: int = 0):
        self.truePositives = int(truePositives)
        self.trueNegatives = int(trueNegatives)
        self.falsePositives = int(falsePositives)
        self.falseNegatives = int(falseNegatives)

    def getNumberOfPatterns(self) -> int:
        return self.truePositives + self.trueNegatives + self.falsePositives + self.falseNegatives

    def calcAccuracy(self) -> float:
        n = self.getNumberOfPatterns()
        return (self.truePositives + self.trueNegatives) / n if n else math.nan

    def as_tuple(self):
        return (self.truePositives, self.trueNegatives, self.falsePositives, self.falseNegatives)

    def __repr__(self) -> str:
        return (f"Number of patterns: {self.getNumberOfPatterns()}\n"
                f"True positives: {self.truePositives}\nTrue negatives: {self.trueNegatives}\n"
                f"False positives: {self.falsePositives}\n"
                f"False negatives: {self.falseNegatives}\n"
                f"Accuracy: {self.calcAccuracy() * 100}%\n")


def reference_statistics(predictions, labels) -> ClassificationStatistics:
    """LogisticRegressionClassifier.test :129-137: MulticlassMetrics' confusion matrix (rows =
    actual, columns = predicted, labels ascending) flattened column-major by toArray and read as
    tn, fp, fn, tp = cm[0], cm[1], cm[2], cm[3].  Spark 1.6's ``labels`` are the classes of the
    ACTUAL labels only (``tpByClass.keys``, built from ``labelCountByClass``), and a prediction
    of a class outside them falls out of the matrix.  With a single actual class the matrix is 1x1
    and the reference's cm[1] throws; so does this (IndexError)."""
    p = np.asarray(predictions, dtype=np.float64)
    a = np.asarray(labels, dtype=np.float64)
    classes = sorted(set(a.tolist()))
    k = len(classes)
    cm = np.zeros((k, k), dtype=np.int64)
    idx = {c: i for i, c in enumerate(classes)}
    for ai, pi in zip(a.tolist(), p.tolist()):
        if pi in idx:
            cm[idx[ai], idx[pi]] += 1
    flat = cm.flatten(order="F")
    tn, fp, fn, tp = (int(flat[0]), int(flat[1]), int(flat[2]), int(flat[3]))
    return ClassificationStatistics(tp, tn, fp, fn)


class LogisticRegressionClassifier:
    """IClassifier for train_clf=logreg (LogisticRegressionClassifier.java), GPU-resident."""

    def __init__(self, context: Optional[Context] = None):
        self._ctx = context
        self.fe = None
        self.config: Dict[str, str] = {}
        self.weights: Optional[np.ndarray] = None
        self.iterations_run = 0
        # Spark partitions of the training RDD (mini-batch sampling only); None = local[*]
        self.num_partitions: Optional[int] = None

    @property
    def context(self) -> Context:
        if self._ctx is None:
            self._ctx = Context(0)
        return self._ctx

    def setFeatureExtraction(self, fe) -> None:
        self.fe = fe

    def getFeatureExtraction(self):
        return self.fe

    def setConfig(self, config: Dict[str, str]) -> None:
        self.config = dict(config)

    def _features(self, epochs):
        if self.fe is None:
            raise ValueError("no feature extraction set")
        ep = np.ascontiguousarray(np.asarray(epochs, dtype=np.float64))
        return self.fe.extractFeaturesBatch(ep)

    def train(self, epochs, targets: Sequence[float], fe) -> None:
        """:85-114 -- the config_* keys select the static train(...) (regParam 0.0), otherwise
        the default LogisticRegressionWithSGD().run (regParam 0.01)."""
        self.fe = fe
        X = self._features(epochs)
        y = np.asarray(targets, dtype=np.float64)
        c = self.config
        if all(k in c for k in ("config_num_iterations", "config_step_size",
                                "config_mini_batch_fraction")):
            self.weights, self.iterations_run = sgd_train(
                self.context, X, y, num_iterations=int(c["config_num_iterations"]),
                step_size=float(c["config_step_size"]), reg_param=0.0,
                mini_batch_fraction=float(c["config_mini_batch_fraction"]),
                num_partitions=self.num_partitions)
        else:
            self.weights, self.iterations_run = sgd_train(
                self.context, X, y, DEFAULT_NUM_ITERATIONS, DEFAULT_STEP_SIZE, DEFAULT_REG_PARAM,
                DEFAULT_MINI_BATCH_FRACTION)

    def predict(self, features) -> np.ndarray:
        if self.weights is None:
            raise RuntimeError("The classifier has not been trained")  # IllegalStateException
        return predict(self.context, features, self.weights)

    def test(self, epochs, targets: Sequence[float]) -> ClassificationStatistics:
        if self.weights is None:
            raise RuntimeError("The classifier has not been trained")
        pred = self.predict(self._features(epochs))
        return reference_statistics(pred, targets)


class SVMClassifier(LogisticRegressionClassifier):
    """IClassifier for train_clf=svm (SVMClassifier.java), GPU-resident: the same flow as
    LogisticRegressionClassifier with SVMWithSGD and SVMModel.predict."""

    def train(self, epochs, targets: Sequence[float], fe) -> None:
        """:83-111 -- with config_num_iterations / config_step_size / config_reg_param /
        config_mini_batch_fraction all set, the static SVMWithSGD.train(rdd, iterations, step,
        regParam, fraction); otherwise new SVMWithSGD().run (step 1.0, 100 iterations,
        regParam 0.01, fraction 1.0)."""
        self.fe = fe
        X = self._features(epochs)
        y = np.asarray(targets, dtype=np.float64)
        c = self.config
        if all(k in c for k in ("config_num_iterations", "config_step_size", "config_reg_param",
                                "config_mini_batch_fraction")):
            self.weights, self.iterations_run = svm_sgd_train(
                self.context, X, y, num_iterations=int(c["config_num_iterations"]),
                step_size=float(c["config_step_size"]), reg_param=float(c["config_reg_param"]),
                mini_batch_fraction=float(c["config_mini_batch_fraction"]))
        else:
            self.weights, self.iterations_run = svm_sgd_train(
                self.context, X, y, DEFAULT_NUM_ITERATIONS, DEFAULT_STEP_SIZE, DEFAULT_REG_PARAM,
                DEFAULT_MINI_BATCH_FRACTION)

    def predict(self, features) -> np.ndarray:
        if self.weights is None:
            raise RuntimeError("The classifier has not been trained")  # IllegalStateException
        return svm_predict(self.context, features, self.weights)


__all__ = ["ClassificationStatistics", "LogisticRegressionClassifier", "SVMClassifier", "predict",
           "reference_statistics", "sgd_train", "spark_sample", "svm_predict", "svm_sgd_train", "EegfxError"]
