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

Spark sums the per-row gradients per partition and combines partitions in a tree, so its
floating-point order depends on the partitioning (local[*] = the host's core count): parity is a
tolerance on the weights, never bit equality.  Rows are summed here in index order (one
partition).  Parity unpinned: no fixture of the reference holds trained weights or statistics
(ClassifierTest.java's accuracy assertion is commented out).
"""
from __future__ import annotations

import math

import numpy as np

DEFAULT_STEP = 1.0
DEFAULT_ITERS = 100
DEFAULT_REG = 0.01
DEFAULT_FRACTION = 1.0
CONVERGENCE_TOL = 0.001


def sgd_train(X, y, num_iterations=DEFAULT_ITERS, step_size=DEFAULT_STEP, reg_param=0.0,
              convergence_tol=CONVERGENCE_TOL, initial=None, gradient="logistic"):
    """Returns (weights, iterations_run).  gradient: "logistic" (LogisticRegressionWithSGD) or
    "hinge" (SVMWithSGD)."""
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
        if gradient == "hinge":
            s_lab = 2.0 * y - 1.0
            mult = np.where(1.0 > s_lab * (X @ w), -s_lab, 0.0)
        else:
            margin = -(X @ w)
            mult = 1.0 / (1.0 + np.exp(margin)) - y
        grad = (mult[:, None] * X).sum(axis=0) / n
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
