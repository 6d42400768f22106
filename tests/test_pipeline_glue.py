"""Classifier-flow glue: java.util.Random + Collections.shuffle + 70/30 split
exactly as PipelineBuilder.java:177-187."""
from eeg_dataanalysispackage_amd.pipeline import (JavaRandom, java_shuffle_permutation,
                                                  labeled_points, reference_split)


def test_java_random_known_values():
    # new Random(1).nextInt(): the JDK's documented LCG; first values of seed 1
    r = JavaRandom(1)
    assert [r._next(32) for _ in range(3)] == [-1155869325, 431529176, 1761283695]
    r = JavaRandom(42)
    assert [r.nextInt(10) for _ in range(5)] == [0, 3, 8, 4, 0]


def test_info_train_split_matches_survey():
    # for the 11 infoTrain epochs the permutation is train [0,7,9,2,5,10,6],
    # test [3,1,8,4]
    tr, te = reference_split(11)
    assert tr == [0, 7, 9, 2, 5, 10, 6]
    assert te == [3, 1, 8, 4]


def test_permutation_is_a_permutation():
    for n in (0, 1, 2, 5, 6, 27, 1000):
        p = java_shuffle_permutation(n)
        assert sorted(p) == list(range(n))
    assert len(reference_split(27)[0]) == int(27 * 0.7)


def test_labeled_points():
    pts = labeled_points([[1.0, 2.0], [3.0, 4.0]], [1.0, 0.0])
    assert pts[0][0] == 1.0 and list(pts[1][1]) == [3.0, 4.0]


def test_reference_statistics_mapping():
    """LogisticRegressionClassifier.test reads MulticlassMetrics' column-major confusion matrix as
    tn, fp, fn, tp: its "fp" counts actual-1/predicted-0."""
    from eeg_dataanalysispackage_amd.classification import reference_statistics
    from oracle import mllib_logreg as ref
    labels = [0, 0, 0, 1, 1, 1, 1]
    pred = [0, 1, 1, 0, 1, 1, 1]  # actual0: 1x pred0, 2x pred1; actual1: 1x pred0, 3x pred1
    s = reference_statistics(pred, labels)
    assert s.as_tuple() == (3, 1, 1, 2) == ref.reference_statistics(pred, labels)
    assert abs(s.calcAccuracy() - 4 / 7) < 1e-15
    import pytest
    with pytest.raises(IndexError):
        reference_statistics([1, 1], [1, 1])
    # MulticlassMetrics.labels are the actual classes only: a single actual class with mixed
    # predictions is still a 1x1 matrix, and the reference's cm[1] throws
    with pytest.raises(IndexError):
        reference_statistics([0, 1, 1], [0, 0, 0])
    with pytest.raises(IndexError):
        ref.reference_statistics([0, 1, 1], [0, 0, 0])


def test_mllib_restatement_basics():
    import numpy as np
    from oracle import mllib_logreg as ref
    X = np.array([[1.0, 0.0], [0.0, 1.0], [1.0, 1.0]])
    y = np.array([1.0, 0.0, 1.0])
    w, it = ref.sgd_train(X, y, 1, 1.0, 0.0)
    # one step from w = 0: multiplier = 0.5 - y; gradient = mean(mult * x)
    g = ((0.5 - y)[:, None] * X).mean(axis=0)
    assert it == 1 and np.allclose(w, -g, rtol=0, atol=1e-16)


def test_mllib_hinge_restatement_by_hand():
    """HingeGradient + SquaredL2Updater, two steps worked by hand (SVMWithSGD defaults)."""
    import math
    import numpy as np
    from oracle import mllib_logreg as ref
    X = np.array([[1.0, 0.0], [0.0, 1.0], [1.0, 1.0]])
    y = np.array([1.0, 0.0, 1.0])
    s = 2 * y - 1
    # step 1 from w = 0: every row violates (1 > 0), gradient = mean(-s x)
    g1 = (-s[:, None] * X).mean(axis=0)
    w1 = np.zeros(2) * (1 - 1.0 * 0.01) - 1.0 * g1
    w, it = ref.sgd_train(X, y, 1, 1.0, 0.01, gradient="hinge")
    assert it == 1 and np.array_equal(w, w1)
    # step 2: only rows with 1 > s * w1.x contribute, step 1/sqrt(2)
    viol = 1.0 > s * (X @ w1)
    g2 = np.where(viol[:, None], -s[:, None] * X, 0.0).sum(axis=0) / 3
    st = 1.0 / math.sqrt(2)
    w2 = w1 * (1 - st * 0.01) - st * g2
    w, it = ref.sgd_train(X, y, 2, 1.0, 0.01, convergence_tol=0.0, gradient="hinge")
    assert it == 2 and np.allclose(w, w2, rtol=0, atol=1e-15)
    assert np.array_equal(ref.svm_predict(X, w2), (X @ w2 > 0).astype(float))
    assert np.array_equal(ref.svm_predict(X, w2, threshold=None), X @ w2)
