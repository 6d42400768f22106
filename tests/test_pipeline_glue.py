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


def test_mllib_restatement_basics():
    import numpy as np
    from oracle import mllib_logreg as ref
    X = np.array([[1.0, 0.0], [0.0, 1.0], [1.0, 1.0]])
    y = np.array([1.0, 0.0, 1.0])
    w, it = ref.sgd_train(X, y, 1, 1.0, 0.0)
    # one step from w = 0: multiplier = 0.5 - y; gradient = mean(mult * x)
    g = ((0.5 - y)[:, None] * X).mean(axis=0)
    assert it == 1 and np.allclose(w, -g, rtol=0, atol=1e-16)
