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
