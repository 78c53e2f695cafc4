"""Reference public helper functions: ``sklearn.utils`` array utilities,
``preprocessing.scale`` / ``minmax_scale``, ``svm.l1_min_c``,
``metrics.pairwise.nan_euclidean_distances`` and the metrics sub-packages."""
import numpy as np
import pytest

import sq_learn_amd.preprocessing as P
import sq_learn_amd.svm as SV
import sq_learn_amd.utils as U
from sq_learn_amd.metrics.pairwise import nan_euclidean_distances

sk = pytest.importorskip("sklearn")


def test_resample_shuffle_parity():
    import sklearn.utils as S
    X = np.arange(40).reshape(20, 2)
    y = np.arange(20) % 3
    for kw in [{}, {"replace": False, "n_samples": 7}, {"stratify": y, "n_samples": 9}]:
        for a, b in zip(S.resample(X, y, random_state=0, **kw),
                        U.resample(X, y, random_state=0, **kw)):
            np.testing.assert_array_equal(a, b)
    for a, b in zip(S.shuffle(X, y, random_state=1), U.shuffle(X, y, random_state=1)):
        np.testing.assert_array_equal(a, b)
    with pytest.raises(ValueError):
        U.resample(X, replace=False, n_samples=30)


def test_scale_minmax_l1minc():
    import sklearn.preprocessing as SP
    import sklearn.svm as SS
    X = np.random.RandomState(0).rand(20, 4) * 5
    y = (X[:, 0] > 2).astype(int)
    for ax in (0, 1):
        np.testing.assert_allclose(P.scale(X, axis=ax), SP.scale(X, axis=ax))
        np.testing.assert_allclose(P.minmax_scale(X, (-1, 2), axis=ax),
                                   SP.minmax_scale(X, (-1, 2), axis=ax))
    np.testing.assert_allclose(P.scale(X, with_mean=False), SP.scale(X, with_mean=False))
    for kw in [{}, {"loss": "log", "fit_intercept": False}]:
        assert SV.l1_min_c(X, y, **kw) == pytest.approx(SS.l1_min_c(X, y, **kw))
    with pytest.raises(ValueError):
        SV.l1_min_c(X, y, loss="hinge")


def test_nan_euclidean_and_metric_packages():
    import sklearn.metrics.pairwise as SMP

    import sq_learn_amd.metrics as M
    rng = np.random.RandomState(0)
    X = rng.rand(6, 4)
    X[1, 2] = np.nan
    X[3, 0] = np.nan
    Y = X[:3].copy()
    Y[0, 1] = np.nan
    np.testing.assert_allclose(SMP.nan_euclidean_distances(X), nan_euclidean_distances(X),
                               atol=1e-7)
    np.testing.assert_allclose(SMP.nan_euclidean_distances(X, Y),
                               nan_euclidean_distances(X, Y), atol=1e-7)
    assert hasattr(M.cluster, "adjusted_rand_score") and hasattr(M.pairwise,
                                                                 "euclidean_distances")


def test_misc_utils():
    X = np.eye(3)
    assert U.check_symmetric(X) is not None
    with pytest.raises(ValueError):
        U.check_symmetric(np.arange(9.0).reshape(3, 3), raise_exception=True)
    with pytest.raises(ValueError):
        U.assert_all_finite(np.array([1.0, np.nan]))
    assert U.safe_sqr(np.array([2.0]))[0] == 4.0
    assert U.murmurhash3_32("abc") == __import__("sklearn.utils", fromlist=["x"]).murmurhash3_32(
        "abc")
    assert len(list(U.gen_batches(10, 3))) == 4
    assert U.is_scalar_nan(float("nan")) and not U.is_scalar_nan("a")
