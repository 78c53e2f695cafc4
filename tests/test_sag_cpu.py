"""SAG / SAGA (reference linear_model/_sag.py:89, _sag_fast.pyx.tp; host
core csrc/host/sag.cpp) against scikit-learn's Cython solvers: same sample
stream (make_dataset's seed draw + xorshift), step size and stopping rule,
so epochs and coefficients agree to rounding."""
import warnings

import numpy as np
import pytest

sk = pytest.importorskip("sklearn")
from sklearn import linear_model as sklm  # noqa: E402
from sklearn.datasets import make_classification, make_regression  # noqa: E402
from sklearn.preprocessing import StandardScaler  # noqa: E402

from sq_learn_amd.models.linear_model import LogisticRegression, Ridge  # noqa: E402
from sq_learn_amd.models.linear_model._ridge import ridge_regression  # noqa: E402
from sq_learn_amd.models.linear_model._sag import get_auto_step_size, sag_solver  # noqa: E402


@pytest.mark.parametrize("K", [2, 3])
@pytest.mark.parametrize("kw", [dict(solver="sag"), dict(solver="saga"),
                                dict(solver="saga", penalty="l1", C=0.5),
                                dict(solver="saga", penalty="elasticnet", l1_ratio=0.3),
                                dict(solver="sag", multi_class="ovr", class_weight={0: 2.0})])
def test_logistic_sag_matches_reference(K, kw):
    X, y = make_classification(300, 6, n_informative=4, n_classes=K, random_state=0)
    X = StandardScaler().fit_transform(X)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a = sklm.LogisticRegression(tol=1e-8, max_iter=5000, random_state=0, **kw).fit(X, y)
        b = LogisticRegression(tol=1e-8, max_iter=5000, random_state=0, **kw).fit(X, y)
    np.testing.assert_allclose(b.coef_, a.coef_, atol=1e-10)
    np.testing.assert_allclose(b.intercept_, a.intercept_, atol=1e-10)
    np.testing.assert_array_equal(b.n_iter_, a.n_iter_)


@pytest.mark.parametrize("kw", [dict(solver="sag"), dict(solver="saga", alpha=3.0),
                                dict(solver="sag", fit_intercept=False)])
def test_ridge_sag_matches_reference(kw):
    X, y = make_regression(300, 5, n_targets=2, noise=1.0, random_state=0)
    sw = np.random.RandomState(0).rand(300) + 0.5
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a = sklm.Ridge(tol=1e-8, random_state=0, **kw).fit(X, y, sample_weight=sw)
        b = Ridge(tol=1e-8, random_state=0, **kw).fit(X, y, sample_weight=sw)
    np.testing.assert_allclose(b.coef_, a.coef_, atol=1e-9)
    np.testing.assert_allclose(b.intercept_, a.intercept_, atol=1e-9)
    np.testing.assert_array_equal(b.n_iter_, a.n_iter_)


def test_ridge_regression_sag_fits_intercept():
    X, y = make_regression(300, 5, noise=1.0, random_state=1)
    a = sklm.ridge_regression(X, y, 1.0, solver="sag", tol=1e-8, random_state=0,
                              return_intercept=True, return_n_iter=True)
    b = ridge_regression(X, y, 1.0, solver="sag", tol=1e-8, random_state=0,
                         return_intercept=True, return_n_iter=True)
    np.testing.assert_allclose(b[0], a[0], atol=1e-9)
    np.testing.assert_array_equal(b[1], a[1])
    assert abs(b[2] - a[2]) < 1e-9
    with pytest.raises(ValueError, match="only 'sag'"):
        ridge_regression(X, y, 1.0, solver="saga", return_intercept=True)


def test_sag_solver_api():
    X, y = make_regression(100, 3, random_state=0)
    assert get_auto_step_size(4.0, 0.1, "squared", True) == pytest.approx(1 / 5.1)
    assert get_auto_step_size(4.0, 0.1, "log", False, n_samples=10, is_saga=True) == \
        pytest.approx(1 / (2 * 1.1 + 1.1))
    with pytest.raises(ValueError, match="Unknown loss"):
        get_auto_step_size(1.0, 0.1, "hinge", False)
    coef, n_iter, mem = sag_solver(X, y, loss="squared", alpha=1.0, tol=1e-10, max_iter=2,
                                   random_state=0)
    assert n_iter == 2 and coef.shape == (3,) and mem["coef"].shape == (3, 1)
    with pytest.raises(ValueError, match="overflow"):
        sag_solver(X, y * 1e308, loss="squared", alpha=1.0, max_iter=5, random_state=0)


@pytest.mark.parametrize("solver", ["sag", "saga"])
def test_sparse_fit_intercept_matches_reference(solver):
    # sparse input: the reference damps intercept updates by
    # SPARSE_INTERCEPT_DECAY = 0.01 (make_dataset, linear_model/_base.py:206)
    import scipy.sparse as sparse
    X, y = make_classification(300, 6, n_informative=4, random_state=1)
    X = StandardScaler().fit_transform(X)
    X[np.abs(X) < 0.5] = 0.0
    Xs = sparse.csr_matrix(X)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a = sklm.LogisticRegression(solver=solver, tol=1e-8, max_iter=5000, random_state=0).fit(Xs, y)
        b = LogisticRegression(solver=solver, tol=1e-8, max_iter=5000, random_state=0).fit(Xs, y)
    np.testing.assert_allclose(b.coef_, a.coef_, atol=1e-8)
    np.testing.assert_allclose(b.intercept_, a.intercept_, atol=1e-8)
    np.testing.assert_array_equal(b.n_iter_, a.n_iter_)
