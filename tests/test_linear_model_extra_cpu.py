"""LARS/OMP, robust regressors, GLMs, quantile, multi-task and
LogisticRegressionCV against scikit-learn (reference
sklearn/linear_model).  The reference's Lars family defaults to
normalize=True (sklearn>=1.2 removed it), so estimator comparisons pass
normalize=False explicitly; LassoLarsIC's criterion changed in sklearn 1.1
(parity unpinned: checked for a sensible fit)."""
import warnings

import numpy as np
import pytest

pytest.importorskip("sklearn")
import sklearn.linear_model as L  # noqa: E402
from sklearn.datasets import make_classification, make_regression  # noqa: E402

import sq_learn_amd.linear_model as M  # noqa: E402

X, y = make_regression(80, 12, n_informative=5, noise=2, random_state=0)


@pytest.fixture(autouse=True)
def _quiet():
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        yield


@pytest.mark.parametrize("method,positive", [("lar", False), ("lasso", False), ("lasso", True)])
def test_lars_path(method, positive):
    a = L.lars_path(X, y, method=method, positive=positive)
    b = M.lars_path(X, y, method=method, positive=positive)
    np.testing.assert_allclose(b[0], a[0], atol=1e-10)
    np.testing.assert_allclose(b[2], a[2], atol=1e-9)
    assert list(a[1]) == list(b[1])


@pytest.mark.parametrize("cls,kw", [
    ("Lars", dict(n_nonzero_coefs=5, normalize=False)), ("LassoLars", dict(alpha=0.5, normalize=False)),
    ("LassoLars", dict(alpha=0.1, positive=True, normalize=False)),
    ("LarsCV", dict(normalize=False)), ("LassoLarsCV", dict(normalize=False)),
    ("OrthogonalMatchingPursuit", dict(normalize=False)),
    ("OrthogonalMatchingPursuit", dict(n_nonzero_coefs=4, normalize=False)),
    ("OrthogonalMatchingPursuit", dict(tol=50.0, normalize=False)),
    ("OrthogonalMatchingPursuitCV", dict(normalize=False)), ("HuberRegressor", {}),
    ("TheilSenRegressor", dict(random_state=0, max_subpopulation=200)),
    ("RANSACRegressor", dict(random_state=0)), ("QuantileRegressor", dict(alpha=0.1, solver="highs"))])
def test_regressors(cls, kw):
    if "normalize" in kw:
        kw = dict(kw)
        import inspect
        if "normalize" not in inspect.signature(getattr(L, cls)).parameters:
            kw_sk = {k: v for k, v in kw.items() if k != "normalize"}
        else:
            kw_sk = kw
    else:
        kw_sk = kw
    a = getattr(L, cls)(**kw_sk).fit(X, y)
    b = getattr(M, cls)(**kw).fit(X, y)
    np.testing.assert_allclose(b.predict(X), a.predict(X), atol=1e-8)


def test_lasso_lars_ic_and_glms():
    m = M.LassoLarsIC().fit(X, y)
    assert m.score(X, y) > 0.95
    rng = np.random.RandomState(0)
    yp = rng.poisson(np.exp(X[:, :2] @ [0.1, 0.2] / 10 + 1))
    yg = np.exp(X[:, 0] / 50) + 0.1
    for cls, yy, kw in [("PoissonRegressor", yp, {}), ("GammaRegressor", yg, {}),
                        ("TweedieRegressor", yg, dict(power=1.5)),
                        ("TweedieRegressor", y, dict(power=0, alpha=0.1))]:
        a = getattr(L, cls)(**kw).fit(X, yy)
        b = getattr(M, cls)(**kw).fit(X, yy)
        np.testing.assert_allclose(b.coef_, a.coef_, atol=1e-6)
        np.testing.assert_allclose(b.score(X, yy), a.score(X, yy), rtol=1e-6)


@pytest.mark.parametrize("cls,kw", [("MultiTaskLasso", dict(alpha=1.0)),
                                    ("MultiTaskElasticNet", dict(alpha=1.0)),
                                    ("MultiTaskLasso", dict(alpha=1.0, selection="random", random_state=0)),
                                    ("MultiTaskLassoCV", dict(cv=3)),
                                    ("MultiTaskElasticNetCV", dict(cv=3))])
def test_multitask(cls, kw):
    Y = np.c_[y, y * 0.5 + X[:, 0]]
    a = getattr(L, cls)(**kw).fit(X, Y)
    b = getattr(M, cls)(**kw).fit(X, Y)
    np.testing.assert_allclose(b.coef_, a.coef_, atol=1e-8)


def test_logistic_regression_cv():
    Xc, yc = make_classification(200, 6, random_state=0)
    a = L.LogisticRegressionCV(cv=3).fit(Xc, yc)
    b = M.LogisticRegressionCV(cv=3).fit(Xc, yc)
    np.testing.assert_allclose(b.C_, a.C_)
    np.testing.assert_allclose(b.coef_, a.coef_, atol=1e-3)


def test_enet_path_multi_output_matches_reference():
    """Multi-output enet / lasso paths (reference _coordinate_descent.py:
    452-498): the multi-task coordinate descent along the warm-started
    alphas, against scikit-learn's Cython solver."""
    import warnings
    import numpy as np
    import pytest
    sk = pytest.importorskip("sklearn.linear_model")
    from sq_learn_amd.models.linear_model._coordinate_descent import enet_path, lasso_path
    rs = np.random.RandomState(0)
    X = rs.randn(60, 8)
    Y = X @ rs.randn(8, 3) + 0.1 * rs.randn(60, 3)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a1, c1, g1 = sk.enet_path(X, Y, l1_ratio=0.7, n_alphas=10)
        a2, c2, g2 = enet_path(X, Y, l1_ratio=0.7, n_alphas=10)
        _, l1c, _ = sk.lasso_path(X, Y, n_alphas=5)
        _, l2c, _ = lasso_path(X, Y, n_alphas=5)
    assert c2.shape == (3, 8, 10)
    np.testing.assert_allclose(a2, a1, rtol=1e-12)
    np.testing.assert_allclose(c2, c1, atol=1e-10)
    np.testing.assert_allclose(g2, g1, atol=1e-10)
    np.testing.assert_allclose(l2c, l1c, atol=1e-10)
    with pytest.raises(ValueError, match="positive"):
        enet_path(X, Y, positive=True)


def test_ridgecv_loo_with_scorer():
    """RidgeCV's built-in LOO with a user scorer (reference _ridge.py:
    1518-1562): the scorer sees the leave-one-out predictions (centred
    space, raveled over targets unless alpha_per_target); pinned against a
    brute-force leave-one-out refit and, per target, against scikit-learn."""
    import warnings
    import numpy as np
    import pytest
    skl = pytest.importorskip("sklearn.linear_model")
    from sklearn.metrics import r2_score
    from sq_learn_amd.models.linear_model import RidgeCV
    from sq_learn_amd.models.linear_model import Ridge
    rs = np.random.RandomState(0)
    X = rs.randn(40, 5)
    y = X @ rs.randn(5) + 0.3 * rs.randn(40)
    Y = np.c_[y, 2 * y + rs.randn(40)]
    alphas = [0.01, 0.1, 1.0, 10.0]
    for al in alphas:
        got = RidgeCV(alphas=[al], scoring="r2").fit(X, Y).best_score_
        P = np.empty_like(Y)
        for i in range(len(X)):
            m = np.arange(len(X)) != i
            P[i] = Ridge(alpha=al).fit(X[m], Y[m]).predict(X[i:i + 1])[0]
        Yc = Y - Y.mean(0)
        want = r2_score(Yc.ravel(), (P - Y.mean(0)).ravel())
        assert abs(got - want) < 1e-9, (al, got, want)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a = skl.RidgeCV(alphas=alphas, scoring="neg_mean_absolute_error", alpha_per_target=True).fit(X, Y)
    b = RidgeCV(alphas=alphas, scoring="neg_mean_absolute_error", alpha_per_target=True).fit(X, Y)
    np.testing.assert_allclose(b.alpha_, a.alpha_)
    np.testing.assert_allclose(b.best_score_, a.best_score_, rtol=1e-10)
    np.testing.assert_allclose(b.coef_, a.coef_, atol=1e-9)
    c = RidgeCV(alphas=alphas, scoring="r2", store_cv_values=True).fit(X, y)
    assert c.cv_values_.shape == (40, 4)
