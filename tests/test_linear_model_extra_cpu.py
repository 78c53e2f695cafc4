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
