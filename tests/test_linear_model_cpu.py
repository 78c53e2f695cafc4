"""Linear models vs the installed upstream scikit-learn (same estimators as
the reference fork's untouched ``sklearn.linear_model``)."""
import warnings

import numpy as np
import pytest
import sklearn.linear_model as S
from sklearn.datasets import make_classification

import sq_learn_amd.linear_model as L


@pytest.fixture(scope="module")
def reg():
    rs = np.random.RandomState(0)
    X = rs.randn(80, 10)
    w = rs.randn(10) * (rs.rand(10) > 0.5)
    return X, X @ w + 0.1 * rs.randn(80) + 3, rs.rand(80) + 0.5


CASES = [("LinearRegression", {}), ("Ridge", {"alpha": 0.7}),
         ("Ridge", {"alpha": 0.7, "solver": "svd"}), ("Lasso", {"alpha": 0.05}),
         ("ElasticNet", {"alpha": 0.05, "l1_ratio": 0.3}), ("Lasso", {"alpha": 0.05, "precompute": True}),
         ("ElasticNet", {"alpha": 0.1, "selection": "random", "random_state": 3}),
         ("Lasso", {"alpha": 0.02, "positive": True}), ("LinearRegression", {"positive": True}),
         ("Ridge", {"alpha": 2.0, "fit_intercept": False})]


@pytest.mark.parametrize("name,kw", CASES)
@pytest.mark.parametrize("weighted", [False, True])
def test_regressors_match(reg, name, kw, weighted):
    X, y, sw = reg
    s = sw if weighted else None
    a = getattr(L, name)(**kw).fit(X, y, sample_weight=s)
    b = getattr(S, name)(**kw).fit(X, y, sample_weight=s)
    np.testing.assert_allclose(a.coef_, b.coef_, atol=1e-10)
    np.testing.assert_allclose(a.intercept_, b.intercept_, atol=1e-10)
    np.testing.assert_allclose(a.predict(X), b.predict(X), atol=1e-9)
    if hasattr(b, "n_iter_") and b.n_iter_ is not None:
        assert a.n_iter_ == b.n_iter_           # same CD iterations (incl. random selection)


def test_multi_target_and_paths(reg):
    X, y, _ = reg
    Y = np.c_[y, -2 * y + 1]
    for name in ("Ridge", "Lasso", "LinearRegression"):
        a, b = getattr(L, name)().fit(X, Y), getattr(S, name)().fit(X, Y)
        np.testing.assert_allclose(a.coef_, b.coef_, atol=1e-10)
    Xc, yc = X - X.mean(0), y - y.mean()
    for fa, fb, kw in ((L.lasso_path, S.lasso_path, {}), (L.enet_path, S.enet_path, {"l1_ratio": 0.4})):
        al, c1, g1 = fa(Xc, yc, n_alphas=15, **kw)
        bl, c2, g2 = fb(Xc, yc, n_alphas=15, **kw)
        np.testing.assert_allclose(al, bl, rtol=1e-12)
        np.testing.assert_allclose(c1, c2, atol=1e-10)


def test_cv_estimators(reg):
    X, y, _ = reg
    a = L.RidgeCV(alphas=[0.01, 0.1, 1, 10]).fit(X, y)
    b = S.RidgeCV(alphas=[0.01, 0.1, 1, 10]).fit(X, y)
    assert a.alpha_ == b.alpha_
    np.testing.assert_allclose(a.best_score_, b.best_score_, rtol=1e-8)
    np.testing.assert_allclose(a.coef_, b.coef_, atol=1e-8)
    a, b = L.LassoCV(cv=4).fit(X, y), S.LassoCV(cv=4).fit(X, y)
    np.testing.assert_allclose(a.alpha_, b.alpha_, rtol=1e-12)
    np.testing.assert_allclose(a.mse_path_, b.mse_path_, rtol=1e-8)
    np.testing.assert_allclose(a.coef_, b.coef_, atol=1e-10)
    a = L.ElasticNetCV(cv=3, l1_ratio=[0.2, 0.8]).fit(X, y)
    b = S.ElasticNetCV(cv=3, l1_ratio=[0.2, 0.8]).fit(X, y)
    assert a.l1_ratio_ == b.l1_ratio_
    np.testing.assert_allclose(a.alpha_, b.alpha_, rtol=1e-10)


def test_ridge_classifier(reg):
    X, y, _ = reg
    yc = (y > 3).astype(int) + (y > 5)
    for cls in ("RidgeClassifier", "RidgeClassifierCV"):
        a, b = getattr(L, cls)().fit(X, yc), getattr(S, cls)().fit(X, yc)
        np.testing.assert_allclose(a.coef_, b.coef_, atol=1e-8)
        np.testing.assert_array_equal(a.predict(X), b.predict(X))


@pytest.mark.parametrize("n_classes", [2, 3])
@pytest.mark.parametrize("kw", [{}, {"C": 0.1}, {"multi_class": "ovr"}, {"penalty": None},
                                {"class_weight": "balanced"}, {"fit_intercept": False},
                                {"penalty": "l1", "solver": "saga", "C": 0.5},
                                {"penalty": "elasticnet", "l1_ratio": 0.5, "solver": "saga"}])
def test_logistic_regression(n_classes, kw):
    X, y = make_classification(300, 8, n_informative=5, n_classes=n_classes, random_state=0)
    kw = dict(kw, tol=1e-10, max_iter=20000)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a, b = L.LogisticRegression(**kw).fit(X, y), S.LogisticRegression(**kw).fit(X, y)
    # same optimum (the solvers' stopping points differ within ~1e-4)
    np.testing.assert_allclose(a.coef_, b.coef_, atol=5e-4)
    np.testing.assert_allclose(a.predict_proba(X), b.predict_proba(X), atol=5e-4)
    assert (a.predict(X) == b.predict(X)).mean() > 0.99
