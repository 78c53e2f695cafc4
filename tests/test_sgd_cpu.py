"""Native SGD family (csrc/host/sgd.cpp) against scikit-learn: the loop,
RNG streams and weight-vector algebra follow the reference's
sklearn/linear_model/_sgd_fast.pyx bit for bit, so coefficients must match
exactly (up to fp reassociation in the averaged path).  log loss is
excluded from the exact comparison: sklearn>=1.2 replaced the reference's
Log loss with a different implementation (parity unpinned there; checked
for accuracy only)."""
import warnings

import numpy as np
import pytest
import scipy.sparse as sp

pytest.importorskip("sklearn")
import sklearn.linear_model as L  # noqa: E402
from sklearn.datasets import make_classification, make_regression  # noqa: E402

import sq_learn_amd.linear_model as M  # noqa: E402


@pytest.fixture(autouse=True)
def _quiet():
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        yield


X, y = make_classification(300, 10, n_informative=5, n_classes=3, random_state=0)
Xb, yb = make_classification(300, 10, random_state=1)
Xr, yr = make_regression(300, 10, noise=1, random_state=0)


def _same(a, b, tol=1e-12):
    np.testing.assert_allclose(b.coef_, a.coef_, atol=tol, rtol=0)
    ia = getattr(a, "intercept_", getattr(a, "offset_", None))
    ib = getattr(b, "intercept_", getattr(b, "offset_", None))
    np.testing.assert_allclose(ib, ia, atol=tol, rtol=0)
    assert a.n_iter_ == b.n_iter_


@pytest.mark.parametrize("loss", ["hinge", "modified_huber", "squared_hinge", "perceptron",
                                  "squared_error", "huber", "epsilon_insensitive"])
@pytest.mark.parametrize("penalty", ["l2", "l1", "elasticnet"])
def test_sgd_classifier_losses(loss, penalty):
    for XX, yy in [(X, y), (Xb, yb)]:
        kw = dict(loss=loss, penalty=penalty, random_state=0)
        _same(L.SGDClassifier(**kw).fit(XX, yy), M.SGDClassifier(**kw).fit(XX, yy))


@pytest.mark.parametrize("kw", [dict(average=True), dict(average=10),
                                dict(learning_rate="invscaling", eta0=0.1),
                                dict(learning_rate="adaptive", eta0=0.1),
                                dict(early_stopping=True), dict(class_weight="balanced"),
                                dict(learning_rate="constant", eta0=0.01, shuffle=False)])
def test_sgd_classifier_options(kw):
    for XX, yy in [(X, y), (Xb, yb)]:
        _same(L.SGDClassifier(random_state=0, **kw).fit(XX, yy),
              M.SGDClassifier(random_state=0, **kw).fit(XX, yy), 1e-12)


def test_sgd_sparse_partial_proba():
    _same(L.SGDClassifier(random_state=0).fit(sp.csr_matrix(X), y),
          M.SGDClassifier(random_state=0).fit(sp.csr_matrix(X), y))
    a, b = L.SGDClassifier(random_state=0), M.SGDClassifier(random_state=0)
    for i in range(3):
        sl = slice(i * 100, (i + 1) * 100)
        a.partial_fit(X[sl], y[sl], classes=[0, 1, 2])
        b.partial_fit(X[sl], y[sl], classes=[0, 1, 2])
    _same(a, b)
    a = L.SGDClassifier(loss="modified_huber", random_state=0).fit(X, y)
    b = M.SGDClassifier(loss="modified_huber", random_state=0).fit(X, y)
    np.testing.assert_allclose(b.predict_proba(X), a.predict_proba(X), atol=1e-12)
    lg = M.SGDClassifier(loss="log_loss", random_state=0).fit(Xb, yb)
    assert lg.score(Xb, yb) > 0.8 and np.allclose(lg.predict_proba(Xb).sum(1), 1)


@pytest.mark.parametrize("loss", ["squared_error", "huber", "epsilon_insensitive",
                                  "squared_epsilon_insensitive"])
def test_sgd_regressor(loss):
    for kw in [{}, dict(penalty="elasticnet"), dict(average=True), dict(early_stopping=True),
               dict(learning_rate="adaptive")]:
        _same(L.SGDRegressor(loss=loss, random_state=0, **kw).fit(Xr, yr),
              M.SGDRegressor(loss=loss, random_state=0, **kw).fit(Xr, yr), 1e-10)


def test_perceptron_pa_oneclass():
    _same(L.Perceptron().fit(X, y), M.Perceptron().fit(X, y))
    _same(L.Perceptron(penalty="elasticnet").fit(X, y), M.Perceptron(penalty="elasticnet").fit(X, y))
    for loss in ["hinge", "squared_hinge"]:
        _same(L.PassiveAggressiveClassifier(loss=loss, random_state=0).fit(X, y),
              M.PassiveAggressiveClassifier(loss=loss, random_state=0).fit(X, y))
    for loss in ["epsilon_insensitive", "squared_epsilon_insensitive"]:
        _same(L.PassiveAggressiveRegressor(loss=loss, random_state=0).fit(Xr, yr),
              M.PassiveAggressiveRegressor(loss=loss, random_state=0).fit(Xr, yr))
    for kw in [{}, dict(average=True), dict(learning_rate="constant", eta0=0.01)]:
        a = L.SGDOneClassSVM(random_state=0, **kw).fit(Xr)
        b = M.SGDOneClassSVM(random_state=0, **kw).fit(Xr)
        _same(a, b)
        assert (a.predict(Xr) == b.predict(Xr)).all()
