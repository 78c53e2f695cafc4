"""MLP / RBM parity with the reference (sklearn 1.x implements the same
algorithms: reference ``neural_network/_multilayer_perceptron.py``,
``_rbm.py``)."""
import pickle
import warnings

import numpy as np
import pytest
import scipy.sparse as sp

from sq_learn_amd import neural_network as Q

S = pytest.importorskip("sklearn.neural_network")


@pytest.fixture(scope="module")
def digits():
    from sklearn.datasets import load_digits
    X, y = load_digits(return_X_y=True)
    return X[:300] / 16, y[:300]


@pytest.mark.parametrize("solver", ["adam", "sgd", "lbfgs"])
@pytest.mark.parametrize("act", ["relu", "tanh", "logistic", "identity"])
def test_mlp_classifier_parity(digits, solver, act):
    X, y = digits
    kw = dict(hidden_layer_sizes=(12, 8), solver=solver, activation=act, max_iter=15,
              random_state=0)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a = S.MLPClassifier(**kw).fit(X, y)
        b = Q.MLPClassifier(**kw).fit(X, y)
    for u, v in zip(a.coefs_, b.coefs_):
        np.testing.assert_allclose(u, v, atol=1e-9)
    assert a.n_iter_ == b.n_iter_
    np.testing.assert_allclose(a.predict_proba(X), b.predict_proba(X), atol=1e-9)
    np.testing.assert_array_equal(a.predict(X), b.predict(X))


def test_mlp_binary_early_stopping_and_pickle(digits):
    X, y = digits
    kw = dict(hidden_layer_sizes=(10,), max_iter=40, random_state=1, early_stopping=True)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a = S.MLPClassifier(**kw).fit(X, y > 4)
        b = Q.MLPClassifier(**kw).fit(X, y > 4)
    assert a.n_iter_ == b.n_iter_
    np.testing.assert_allclose(a.validation_scores_, b.validation_scores_)
    np.testing.assert_allclose(a.predict_proba(X), b.predict_proba(X), atol=1e-12)
    c = pickle.loads(pickle.dumps(b))
    np.testing.assert_allclose(c.predict_proba(X), b.predict_proba(X))


@pytest.mark.parametrize("solver", ["adam", "sgd", "lbfgs"])
@pytest.mark.parametrize("lr", ["constant", "invscaling", "adaptive"])
def test_mlp_regressor_parity(solver, lr):
    from sklearn.datasets import make_regression
    X, y = make_regression(200, 6, n_targets=2, random_state=0)
    y /= 100
    kw = dict(hidden_layer_sizes=(16,), solver=solver, max_iter=25, random_state=0,
              learning_rate=lr, batch_size=32)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a = S.MLPRegressor(**kw).fit(X, y)
        b = Q.MLPRegressor(**kw).fit(X, y)
    np.testing.assert_allclose(a.predict(X), b.predict(X), atol=1e-9)
    if solver != "lbfgs":
        np.testing.assert_allclose(a.loss_curve_, b.loss_curve_, rtol=1e-10)


def test_mlp_partial_fit_and_errors(digits):
    X, y = digits
    a, b = S.MLPClassifier((10,), random_state=0), Q.MLPClassifier((10,), random_state=0)
    for _ in range(3):
        a.partial_fit(X[:100], y[:100], classes=np.arange(10))
        b.partial_fit(X[:100], y[:100], classes=np.arange(10))
    np.testing.assert_allclose(a.predict_proba(X), b.predict_proba(X), atol=1e-12)
    with pytest.raises(AttributeError):
        Q.MLPClassifier(solver="lbfgs").partial_fit
        Q.MLPClassifier(solver="lbfgs").partial_fit(X, y, classes=np.arange(10))
    with pytest.raises(ValueError):
        Q.MLPClassifier(hidden_layer_sizes=(0,)).fit(X, y)
    with pytest.raises(ValueError):
        Q.MLPClassifier(max_iter=0).fit(X, y)
    with pytest.raises(ValueError):
        b.predict(X[:, :5])


def test_rbm_parity():
    from sklearn.datasets import load_digits
    X = (load_digits().data[:200] > 8).astype(float)
    for Xin in (X, sp.csr_matrix(X)):
        a = S.BernoulliRBM(12, n_iter=4, random_state=0).fit(Xin)
        b = Q.BernoulliRBM(12, n_iter=4, random_state=0).fit(Xin)
        np.testing.assert_allclose(a.components_, b.components_, atol=1e-12)
        np.testing.assert_allclose(a.transform(Xin), b.transform(Xin), atol=1e-12)
        np.testing.assert_allclose(a.score_samples(Xin), b.score_samples(Xin), atol=1e-10)
    np.testing.assert_array_equal(a.gibbs(X[:5]), b.gibbs(X[:5]))
    a, b = S.BernoulliRBM(8, random_state=3), Q.BernoulliRBM(8, random_state=3)
    for i in range(3):
        a.partial_fit(X[i * 20:(i + 1) * 20])
        b.partial_fit(X[i * 20:(i + 1) * 20])
    np.testing.assert_allclose(a.components_, b.components_, atol=1e-12)
