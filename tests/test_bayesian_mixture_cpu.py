"""Variational Bayesian Gaussian mixture (reference
``mixture/_bayesian_mixture.py``)."""
import pickle
import warnings

import numpy as np
import pytest

from sq_learn_amd.mixture import BayesianGaussianMixture as Q

SM = pytest.importorskip("sklearn.mixture")


@pytest.fixture(scope="module")
def X():
    from sklearn.datasets import make_blobs
    return make_blobs(300, 3, centers=4, random_state=0)[0]


@pytest.mark.parametrize("ct", ["full", "tied", "diag", "spherical"])
@pytest.mark.parametrize("wt", ["dirichlet_process", "dirichlet_distribution"])
def test_parity(X, ct, wt):
    kw = dict(n_components=6, covariance_type=ct, weight_concentration_prior_type=wt,
              init_params="random", random_state=0, max_iter=200)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a = SM.BayesianGaussianMixture(**kw).fit(X)
        b = Q(**kw).fit(X)
    assert a.n_iter_ == b.n_iter_
    np.testing.assert_allclose(a.weights_, b.weights_, atol=1e-10)
    np.testing.assert_allclose(a.means_, b.means_, atol=1e-10)
    np.testing.assert_allclose(a.precisions_, b.precisions_, rtol=1e-8, atol=1e-10)
    assert a.lower_bound_ == pytest.approx(b.lower_bound_, rel=1e-10)
    np.testing.assert_allclose(a.score_samples(X), b.score_samples(X), atol=1e-9)
    np.testing.assert_array_equal(a.predict(X), b.predict(X))
    c = pickle.loads(pickle.dumps(b))
    np.testing.assert_allclose(c.predict_proba(X), b.predict_proba(X))


def test_priors_and_errors(X):
    b = Q(n_components=3, weight_concentration_prior=0.01, mean_precision_prior=0.5,
          degrees_of_freedom_prior=5, covariance_prior=np.eye(3), mean_prior=np.zeros(3),
          random_state=0).fit(X)
    assert b.weights_.shape == (3,) and np.isclose(b.weights_.sum(), 1)
    for bad in (dict(weight_concentration_prior=-1.0), dict(mean_precision_prior=0.0),
                dict(degrees_of_freedom_prior=1.0), dict(weight_concentration_prior_type="x"),
                dict(covariance_type="diag", covariance_prior=-np.ones(3))):
        with pytest.raises(ValueError):
            Q(n_components=2, **bad).fit(X)
