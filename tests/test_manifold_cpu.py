"""Manifold learners against scikit-learn (reference sklearn/manifold).
LLE (all four methods) and Isomap match to fp precision; t-SNE uses the
exact device gradient (also for method='barnes_hut', where the reference
approximates), so it is compared on KL divergence and trustworthiness;
sklearn>=1.2 changed the MDS stress definition (parity unpinned: metric
SMACOF compared on stress)."""
import warnings

import numpy as np
import pytest

pytest.importorskip("sklearn")
import sklearn.manifold as S  # noqa: E402
from sklearn.datasets import load_digits, make_s_curve  # noqa: E402

import sq_learn_amd.manifold as M  # noqa: E402

X, _ = make_s_curve(300, random_state=0)


@pytest.fixture(autouse=True)
def _quiet():
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        yield


@pytest.mark.parametrize("method", ["standard", "hessian", "modified", "ltsa"])
@pytest.mark.parametrize("solver", ["dense", "arpack"])
def test_lle(method, solver):
    a = S.LocallyLinearEmbedding(n_neighbors=12, method=method, eigen_solver=solver,
                                 random_state=0).fit(X)
    b = M.LocallyLinearEmbedding(n_neighbors=12, method=method, eigen_solver=solver,
                                 random_state=0).fit(X)
    np.testing.assert_allclose(np.abs(b.embedding_), np.abs(a.embedding_), atol=1e-7)
    assert abs(a.reconstruction_error_ - b.reconstruction_error_) < 1e-10


def test_isomap_mds():
    a, b = S.Isomap(n_neighbors=8).fit(X), M.Isomap(n_neighbors=8).fit(X)
    np.testing.assert_allclose(np.abs(b.embedding_), np.abs(a.embedding_), atol=1e-9)
    np.testing.assert_allclose(np.abs(b.transform(X[:5])), np.abs(a.transform(X[:5])), atol=1e-9)
    assert abs(a.reconstruction_error() - b.reconstruction_error()) < 1e-9
    m = M.MDS(random_state=0, n_init=2).fit(X[:100])
    try:
        r = S.MDS(random_state=0, n_init=2, normalized_stress=False).fit(X[:100])
    except TypeError:
        r = S.MDS(random_state=0, n_init=2).fit(X[:100])
    assert abs(m.stress_ - r.stress_) < 0.01 * r.stress_
    nm = M.MDS(random_state=0, n_init=1, metric=False).fit(X[:60])
    assert np.isfinite(nm.stress_) and nm.embedding_.shape == (60, 2)


@pytest.mark.parametrize("method", ["exact", "barnes_hut"])
def test_tsne(method):
    Xd = load_digits(return_X_y=True)[0][:300]
    a = S.TSNE(method=method, init="random", learning_rate=200.0, random_state=0).fit(Xd)
    b = M.TSNE(method=method, init="random", learning_rate=200.0, random_state=0).fit(Xd)
    assert abs(a.kl_divergence_ - b.kl_divergence_) < 0.1 * a.kl_divergence_
    assert M.trustworthiness(Xd, b.embedding_) > S.trustworthiness(Xd, a.embedding_) - 0.01
    assert M.trustworthiness(Xd, a.embedding_) == pytest.approx(S.trustworthiness(Xd, a.embedding_))
