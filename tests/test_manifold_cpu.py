"""Manifold learners against scikit-learn (reference sklearn/manifold).
LLE (all four methods) and Isomap match to fp precision; t-SNE (exact
device gradient, or the host Barnes-Hut kernel in fp64 where the reference
computes in fp32) is compared on KL divergence and trustworthiness, the
Barnes-Hut gradient against the exact formula (angle 0) and its angle
error;
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


def _exact_bh_reference(Y, P, dof):
    D = ((Y[:, None, :] - Y[None, :, :]) ** 2).sum(-1)
    W = (dof / (dof + D)) ** ((dof + 1) / 2)
    np.fill_diagonal(W, 0.0)
    Z = W.sum()
    Pd = P.toarray()
    g = np.stack([((Pd[i] * W[i])[:, None] * (Y[i] - Y)).sum(0)
                  - ((W[i] ** 2)[:, None] * (Y[i] - Y)).sum(0) / Z for i in range(len(Y))])
    m = Pd > 0
    kl = (Pd[m] * np.log(np.maximum(Pd[m], 2.2e-16) / np.maximum(W[m] / Z, 2.2e-16))).sum()
    return kl, g * 2 * (dof + 1) / dof


@pytest.mark.parametrize("dim,dof", [(2, 1.0), (3, 2.0)])
def test_barnes_hut_gradient_kernel(dim, dof):
    """Host Barnes-Hut kernel (csrc/host/tsne_bh.cpp): angle 0 is the exact
    gradient and KL; angle 0.5 stays within a few percent; duplicate
    points are handled."""
    import scipy.sparse as sp
    from sq_learn_amd.models.manifold._embed import _kl_grad_bh
    rs = np.random.RandomState(0)
    n = 300
    Y = rs.randn(n, dim)
    Y[7] = Y[6]
    Y[8] = Y[6]
    ind = np.array([rs.choice(np.delete(np.arange(n), i), 10, replace=False) for i in range(n)])
    P = sp.csr_matrix((rs.rand(n * 10), ind.ravel(), np.arange(0, n * 10 + 1, 10)), shape=(n, n))
    P = P + P.T
    P = (P / P.sum()).tocsr()
    ke, ge = _exact_bh_reference(Y, P, dof)
    k0, g0 = _kl_grad_bh(Y, P, dof, 0.0)
    assert abs(k0 - ke) < 1e-10 * abs(ke)
    np.testing.assert_allclose(g0, ge, rtol=0, atol=1e-12 * np.abs(ge).max())
    k5, g5 = _kl_grad_bh(Y, P, dof, 0.5)
    assert np.abs(g5 - ge).max() < 0.05 * np.abs(ge).max()
    assert abs(k5 - ke) < 0.05 * ke
    assert _kl_grad_bh(Y, P, dof, 0.5, compute_error=False)[0] is None


def test_tsne_barnes_hut_sparse_scales():
    """method='barnes_hut' never forms an n x n matrix: 4000 points embed
    quickly with a good neighbourhood preservation."""
    from sklearn.datasets import make_blobs
    Xb, _ = make_blobs(4000, 10, centers=6, random_state=0)
    t = M.TSNE(method="barnes_hut", init="pca", learning_rate="auto", n_iter=300,
               random_state=0)
    E = t.fit_transform(Xb)
    assert E.shape == (4000, 2) and np.isfinite(E).all()
    assert M.trustworthiness(Xb[:1000], E[:1000], n_neighbors=5) > 0.9
    with pytest.raises(ValueError):
        M.TSNE(n_components=4, method="barnes_hut").fit(Xb[:50])
