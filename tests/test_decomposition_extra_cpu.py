"""KernelPCA, FastICA, FactorAnalysis, NMF and LDA against scikit-learn
(reference sklearn/decomposition).  FastICA: sklearn>=1.1 changed the
whitening sign convention and defaults, so the check is source recovery
(parity unpinned for the exact iterates)."""
import warnings

import numpy as np
import pytest

pytest.importorskip("sklearn")
import sklearn.decomposition as S  # noqa: E402
from sklearn.datasets import make_classification, make_multilabel_classification  # noqa: E402

import sq_learn_amd.decomposition as M  # noqa: E402

X, y = make_classification(300, 8, n_informative=5, random_state=0)


@pytest.fixture(autouse=True)
def _quiet():
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        yield


@pytest.mark.parametrize("kernel,kw", [("linear", {}), ("rbf", dict(gamma=0.1)),
                                       ("poly", dict(degree=2)), ("cosine", {})])
@pytest.mark.parametrize("solver", ["dense", "arpack"])
def test_kernel_pca(kernel, kw, solver):
    inv = kernel == "rbf"
    a = S.KernelPCA(4, kernel=kernel, eigen_solver=solver, random_state=0,
                    fit_inverse_transform=inv, **kw).fit(X)
    b = M.KernelPCA(4, kernel=kernel, eigen_solver=solver, random_state=0,
                    fit_inverse_transform=inv, **kw).fit(X)
    ta, tb = a.transform(X), b.transform(X)
    np.testing.assert_allclose(np.abs(tb), np.abs(ta), atol=1e-9)
    np.testing.assert_allclose(b.eigenvalues_, a.eigenvalues_, rtol=1e-10)
    if inv:
        np.testing.assert_allclose(b.inverse_transform(tb), a.inverse_transform(ta), atol=1e-9)


@pytest.mark.parametrize("algorithm", ["parallel", "deflation"])
@pytest.mark.parametrize("fun", ["logcosh", "exp", "cube"])
def test_fastica_recovers_sources(algorithm, fun):
    rng = np.random.RandomState(0)
    src = rng.laplace(size=(2000, 3))
    Xi = src @ rng.randn(3, 3).T
    ica = M.FastICA(3, algorithm=algorithm, fun=fun, random_state=0)
    est = ica.fit_transform(Xi)
    C = np.abs(np.corrcoef(src.T, est.T)[:3, 3:])
    assert (C.max(axis=1) > 0.95).all()
    np.testing.assert_allclose(ica.inverse_transform(est), Xi, atol=1e-8)


@pytest.mark.parametrize("svd_method", ["lapack", "randomized"])
@pytest.mark.parametrize("rotation", [None, "varimax", "quartimax"])
def test_factor_analysis(svd_method, rotation):
    a = S.FactorAnalysis(3, svd_method=svd_method, rotation=rotation, random_state=0).fit(X)
    b = M.FactorAnalysis(3, svd_method=svd_method, rotation=rotation, random_state=0).fit(X)
    np.testing.assert_allclose(np.abs(b.components_), np.abs(a.components_), atol=1e-8)
    np.testing.assert_allclose(b.score_samples(X), a.score_samples(X), atol=1e-8)
    assert a.n_iter_ == b.n_iter_


@pytest.mark.parametrize("solver,beta", [("cd", "frobenius"), ("mu", "frobenius"),
                                         ("mu", "kullback-leibler"), ("mu", 1.5)])
@pytest.mark.parametrize("init", ["random", "nndsvda", "nndsvdar"])
def test_nmf(solver, beta, init):
    Xn = np.abs(X)
    a = S.NMF(4, solver=solver, beta_loss=beta, init=init, random_state=0, max_iter=300)
    b = M.NMF(4, solver=solver, beta_loss=beta, init=init, random_state=0, max_iter=300)
    np.testing.assert_allclose(b.fit_transform(Xn), a.fit_transform(Xn), atol=1e-10)
    np.testing.assert_allclose(b.components_, a.components_, atol=1e-10)
    assert a.n_iter_ == b.n_iter_
    np.testing.assert_allclose(b.transform(Xn), a.transform(Xn), atol=1e-10)


@pytest.mark.parametrize("method", ["batch", "online"])
def test_lda(method):
    Xc, _ = make_multilabel_classification(200, 30, n_classes=5, random_state=0)
    a = S.LatentDirichletAllocation(5, learning_method=method, random_state=0, max_iter=5).fit(Xc)
    b = M.LatentDirichletAllocation(5, learning_method=method, random_state=0, max_iter=5).fit(Xc)
    np.testing.assert_allclose(b.components_, a.components_, rtol=1e-6)
    np.testing.assert_allclose(b.transform(Xc), a.transform(Xc), atol=1e-6)
    np.testing.assert_allclose(b.perplexity(Xc), a.perplexity(Xc), rtol=1e-8)
