"""Device (MI355X) paths of the estimators whose heavy algebra runs in
torch on the resolved device: Gaussian mixture EM, label spreading,
kernel density, NCA, Bayesian ridge, PLSSVD.  Compared with scikit-learn
(fp64 on the GPU, so tolerances stay tight)."""
import warnings

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
pytest.importorskip("sklearn")


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        yield


def test_device_resolution():
    from sq_learn_amd.runtime.device import resolve_device
    assert resolve_device(None).type == "cuda"


def test_gmm_labelspreading_kde_on_device():
    import sklearn.mixture as SM
    import sklearn.neighbors as SN
    import sklearn.semi_supervised as SS
    from sklearn.datasets import make_blobs

    import sq_learn_amd.mixture as MM
    import sq_learn_amd.neighbors as MN
    import sq_learn_amd.semi_supervised as MS
    X, y = make_blobs(600, 4, centers=4, random_state=0)
    for cov in ["full", "diag"]:
        a = SM.GaussianMixture(4, covariance_type=cov, random_state=0, init_params="random").fit(X)
        b = MM.GaussianMixture(4, covariance_type=cov, random_state=0, init_params="random").fit(X)
        np.testing.assert_allclose(b.means_, a.means_, atol=1e-6)
    ys = y.copy()
    ys[np.random.RandomState(0).rand(len(y)) < 0.8] = -1
    Xs = X / X.std(0) / 3
    a = SS.LabelSpreading(gamma=1).fit(Xs, ys)
    b = MS.LabelSpreading(gamma=1).fit(Xs, ys)
    np.testing.assert_allclose(b.label_distributions_, a.label_distributions_, atol=1e-10)
    a = SN.KernelDensity(bandwidth=0.7).fit(X).score_samples(X[:50])
    b = MN.KernelDensity(bandwidth=0.7).fit(X).score_samples(X[:50])
    np.testing.assert_allclose(b, a, atol=1e-9)


def test_nca_bayes_pls_on_device():
    import sklearn.cross_decomposition as SCD
    import sklearn.linear_model as SL
    import sklearn.neighbors as SN
    from sklearn.datasets import make_classification

    import sq_learn_amd.cross_decomposition as MCD
    import sq_learn_amd.linear_model as ML
    import sq_learn_amd.neighbors as MN
    X, y = make_classification(200, 6, n_informative=4, n_classes=3, random_state=0)
    a = SN.NeighborhoodComponentsAnalysis(n_components=2, init="identity").fit(X, y)
    b = MN.NeighborhoodComponentsAnalysis(n_components=2, init="identity").fit(X, y)
    # L-BFGS stops at a slightly different point under device fp order
    assert np.abs(a.components_ - b.components_).max() / np.abs(a.components_).max() < 1e-2
    yr = X[:, 0] * 2 - X[:, 1]
    # evidence iterations stop at tol=1e-3: device SVD rounding can shift
    # the stopping iterate slightly
    np.testing.assert_allclose(ML.BayesianRidge().fit(X, yr).coef_,
                               SL.BayesianRidge().fit(X, yr).coef_, atol=1e-4)
    Y = np.c_[yr, X[:, 2]]
    np.testing.assert_allclose(np.abs(MCD.PLSSVD(2).fit(X, Y).transform(X)),
                               np.abs(SCD.PLSSVD(2).fit(X, Y).transform(X)), atol=1e-9)


def test_tsne_mds_on_device():
    import sklearn.manifold as SMf
    from sklearn.datasets import load_digits

    import sq_learn_amd.manifold as MMf
    Xd = load_digits(return_X_y=True)[0][:800]
    a = SMf.TSNE(method="exact", init="random", learning_rate=200.0, random_state=0).fit(Xd)
    b = MMf.TSNE(method="exact", init="random", learning_rate=200.0, random_state=0).fit(Xd)
    assert abs(a.kl_divergence_ - b.kl_divergence_) < 0.1 * a.kl_divergence_
    assert MMf.trustworthiness(Xd, b.embedding_) > 0.98


def test_mlp_trains_on_device():
    import sklearn.neural_network as SNN
    from sklearn.datasets import load_digits

    import sq_learn_amd.neural_network as MNN
    X, y = load_digits(return_X_y=True)
    X = X[:600] / 16
    y = y[:600]
    kw = dict(hidden_layer_sizes=(64, 32), max_iter=20, random_state=0)
    b = MNN.MLPClassifier(**kw).fit(X, y)
    assert b._W[0].device.type == "cuda"
    a = SNN.MLPClassifier(**kw).fit(X, y)
    # same RNG stream, device GEMM reduction order: tiny drift only
    np.testing.assert_allclose(a.predict_proba(X), b.predict_proba(X), atol=1e-6)


def test_mixtures_split_k_on_device():
    import sklearn.mixture as SMx
    from sklearn.datasets import make_blobs

    import sq_learn_amd.mixture as MMx
    X = make_blobs(5000, 6, centers=4, random_state=0)[0]   # n > split-K threshold
    for ct in ("full", "tied", "diag", "spherical"):
        kw = dict(n_components=4, covariance_type=ct, init_params="random", random_state=0)
        a = SMx.GaussianMixture(**kw).fit(X)
        b = MMx.GaussianMixture(**kw).fit(X)
        np.testing.assert_allclose(a.means_, b.means_, atol=1e-6)
        a = SMx.BayesianGaussianMixture(max_iter=200, **kw).fit(X)
        b = MMx.BayesianGaussianMixture(max_iter=200, **kw).fit(X)
        assert b._pc.device.type == "cuda"
        np.testing.assert_allclose(a.weights_, b.weights_, atol=1e-6)
        np.testing.assert_allclose(a.means_, b.means_, atol=1e-5)


def test_sparse_encode_batched_cd_on_device():
    import sklearn.decomposition as SD

    import sq_learn_amd.decomposition as MD
    rng = np.random.RandomState(0)
    X = rng.randn(300, 24)
    D = rng.randn(10, 24)
    D /= np.linalg.norm(D, axis=1, keepdims=True)
    for pos in (False, True):
        a = SD.sparse_encode(X, D, algorithm="lasso_cd", alpha=0.3, positive=pos)
        b = MD.sparse_encode(X, D, algorithm="lasso_cd", alpha=0.3, positive=pos)
        np.testing.assert_allclose(a, b, atol=1e-8)
