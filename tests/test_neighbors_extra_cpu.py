"""Host KD/ball trees (csrc/host/binary_tree.cpp), metric/algorithm
routing, radius estimators, graphs, KDE, LOF, NearestCentroid and NCA
against scikit-learn (reference sklearn/neighbors).  Compact-kernel KDE
values at points with no support are -inf here (exact evaluation); the
comparison covers the finite entries."""
import pickle
import warnings

import numpy as np
import pytest

pytest.importorskip("sklearn")
import sklearn.neighbors as S  # noqa: E402

import sq_learn_amd.neighbors as M  # noqa: E402

rng = np.random.RandomState(0)
X, Q = rng.randn(500, 4), rng.randn(50, 4)
y = (X[:, 0] > 0).astype(int)
yr = X[:, 0] + X[:, 1]


@pytest.fixture(autouse=True)
def _quiet():
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        yield


@pytest.mark.parametrize("cls", ["KDTree", "BallTree"])
@pytest.mark.parametrize("kw", [{}, dict(metric="manhattan"), dict(metric="chebyshev"),
                                dict(metric="minkowski", p=3)])
def test_trees(cls, kw):
    a = getattr(S, cls)(X, leaf_size=10, **kw)
    b = getattr(M, cls)(X, leaf_size=10, **kw)
    da, ia = a.query(Q, k=5)
    db, ib = b.query(Q, k=5)
    np.testing.assert_allclose(db, da, atol=1e-12)
    assert (ia == ib).mean() > 0.99
    for u, v in zip(a.query_radius(Q, r=1.0), b.query_radius(Q, r=1.0)):
        assert set(u) == set(v)
    assert (a.query_radius(Q, r=1.0, count_only=True) == b.query_radius(Q, r=1.0, count_only=True)).all()
    assert (a.two_point_correlation(Q, [0.5, 1, 2]) == b.two_point_correlation(Q, [0.5, 1, 2])).all()
    _, _, na, ba = a.get_arrays()
    _, _, nb, bb = b.get_arrays()
    assert na.shape == nb.shape and ba.shape == bb.shape
    b2 = pickle.loads(pickle.dumps(b))
    np.testing.assert_allclose(b2.query(Q, k=3)[0], db[:, :3])


@pytest.mark.parametrize("kernel", ["gaussian", "tophat", "epanechnikov", "exponential", "linear"])
def test_kde(kernel):
    a = S.KernelDensity(bandwidth=0.5, kernel=kernel).fit(X).score_samples(Q)
    b = M.KernelDensity(bandwidth=0.5, kernel=kernel).fit(X).score_samples(Q)
    f = np.isfinite(b)
    np.testing.assert_allclose(b[f], a[f], atol=1e-10)
    if kernel == "gaussian":
        np.testing.assert_allclose(M.KernelDensity(bandwidth=0.5).fit(X).sample(5, random_state=0),
                                   S.KernelDensity(bandwidth=0.5).fit(X).sample(5, random_state=0))


@pytest.mark.parametrize("algo,metric", [("brute", "euclidean"), ("brute", "manhattan"),
                                         ("brute", "cosine"), ("kd_tree", "euclidean"),
                                         ("kd_tree", "manhattan"), ("ball_tree", "euclidean")])
def test_nearest_neighbors_routing(algo, metric):
    a = S.NearestNeighbors(n_neighbors=4, algorithm=algo, metric=metric).fit(X)
    b = M.NearestNeighbors(n_neighbors=4, algorithm=algo, metric=metric).fit(X)
    np.testing.assert_allclose(b.kneighbors(Q)[0], a.kneighbors(Q)[0], atol=1e-10)
    assert abs(a.kneighbors_graph(Q, mode="distance") - b.kneighbors_graph(Q, mode="distance")).max() < 1e-10
    assert abs(a.radius_neighbors_graph(Q, radius=1.0, mode="distance")
               - b.radius_neighbors_graph(Q, radius=1.0, mode="distance")).max() < 1e-10


def test_radius_models_lof_centroid():
    a = S.RadiusNeighborsClassifier(radius=1.5, outlier_label="most_frequent").fit(X, y)
    b = M.RadiusNeighborsClassifier(radius=1.5, outlier_label="most_frequent").fit(X, y)
    assert (a.predict(Q) == b.predict(Q)).all()
    np.testing.assert_allclose(b.predict_proba(Q), a.predict_proba(Q))
    a = S.RadiusNeighborsRegressor(radius=1.5, weights="distance").fit(X, yr)
    b = M.RadiusNeighborsRegressor(radius=1.5, weights="distance").fit(X, yr)
    np.testing.assert_allclose(b.predict(Q), a.predict(Q), atol=1e-12)
    a, b = S.LocalOutlierFactor().fit(X), M.LocalOutlierFactor().fit(X)
    np.testing.assert_allclose(b.negative_outlier_factor_, a.negative_outlier_factor_, atol=1e-12)
    a, b = S.LocalOutlierFactor(novelty=True).fit(X), M.LocalOutlierFactor(novelty=True).fit(X)
    np.testing.assert_allclose(b.score_samples(Q), a.score_samples(Q), atol=1e-12)
    for st in [None, 0.5]:
        a = S.NearestCentroid(shrink_threshold=st).fit(X, y)
        b = M.NearestCentroid(shrink_threshold=st).fit(X, y)
        np.testing.assert_allclose(b.centroids_, a.centroids_)
    a = S.KNeighborsTransformer(n_neighbors=3).fit(X)
    b = M.KNeighborsTransformer(n_neighbors=3).fit(X)
    assert abs(a.transform(Q) - b.transform(Q)).max() < 1e-10


@pytest.mark.parametrize("init", ["identity", "lda", "random", "pca"])
def test_nca(init):
    from sklearn.datasets import make_classification
    Xc, yc = make_classification(150, 6, n_informative=4, n_classes=3, random_state=0)
    a = S.NeighborhoodComponentsAnalysis(n_components=2, init=init, random_state=0).fit(Xc, yc)
    b = M.NeighborhoodComponentsAnalysis(n_components=2, init=init, random_state=0).fit(Xc, yc)
    # PCA/LDA sign conventions differ between sklearn versions: compare
    # up to a per-row sign, relative to the component scale
    rel = np.abs(np.abs(a.components_) - np.abs(b.components_)).max() / np.abs(a.components_).max()
    assert rel < 1e-2
