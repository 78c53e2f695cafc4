"""AffinityPropagation, MeanShift, Birch, OPTICS, SpectralClustering and
SpectralEmbedding against scikit-learn (reference sklearn/cluster,
sklearn/manifold/_spectral_embedding.py).  OPTICS with euclidean
distances is BLAS-rounding sensitive (reachabilities are rounded to 15
decimals, ties then follow the last-ulp of the GEMM expansion), so the
exact comparison uses manhattan; euclidean compares the clustering."""
import warnings

import numpy as np
import pytest

pytest.importorskip("sklearn")
import sklearn.cluster as S  # noqa: E402
import sklearn.manifold as SMf  # noqa: E402
from sklearn.datasets import make_blobs  # noqa: E402
from sklearn.metrics import adjusted_rand_score  # noqa: E402

import sq_learn_amd.cluster as M  # noqa: E402
import sq_learn_amd.manifold as MMf  # noqa: E402

X, y = make_blobs(300, 3, centers=4, cluster_std=0.8, random_state=0)


@pytest.fixture(autouse=True)
def _quiet():
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        yield


def test_affinity_propagation():
    a = S.AffinityPropagation(random_state=0).fit(X)
    b = M.AffinityPropagation(random_state=0).fit(X)
    assert list(a.cluster_centers_indices_) == list(b.cluster_centers_indices_)
    assert (a.labels_ == b.labels_).all() and a.n_iter_ == b.n_iter_
    assert (a.predict(X[:20]) == b.predict(X[:20])).all()


@pytest.mark.parametrize("kw", [{}, dict(bin_seeding=True), dict(cluster_all=False, bandwidth=1.0)])
def test_mean_shift(kw):
    a, b = S.MeanShift(**kw).fit(X), M.MeanShift(**kw).fit(X)
    np.testing.assert_allclose(b.cluster_centers_, a.cluster_centers_, atol=1e-10)
    assert (a.labels_ == b.labels_).all()
    assert S.estimate_bandwidth(X) == pytest.approx(M.estimate_bandwidth(X), rel=1e-12)


@pytest.mark.parametrize("kw", [{}, dict(threshold=0.3, branching_factor=10), dict(n_clusters=None)])
def test_birch(kw):
    a, b = S.Birch(**kw).fit(X), M.Birch(**kw).fit(X)
    sa = a.subcluster_centers_[np.lexsort(a.subcluster_centers_.T)]
    sb = b.subcluster_centers_[np.lexsort(b.subcluster_centers_.T)]
    np.testing.assert_allclose(sb, sa, atol=1e-12)
    assert (a.labels_ == b.labels_).all()


def test_optics():
    kw = dict(metric="manhattan", algorithm="ball_tree")
    a, b = S.OPTICS(**kw).fit(X), M.OPTICS(**kw).fit(X)
    assert (a.ordering_ == b.ordering_).all() and (a.labels_ == b.labels_).all()
    np.testing.assert_allclose(b.core_distances_, a.core_distances_)
    for kw in [{}, dict(cluster_method="dbscan", eps=0.5)]:
        a, b = S.OPTICS(**kw).fit(X), M.OPTICS(**kw).fit(X)
        np.testing.assert_allclose(b.core_distances_, a.core_distances_, atol=1e-12)
        assert adjusted_rand_score(a.labels_, b.labels_) > 0.9


@pytest.mark.parametrize("kw", [dict(affinity="rbf", gamma=0.5), dict(affinity="nearest_neighbors"),
                                dict(affinity="rbf", gamma=0.5, assign_labels="discretize")])
def test_spectral(kw):
    a = S.SpectralClustering(4, random_state=0, **kw).fit(X)
    b = M.SpectralClustering(4, random_state=0, **kw).fit(X)
    assert adjusted_rand_score(a.labels_, b.labels_) == pytest.approx(1.0)
    for aff in ["rbf", "nearest_neighbors"]:
        ea = SMf.SpectralEmbedding(2, random_state=0, affinity=aff).fit_transform(X)
        eb = MMf.SpectralEmbedding(2, random_state=0, affinity=aff).fit_transform(X)
        np.testing.assert_allclose(eb, ea, atol=1e-8)
