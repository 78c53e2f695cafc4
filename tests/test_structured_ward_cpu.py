"""Connectivity-constrained Ward agglomeration (reference
``cluster/_agglomerative.py`` ``ward_tree`` structured branch,
``_fix_connectivity``, ``_hierarchical_fast.pyx``)."""
import warnings

import numpy as np
import pytest

import sq_learn_amd.cluster as Q
from sq_learn_amd.models.cluster.hierarchical import ward_tree

S = pytest.importorskip("sklearn.cluster")


@pytest.fixture(scope="module")
def data():
    from sklearn.neighbors import kneighbors_graph
    X = np.random.RandomState(0).rand(120, 3)
    return X, kneighbors_graph(X, 6, include_self=False), kneighbors_graph(X, 2)


def test_ward_tree_parity(data):
    X, G, _ = data
    a = S.ward_tree(X, connectivity=G, return_distance=True)
    b = ward_tree(X, connectivity=G, return_distance=True)
    np.testing.assert_array_equal(a[0], b[0])
    assert a[1] == b[1] and a[2] == b[2]
    np.testing.assert_array_equal(a[3], b[3])
    np.testing.assert_allclose(a[4], b[4], rtol=1e-12)


@pytest.mark.parametrize("kw", [dict(n_clusters=4), dict(n_clusters=4, compute_full_tree=True),
                                dict(n_clusters=None, distance_threshold=0.5)])
def test_agglomerative_connectivity(data, kw):
    X, G, _ = data
    a = S.AgglomerativeClustering(connectivity=G, **kw).fit(X)
    b = Q.AgglomerativeClustering(connectivity=G, **kw).fit(X)
    np.testing.assert_array_equal(a.labels_, b.labels_)
    np.testing.assert_array_equal(a.children_, b.children_)


def test_disconnected_graph_is_completed(data):
    X, _, G2 = data
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a = S.AgglomerativeClustering(5, connectivity=G2).fit(X)
        b = Q.AgglomerativeClustering(5, connectivity=G2).fit(X)
    np.testing.assert_array_equal(a.labels_, b.labels_)
    assert a.n_connected_components_ == b.n_connected_components_
    with pytest.raises(ValueError):
        ward_tree(X, connectivity=G2[:10, :10])
