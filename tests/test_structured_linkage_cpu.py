"""Connectivity-constrained agglomerative clustering for every linkage
(reference cluster/_agglomerative.py:501-603) against scikit-learn: same
merge order, labels and merge distances, full and partial trees."""
import warnings

import numpy as np
import pytest

sk = pytest.importorskip("sklearn")
from sklearn.cluster import AgglomerativeClustering as SKAgg  # noqa: E402
from sklearn.neighbors import kneighbors_graph  # noqa: E402

from sq_learn_amd.models.cluster.hierarchical import (AgglomerativeClustering,  # noqa: E402
                                                      linkage_tree)

X = np.random.RandomState(0).randn(120, 3)


@pytest.mark.parametrize("linkage,metric", [("complete", "euclidean"), ("complete", "manhattan"),
                                            ("average", "euclidean"), ("average", "cosine"),
                                            ("single", "euclidean"), ("single", "manhattan"),
                                            ("ward", "euclidean")])
@pytest.mark.parametrize("nn", [4, 10])
@pytest.mark.parametrize("nc,thr", [(4, None), (None, 1.5)])
def test_structured_linkage_matches(linkage, metric, nn, nc, thr):
    conn = kneighbors_graph(X, nn, include_self=False)
    kw = dict(n_clusters=nc, distance_threshold=thr, linkage=linkage, connectivity=conn,
              compute_distances=True)
    if thr is not None:
        kw["compute_full_tree"] = True
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a = SKAgg(metric=metric, **kw).fit(X)
        b = AgglomerativeClustering(affinity=metric, **kw).fit(X)
    np.testing.assert_array_equal(b.children_, a.children_)
    np.testing.assert_array_equal(b.labels_, a.labels_)
    np.testing.assert_allclose(b.distances_, a.distances_, rtol=1e-12, atol=1e-12)
    assert b.n_connected_components_ == a.n_connected_components_


def test_disconnected_graph_is_completed():
    conn = kneighbors_graph(X, 2, include_self=False)
    with pytest.warns(UserWarning, match="connected components"):
        out = linkage_tree(X, connectivity=conn, linkage="average", return_distance=True)
    assert out[1] > 1 and out[0].shape == (X.shape[0] - 1, 2)
