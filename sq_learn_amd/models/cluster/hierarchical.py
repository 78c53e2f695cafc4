"""Agglomerative clustering (reference ``cluster/_agglomerative.py`` +
``_hierarchical_fast.pyx``).

Pairwise distances are computed on the data's device (exact difference
form, no norm expansion, so merge heights match a float64 pdist), reduced
to the condensed upper triangle, and handed to the host-native linkage core
``sqh_linkage`` (``csrc/host/hier_host.cpp``: nearest-neighbour chain with
Lance-Williams updates, Prim's MST for single linkage, stable height sort,
union-find relabelling).  Connectivity-constrained trees (reference
``_agglomerative.py:501-603``) merge only along graph edges: ward through a
heap of edge inertias, complete / average through per-node neighbour maps
merged by max / size-weighted mean, single through the minimum spanning
tree of the graph and union-find labelling.
"""

from heapq import heappush, heappushpop

import numpy as np
import torch

from ...base import BaseEstimator, ClusterMixin, TransformerMixin
from ...ops import _host
from ...runtime.device import resolve_device, to_tensor
from ...utils.validation import check_array, check_is_fitted

_METHODS = {"single": 0, "complete": 1, "average": 2, "weighted": 3, "ward": 4}


def _condensed(X, affinity, device=None):
    """float64 condensed distance vector (n(n-1)/2) for the affinity."""
    if affinity == "precomputed":
        D = np.asarray(X, dtype=np.float64)
        iu = np.triu_indices(D.shape[0], k=1)
        return np.ascontiguousarray(D[iu])
    if callable(affinity):
        D = np.asarray(affinity(np.asarray(X)), dtype=np.float64)
        iu = np.triu_indices(D.shape[0], k=1)
        return np.ascontiguousarray(D[iu])
    Xt = X if isinstance(X, torch.Tensor) else to_tensor(np.asarray(X, dtype=np.float64),
                                                         resolve_device(device))
    Xt = Xt.to(torch.float64)
    n = Xt.shape[0]
    if affinity in ("euclidean", "l2"):
        D = torch.cdist(Xt, Xt, compute_mode="donot_use_mm_for_euclid_dist")
    elif affinity in ("l1", "manhattan", "cityblock"):
        D = torch.cdist(Xt, Xt, p=1.0)
    elif affinity == "cosine":
        nrm = torch.linalg.vector_norm(Xt, dim=1, keepdim=True)
        D = (1.0 - (Xt / nrm) @ (Xt / nrm).T).clamp_(min=0)
    else:
        from scipy.spatial.distance import pdist
        return np.ascontiguousarray(pdist(np.asarray(Xt.cpu()), metric=affinity))
    iu = torch.triu_indices(n, n, offset=1, device=D.device)
    return np.ascontiguousarray(D[iu[0], iu[1]].cpu().numpy())


def _linkage_matrix(cond, n, method, ordered_children=True):
    Z = np.zeros((max(n - 1, 0), 4), dtype=np.float64)
    if n > 1:
        rc = _host.lib().sqh_linkage(_host.ptr(cond), n, _METHODS[method],
                                     int(ordered_children), _host.ptr(Z))
        if rc != 0:
            raise ValueError("Unknown linkage type %s" % method)
    return Z


def _fix_connectivity(X, connectivity, affinity="euclidean"):
    """Symmetrise the connectivity graph and join disconnected components
    through their closest pair (reference ``cluster/_agglomerative.py``)."""
    import warnings

    from scipy import sparse
    from scipy.sparse.csgraph import connected_components

    from ...utils.pairwise import pairwise_distances
    n = X.shape[0]
    if connectivity.shape[0] != n or connectivity.shape[1] != n:
        raise ValueError("Wrong shape for connectivity matrix: %s when X is %s"
                         % (connectivity.shape, X.shape))
    C = sparse.csr_matrix(connectivity)
    C = (C + C.T).tolil()
    ncc, labels = connected_components(C)
    if ncc > 1:
        warnings.warn("the number of connected components of the connectivity matrix is %d > 1. "
                      "Completing it to avoid stopping the tree early." % ncc, stacklevel=2)
        Xn = np.asarray(X.detach().cpu().numpy() if hasattr(X, "detach") else X)
        for i in range(ncc):
            ii = np.where(labels == i)[0]
            for j in range(i):
                jj = np.where(labels == j)[0]
                D = np.asarray(pairwise_distances(Xn[ii], Xn[jj], metric=affinity))
                a, b = np.where(D == np.min(D))
                C[ii[a[0]], jj[b[0]]] = True
                C[jj[b[0]], ii[a[0]]] = True
    return C, ncc


def _structured_ward(X, connectivity, n_clusters, return_distance):
    """Ward agglomeration restricted to a connectivity graph: a heap of
    candidate merges along graph edges (reference ``ward_tree`` structured
    branch and ``_hierarchical_fast.pyx`` ``compute_ward_dist`` /
    ``_get_parents``)."""
    import heapq
    Xn = np.asarray(X.detach().cpu().numpy() if hasattr(X, "detach") else X, dtype=np.float64)
    n, d = Xn.shape
    C, ncc = _fix_connectivity(Xn, connectivity)
    rows_i, cols_i, A = [], [], []
    for ind, row in enumerate(C.rows):
        A.append(list(row))
        lower = [i for i in row if i < ind]
        rows_i.extend([ind] * len(lower))
        cols_i.extend(lower)
    if n_clusters is None:
        n_nodes = 2 * n - 1
    else:
        if n_clusters > n:
            raise ValueError("Cannot provide more clusters than samples. %i n_clusters was asked, "
                             "and there are %i samples." % (n_clusters, n))
        n_nodes = 2 * n - n_clusters
    m1 = np.zeros(n_nodes)
    m1[:n] = 1
    m2 = np.zeros((n_nodes, d))
    m2[:n] = Xn

    def ward_dist(r, c):
        r = np.asarray(r, dtype=np.intp)
        c = np.asarray(c, dtype=np.intp)
        w = m1[r] * m1[c] / (m1[r] + m1[c])
        diff = m2[r] / m1[r][:, None] - m2[c] / m1[c][:, None]
        return (diff * diff).sum(1) * w

    heap = list(zip(ward_dist(rows_i, cols_i).tolist(), rows_i, cols_i))
    heapq.heapify(heap)
    parent = np.arange(n_nodes, dtype=np.intp)
    used = np.ones(n_nodes, dtype=bool)
    children = []
    dist = np.empty(n_nodes - n) if return_distance else None
    for k in range(n, n_nodes):
        while True:
            inert, i, j = heapq.heappop(heap)
            if used[i] and used[j]:
                break
        parent[i] = parent[j] = k
        children.append((i, j))
        used[i] = used[j] = False
        if return_distance:
            dist[k - n] = inert
        m1[k] = m1[i] + m1[j]
        m2[k] = m2[i] + m2[j]
        heads, seen = [], np.ones(n_nodes, dtype=bool)
        seen[k] = False
        for node0 in A[i] + A[j]:
            node = node0
            p = parent[node]
            while p != node:
                node = p
                p = parent[node]
            if seen[node]:
                seen[node] = False
                heads.append(node)
        for c in heads:
            A[c].append(k)
        A.append(heads)
        if heads:
            for dd, c in zip(ward_dist([k] * len(heads), heads).tolist(), heads):
                heapq.heappush(heap, (dd, k, c))
    children = np.array([c[::-1] for c in children], dtype=np.intp)
    if return_distance:
        return children, ncc, n, parent, np.sqrt(2.0 * dist)
    return children, ncc, n, parent


def ward_tree(X, *, connectivity=None, n_clusters=None, return_distance=False, device=None):
    """(children, n_connected_components, n_leaves, parents[, distances])."""
    if connectivity is not None:
        return _structured_ward(X, connectivity, n_clusters, return_distance)
    X = X if isinstance(X, torch.Tensor) else check_array(X)
    n = X.shape[0]
    if n_clusters is not None:
        import warnings
        warnings.warn("Partial build of the tree is implemented only for structured clustering "
                      "(i.e. with explicit connectivity). The algorithm will build the full "
                      "tree and only retain the lower branches required for the specified "
                      "number of clusters", stacklevel=2)
    Z = _linkage_matrix(_condensed(X, "euclidean", device), n, "ward")
    children = Z[:, :2].astype(np.intp)
    if return_distance:
        return children, 1, n, None, Z[:, 2]
    return children, 1, n, None


class _Edge:
    """Heap entry ordered by weight only (ties keep heap order, like the
    reference's WeightedEdge)."""
    __slots__ = ("w", "a", "b")

    def __init__(self, w, a, b):
        self.w, self.a, self.b = w, a, b

    def __lt__(self, other):
        return self.w < other.w


def _label_mst(edges, n):
    """Union-find labelling of weight-sorted MST edges into a linkage
    matrix (reference ``_single_linkage_label``)."""
    parent = np.full(2 * n - 1, -1, dtype=np.intp)
    size = np.zeros(2 * n - 1, dtype=np.intp)
    size[:n] = 1
    nxt = n
    out = np.zeros((len(edges), 4))

    def find(v):
        root = v
        while parent[root] != -1:
            root = parent[root]
        while v != root and parent[v] != root:
            parent[v], v = root, parent[v]
        return root

    for t, (a, b, w) in enumerate(edges):
        ra, rb = find(int(a)), find(int(b))
        out[t] = (ra, rb, w, size[ra] + size[rb])
        parent[ra] = parent[rb] = nxt
        size[nxt] = size[ra] + size[rb]
        nxt += 1
    return out


def _structured_linkage(X, connectivity, n_clusters, linkage, affinity, return_distance):
    """complete / average / single linkage restricted to a connectivity
    graph (reference ``linkage_tree`` structured branch)."""
    import heapq

    from scipy.sparse.csgraph import minimum_spanning_tree

    from ...utils.pairwise import paired_distances
    Xn = np.asarray(X.detach().cpu().numpy() if hasattr(X, "detach") else X)
    if Xn.ndim == 1:
        Xn = Xn.reshape(-1, 1)
    n = Xn.shape[0]
    C, ncc = _fix_connectivity(Xn, connectivity, affinity=affinity)
    C = C.tocoo()
    keep = C.row != C.col
    rows, cols = C.row[keep], C.col[keep]
    if affinity == "precomputed":
        dist = np.asarray(Xn[rows, cols], dtype=np.float64)
    else:
        dist = np.asarray(paired_distances(Xn[rows], Xn[cols], metric=affinity),
                          dtype=np.float64)
    if n_clusters is None:
        n_nodes = 2 * n - 1
    else:
        if n_clusters > n:
            raise ValueError("Cannot provide more clusters than samples. %i n_clusters was asked, "
                             "and there are %i samples." % (n_clusters, n))
        n_nodes = 2 * n - n_clusters
    from scipy import sparse
    G = sparse.coo_matrix((dist, (rows, cols)), shape=(n, n))
    if linkage == "single":
        # zero-length edges survive the MST as machine epsilon, then go back to 0
        G = G.astype(np.float64)
        eps = np.finfo(np.float64).eps
        G.data[G.data == 0] = eps
        mst = minimum_spanning_tree(G.tocsr()).tocoo()
        mst.data[mst.data == eps] = 0
        E = np.vstack([mst.row, mst.col, mst.data]).T
        E = E[np.argsort(E[:, 2], kind="mergesort")]
        Z = _label_mst(E, n)
        children = Z[:, :2].astype(np.intp)
        parent = np.arange(n_nodes, dtype=np.intp)
        for i, (left, right) in enumerate(children, n):
            if n_clusters is not None and i >= n_nodes:
                break
            if left < n_nodes:
                parent[left] = i
            if right < n_nodes:
                parent[right] = i
        if return_distance:
            return children, ncc, n, parent, Z[:, 2]
        return children, ncc, n, parent
    # per-node neighbour maps (key order = the reference's std::map order)
    L = G.tolil()
    A = [dict(zip(r, d)) for r, d in zip(L.rows, L.data)] + [None] * (n_nodes - n)
    heap = [_Edge(d, i, r) for i, (r_, d_) in enumerate(zip(L.rows, L.data))
            for r, d in zip(r_, d_) if r < i]
    heapq.heapify(heap)
    parent = np.arange(n_nodes, dtype=np.intp)
    used = np.ones(n_nodes, dtype=np.intp)
    children = []
    distances = np.empty(n_nodes - n) if return_distance else None
    for k in range(n, n_nodes):
        while True:
            e = heapq.heappop(heap)
            if used[e.a] and used[e.b]:
                break
        i, j = e.a, e.b
        if return_distance:
            distances[k - n] = e.w
        parent[i] = parent[j] = k
        children.append((i, j))
        n_i, n_j = used[i], used[j]
        used[k] = n_i + n_j
        used[i] = used[j] = 0
        merged = {c: v for c, v in A[i].items() if used[c]}
        for c, v in A[j].items():
            if not used[c]:
                continue
            if c in merged:
                merged[c] = (max(merged[c], v) if linkage == "complete"
                             else (n_i * merged[c] + n_j * v) / (n_i + n_j))
            else:
                merged[c] = v
        merged = dict(sorted(merged.items()))
        for c, v in merged.items():
            A[c][k] = v
            heapq.heappush(heap, _Edge(v, k, c))
        A[k] = merged
        A[i] = A[j] = None
    children = np.array(children, dtype=np.intp)[:, ::-1]
    if return_distance:
        return children, ncc, n, parent, distances
    return children, ncc, n, parent


def linkage_tree(X, connectivity=None, n_clusters=None, linkage="complete",
                 affinity="euclidean", return_distance=False, device=None):
    if linkage not in ("average", "complete", "single"):
        raise ValueError("Unknown linkage option, linkage should be one of %s, but %s was given"
                         % (("average", "complete", "single"), linkage))
    if connectivity is not None:
        if affinity == "cosine" and np.any(~np.any(np.asarray(X), axis=1)):
            raise ValueError("Cosine affinity cannot be used when X contains zero vectors")
        return _structured_linkage(X, connectivity, n_clusters, linkage, affinity,
                                   return_distance)
    if linkage not in ("average", "complete", "single"):
        raise ValueError("Unknown linkage option, linkage should be one of %s, but %s was given"
                         % (("average", "complete", "single"), linkage))
    if affinity == "precomputed":
        X = check_array(X)
        if X.shape[0] != X.shape[1]:
            raise ValueError("Distance matrix should be square, Got matrix of shape {X.shape}")
    n = X.shape[0]
    # the reference labels single-linkage MST edges without ordering the
    # children for its own (non-scipy) metrics
    mst_path = linkage == "single" and affinity in ("euclidean", "l2", "l1", "manhattan",
                                                    "cityblock", "chebyshev", "minkowski")
    Z = _linkage_matrix(_condensed(X, affinity, device), n, linkage,
                        ordered_children=not mst_path)
    children = Z[:, :2].astype(np.intp)
    if return_distance:
        return children, 1, n, None, Z[:, 2]
    return children, 1, n, None


def _complete_linkage(*a, **k):
    return linkage_tree(*a, linkage="complete", **k)


def _average_linkage(*a, **k):
    return linkage_tree(*a, linkage="average", **k)


def _single_linkage(*a, **k):
    return linkage_tree(*a, linkage="single", **k)


_TREE_BUILDERS = dict(ward=ward_tree, complete=_complete_linkage, average=_average_linkage,
                      single=_single_linkage)


def _hc_get_descendent(node, children, n_leaves):
    ind = [node]
    if node < n_leaves:
        return ind
    descendent = []
    while ind:
        i = ind.pop()
        if i < n_leaves:
            descendent.append(i)
        else:
            ind.extend(children[i - n_leaves])
    return descendent


def _hc_cut(n_clusters, children, n_leaves):
    if n_clusters > n_leaves:
        raise ValueError("Cannot extract more clusters than samples: %s clusters where given "
                         "for a tree with %s leaves." % (n_clusters, n_leaves))
    nodes = [-(max(children[-1]) + 1)]
    for _ in range(n_clusters - 1):
        these = children[-nodes[0] - n_leaves]
        heappush(nodes, -these[0])
        heappushpop(nodes, -these[1])
    label = np.zeros(n_leaves, dtype=np.intp)
    for i, node in enumerate(nodes):
        label[_hc_get_descendent(-node, children, n_leaves)] = i
    return label


class AgglomerativeClustering(ClusterMixin, BaseEstimator):
    """Recursively merges the pair of clusters that minimally increases a
    linkage distance (n_clusters or distance_threshold; linkage ward /
    complete / average / single)."""

    def __init__(self, n_clusters=2, *, affinity="euclidean", memory=None, connectivity=None,
                 compute_full_tree="auto", linkage="ward", distance_threshold=None,
                 compute_distances=False, device=None):
        self.n_clusters = n_clusters
        self.distance_threshold = distance_threshold
        self.memory = memory
        self.connectivity = connectivity
        self.compute_full_tree = compute_full_tree
        self.linkage = linkage
        self.affinity = affinity
        self.compute_distances = compute_distances
        self.device = device

    def fit(self, X, y=None):
        if not isinstance(X, torch.Tensor):
            X = check_array(X, ensure_min_samples=2)
        self.n_features_in_ = X.shape[1]
        if self.n_clusters is not None and self.n_clusters <= 0:
            raise ValueError("n_clusters should be an integer greater than 0. %s was provided."
                             % str(self.n_clusters))
        if not ((self.n_clusters is None) ^ (self.distance_threshold is None)):
            raise ValueError("Exactly one of n_clusters and distance_threshold has to be set, "
                             "and the other needs to be None.")
        if self.distance_threshold is not None and not self.compute_full_tree:
            raise ValueError("compute_full_tree must be True if distance_threshold is set.")
        if self.linkage == "ward" and self.affinity != "euclidean":
            raise ValueError("%s was provided as affinity. Ward can only work with euclidean "
                             "distances." % (self.affinity,))
        if self.linkage not in _TREE_BUILDERS:
            raise ValueError("Unknown linkage type %s. Valid options are %s"
                             % (self.linkage, _TREE_BUILDERS.keys()))
        connectivity = self.connectivity
        if connectivity is not None:
            if callable(connectivity):
                connectivity = connectivity(X)
        full = self.compute_full_tree
        if connectivity is None:
            full = True
        if full == "auto":
            full = True if self.distance_threshold is not None else \
                self.n_clusters < max(100, 0.02 * X.shape[0])
        kwargs = {} if self.linkage == "ward" else {"affinity": self.affinity}
        return_distance = self.distance_threshold is not None or self.compute_distances
        out = _TREE_BUILDERS[self.linkage](X, connectivity=connectivity,
                                           n_clusters=None if full else self.n_clusters,
                                           return_distance=return_distance, device=self.device,
                                           **kwargs)
        self.children_, self.n_connected_components_, self.n_leaves_, parents = out[:4]
        if return_distance:
            self.distances_ = out[-1]
        if self.distance_threshold is not None:
            self.n_clusters_ = int(np.count_nonzero(self.distances_ >= self.distance_threshold)) + 1
        else:
            self.n_clusters_ = self.n_clusters
        if full:
            self.labels_ = _hc_cut(self.n_clusters_, self.children_, self.n_leaves_)
        else:
            heads = np.array(parents, copy=True)
            for node0 in range(len(heads)):
                node = node0
                p = heads[node]
                while p != node:
                    heads[node0] = p
                    node = p
                    p = heads[node]
            lab = heads[:X.shape[0]]
            self.labels_ = np.searchsorted(np.unique(lab), lab)
        return self

    def fit_predict(self, X, y=None):
        return self.fit(X).labels_


class FeatureAgglomeration(AgglomerativeClustering, TransformerMixin):
    """Agglomerates features: clusters the columns, then pools each cluster
    (``pooling_func``, default mean)."""

    def __init__(self, n_clusters=2, *, affinity="euclidean", memory=None, connectivity=None,
                 compute_full_tree="auto", linkage="ward", pooling_func=np.mean,
                 distance_threshold=None, compute_distances=False, device=None):
        super().__init__(n_clusters=n_clusters, memory=memory, connectivity=connectivity,
                         compute_full_tree=compute_full_tree, linkage=linkage, affinity=affinity,
                         distance_threshold=distance_threshold,
                         compute_distances=compute_distances, device=device)
        self.pooling_func = pooling_func

    def fit(self, X, y=None, **params):
        X = check_array(X, ensure_min_features=2)
        super().fit(X.T)
        self.n_features_in_ = X.shape[1]
        return self

    @property
    def fit_predict(self):
        raise AttributeError

    def transform(self, X):
        check_is_fitted(self)
        X = check_array(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError(f"X has {X.shape[1]} features, but FeatureAgglomeration is "
                             f"expecting {self.n_features_in_} features as input.")
        if self.pooling_func == np.mean:
            size = np.bincount(self.labels_)
            n_samples = X.shape[0]
            nX = np.array([np.bincount(self.labels_, X[i, :]) / size for i in range(n_samples)])
        else:
            nX = [self.pooling_func(X[:, self.labels_ == l], axis=1)
                  for l in np.unique(self.labels_)]
            nX = np.array(nX).T
        return nX

    def inverse_transform(self, Xred):
        check_is_fitted(self)
        unil, inverse = np.unique(self.labels_, return_inverse=True)
        return Xred[..., inverse]
