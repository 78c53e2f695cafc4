"""Remaining clustering estimators (reference ``sklearn/cluster``):
``AffinityPropagation`` (``_affinity_propagation.py``), ``MeanShift``
(``_mean_shift.py``), ``Birch`` (``_birch.py``), ``OPTICS``
(``_optics.py``) and ``SpectralClustering`` (``_spectral.py``).

MI355X mapping:
* affinity propagation's responsibility / availability sweeps are dense
  n x n fp64 tensor updates on the device (one host sync per convergence
  check);
* mean shift runs all seeds at once on the device - every iteration is a
  seeds x samples distance GEMM and a masked mean;
* the OPTICS ordering is host C++ (``sqh_optics_order``, OpenMP relaxation
  of the reachabilities), the xi cluster extraction stays in numpy;
* Birch's CF-tree is inherently sequential (host).
"""

import ctypes
import numbers
import warnings
from collections import defaultdict

import numpy as np
import scipy.sparse as sp
import torch

from ...base import BaseEstimator, ClusterMixin, TransformerMixin
from ...exceptions import ConvergenceWarning
from ...ops import _host
from ...runtime.device import resolve_device
from ...utils.validation import check_is_fitted, check_random_state


def _dense(X):
    if hasattr(X, "detach"):
        X = X.detach().cpu().numpy()
    return np.asarray(X.toarray() if sp.issparse(X) else X, dtype=np.float64)


def _c(a):
    return ctypes.c_void_p(a.ctypes.data)


def _sq_dists(A, B):
    """Squared euclidean distances, fp64 on the device, as numpy."""
    dev = resolve_device(None)
    a = torch.as_tensor(A, dtype=torch.float64, device=dev)
    b = torch.as_tensor(B, dtype=torch.float64, device=dev)
    D = (a * a).sum(1)[:, None] + (b * b).sum(1)[None, :] - 2.0 * a @ b.T
    return D.clamp_(min=0).cpu().numpy()


# ------------------------------------------------------ AffinityPropagation
def affinity_propagation(S, *, preference=None, convergence_iter=15, max_iter=200, damping=0.5,
                         copy=True, verbose=False, return_n_iter=False, random_state=0):
    S = np.array(S, dtype=np.float64, copy=True)
    n = S.shape[0]
    if S.shape[0] != S.shape[1]:
        raise ValueError("S must be a square array (shape=%s)" % repr(S.shape))
    if preference is None:
        preference = np.median(S)
    if damping < 0.5 or damping >= 1:
        raise ValueError("damping must be >= 0.5 and < 1")
    pref = np.asarray(preference)
    if n == 1 or (np.all(S[~np.eye(n, dtype=bool)] == S[0, 1] if n > 1 else True)
                  and np.all(pref == pref.flat[0])):
        warnings.warn("All samples have mutually equal similarities. Returning arbitrary "
                      "cluster center(s).")
        if pref.flat[0] > (S[0, 1] if n > 1 else -np.inf):
            out = (np.arange(n), np.arange(n))
        else:
            out = (np.array([0]), np.array([0] * n))
        return out + ((0,) if return_n_iter else ())
    rs = check_random_state(random_state)
    S.flat[::n + 1] = preference
    S += (np.finfo(S.dtype).eps * S + np.finfo(S.dtype).tiny * 100) * rs.randn(n, n)
    dev = resolve_device(None)
    St = torch.as_tensor(S, device=dev)
    A = torch.zeros_like(St)
    R = torch.zeros_like(St)
    ar = torch.arange(n, device=dev)
    e = torch.zeros((n, convergence_iter), dtype=torch.bool, device=dev)
    never = True
    it = 0
    for it in range(max_iter):
        T = A + St
        Imax = torch.argmax(T, dim=1)
        Y = T[ar, Imax]
        T[ar, Imax] = -float("inf")
        Y2 = T.max(dim=1).values
        T = St - Y[:, None]
        T[ar, Imax] = St[ar, Imax] - Y2
        R = damping * R + (1 - damping) * T
        T = R.clamp(min=0)
        T.diagonal().copy_(R.diagonal())
        T = T - T.sum(dim=0, keepdim=True)
        dA = T.diagonal().clone()
        T = T.clamp(min=0)
        T.diagonal().copy_(dA)
        A = damping * A - (1 - damping) * T
        E = (A.diagonal() + R.diagonal()) > 0
        e[:, it % convergence_iter] = E
        K = int(E.sum())
        if it >= convergence_iter:
            se = e.sum(dim=1)
            unconverged = int(((se == convergence_iter) | (se == 0)).sum()) != n
            if (not unconverged and K > 0) or it == max_iter:
                never = False
                break
    E = E.cpu().numpy()
    I = np.flatnonzero(E)
    K = I.size
    if K > 0 and not never:
        c = np.argmax(S[:, I], axis=1)
        c[I] = np.arange(K)
        for k in range(K):
            ii = np.where(c == k)[0]
            I[k] = ii[np.argmax(np.sum(S[ii[:, np.newaxis], ii], axis=0))]
        c = np.argmax(S[:, I], axis=1)
        c[I] = np.arange(K)
        labels = I[c]
        centers = np.unique(labels)
        labels = np.searchsorted(centers, labels)
    else:
        warnings.warn("Affinity propagation did not converge, this model will not have any "
                      "cluster centers.", ConvergenceWarning)
        labels = np.array([-1] * n)
        centers = []
    return (centers, labels, it + 1) if return_n_iter else (centers, labels)


class AffinityPropagation(ClusterMixin, BaseEstimator):
    def __init__(self, *, damping=0.5, max_iter=200, convergence_iter=15, copy=True,
                 preference=None, affinity="euclidean", verbose=False, random_state=None):
        self.damping = damping
        self.max_iter = max_iter
        self.convergence_iter = convergence_iter
        self.copy = copy
        self.verbose = verbose
        self.preference = preference
        self.affinity = affinity
        self.random_state = random_state

    def fit(self, X, y=None):
        if self.affinity == "precomputed":
            X = _dense(X)
            self.affinity_matrix_ = X.copy()
        elif self.affinity == "euclidean":
            X = _dense(X)
            self.affinity_matrix_ = -_sq_dists(X, X)
        else:
            raise ValueError("Affinity must be 'precomputed' or 'euclidean'. Got %s instead"
                             % str(self.affinity))
        self.n_features_in_ = X.shape[1]
        rs = 0 if self.random_state is None else self.random_state
        self.cluster_centers_indices_, self.labels_, self.n_iter_ = affinity_propagation(
            self.affinity_matrix_, preference=self.preference, max_iter=self.max_iter,
            convergence_iter=self.convergence_iter, damping=self.damping, copy=self.copy,
            return_n_iter=True, random_state=rs)
        if self.affinity != "precomputed":
            self.cluster_centers_ = X[self.cluster_centers_indices_].copy()
        return self

    def predict(self, X):
        check_is_fitted(self, "cluster_centers_indices_")
        if self.affinity == "precomputed":
            raise ValueError("Predict method is not supported when affinity='precomputed'.")
        X = _dense(X)
        if len(self.cluster_centers_) > 0:
            return np.argmin(_sq_dists(X, self.cluster_centers_), axis=1)
        warnings.warn("This model does not have any cluster centers because affinity "
                      "propagation did not converge. Labeling every sample as '-1'.",
                      ConvergenceWarning)
        return np.array([-1] * X.shape[0])

    def fit_predict(self, X, y=None):
        return self.fit(X).labels_


# ---------------------------------------------------------------- MeanShift
def estimate_bandwidth(X, *, quantile=0.3, n_samples=None, random_state=0, n_jobs=None):
    from ..neighbors import NearestNeighbors
    X = _dense(X)
    rs = check_random_state(random_state)
    if n_samples is not None:
        X = X[rs.permutation(X.shape[0])[:n_samples]]
    k = max(1, int(X.shape[0] * quantile))
    nn = NearestNeighbors(n_neighbors=k).fit(X)
    bw = 0.0
    for s in range(0, len(X), 500):
        d, _ = nn.kneighbors(X[s:s + 500], return_distance=True)
        bw += np.max(np.asarray(d), axis=1).sum()
    return bw / X.shape[0]


def get_bin_seeds(X, bin_size, min_bin_freq=1):
    if bin_size == 0:
        return X
    sizes = defaultdict(int)
    for pt in X:
        sizes[tuple(np.round(pt / bin_size))] += 1
    seeds = np.array([p for p, f in sizes.items() if f >= min_bin_freq], dtype=np.float32)
    if len(seeds) == len(X):
        warnings.warn("Binning data failed with provided bin_size=%f, using data points as "
                      "seeds." % bin_size)
        return X
    return seeds * bin_size


def _shift_all(seeds, X, bw, max_iter):
    """Iterate every seed to its mode on the device; returns (modes,
    window counts, iterations)."""
    dev = resolve_device(None)
    Xt = torch.as_tensor(X, dtype=torch.float64, device=dev)
    xn = (Xt * Xt).sum(1)
    M = torch.as_tensor(np.asarray(seeds, dtype=np.float64), device=dev).clone()
    m = M.shape[0]
    active = torch.ones(m, dtype=torch.bool, device=dev)
    counts = torch.zeros(m, dtype=torch.int64, device=dev)
    iters = torch.zeros(m, dtype=torch.int64, device=dev)
    stop = 1e-3 * bw
    for _ in range(max_iter + 1):
        idx = torch.nonzero(active).flatten()
        if idx.numel() == 0:
            break
        q = M[idx]
        D = ((q * q).sum(1)[:, None] + xn[None, :] - 2.0 * q @ Xt.T).clamp_(min=0).sqrt_()
        W = (D <= bw).to(torch.float64)
        cnt = W.sum(1)
        empty = cnt == 0
        new = (W @ Xt) / cnt.clamp(min=1)[:, None]
        shift = torch.linalg.norm(new - q, dim=1)
        new = torch.where(empty[:, None], q, new)
        M[idx] = new
        counts[idx] = cnt.to(torch.int64)
        done = empty | (shift < stop) | (iters[idx] == max_iter)
        iters[idx] = torch.where(done, iters[idx], iters[idx] + 1)
        active[idx[done]] = False
    return M.cpu().numpy(), counts.cpu().numpy(), iters.cpu().numpy()


def mean_shift(X, *, bandwidth=None, seeds=None, bin_seeding=False, min_bin_freq=1,
               cluster_all=True, max_iter=300, n_jobs=None):
    m = MeanShift(bandwidth=bandwidth, seeds=seeds, min_bin_freq=min_bin_freq,
                  bin_seeding=bin_seeding, cluster_all=cluster_all, n_jobs=n_jobs,
                  max_iter=max_iter).fit(X)
    return m.cluster_centers_, m.labels_


class MeanShift(ClusterMixin, BaseEstimator):
    def __init__(self, *, bandwidth=None, seeds=None, bin_seeding=False, min_bin_freq=1,
                 cluster_all=True, n_jobs=None, max_iter=300):
        self.bandwidth = bandwidth
        self.seeds = seeds
        self.bin_seeding = bin_seeding
        self.cluster_all = cluster_all
        self.min_bin_freq = min_bin_freq
        self.n_jobs = n_jobs
        self.max_iter = max_iter

    def fit(self, X, y=None):
        X = _dense(X)
        self.n_features_in_ = X.shape[1]
        bw = self.bandwidth if self.bandwidth is not None else estimate_bandwidth(X)
        if bw <= 0:
            raise ValueError("bandwidth needs to be greater than zero or None, got %f" % bw)
        seeds = self.seeds
        if seeds is None:
            seeds = get_bin_seeds(X, bw, self.min_bin_freq) if self.bin_seeding else X
        modes, counts, iters = _shift_all(seeds, X, bw, self.max_iter)
        centers = {}
        for mode, cnt in zip(modes, counts):
            if cnt:
                centers[tuple(mode)] = int(cnt)
        self.n_iter_ = int(iters.max()) if len(iters) else 0
        if not centers:
            raise ValueError("No point was within bandwidth=%f of any seed. Try a different "
                             "seeding strategy or increase the bandwidth." % bw)
        ranked = sorted(centers.items(), key=lambda t: (t[1], t[0]), reverse=True)
        sc = np.array([t[0] for t in ranked])
        D = np.sqrt(_sq_dists(sc, sc))
        unique = np.ones(len(sc), dtype=bool)
        for i in range(len(sc)):
            if unique[i]:
                unique[D[i] <= bw] = False
                unique[i] = True
        cc = sc[unique]
        D = np.sqrt(_sq_dists(X, cc))
        idx = np.argmin(D, axis=1)
        if self.cluster_all:
            labels = idx
        else:
            labels = np.full(X.shape[0], -1)
            ok = D[np.arange(X.shape[0]), idx] <= bw
            labels[ok] = idx[ok]
        self.cluster_centers_, self.labels_ = cc, labels
        return self

    def predict(self, X):
        check_is_fitted(self, "cluster_centers_")
        return np.argmin(_sq_dists(_dense(X), self.cluster_centers_), axis=1)


# -------------------------------------------------------------------- Birch
class _CFSubcluster:
    __slots__ = ("n_samples_", "squared_sum_", "linear_sum_", "centroid_", "sq_norm_", "child_")

    def __init__(self, *, linear_sum=None):
        if linear_sum is None:
            self.n_samples_, self.squared_sum_ = 0, 0.0
            self.centroid_ = self.linear_sum_ = 0
        else:
            self.n_samples_ = 1
            self.centroid_ = self.linear_sum_ = linear_sum
            self.squared_sum_ = self.sq_norm_ = np.dot(linear_sum, linear_sum)
        self.child_ = None

    def update(self, sub):
        self.n_samples_ += sub.n_samples_
        self.linear_sum_ = self.linear_sum_ + sub.linear_sum_
        self.squared_sum_ += sub.squared_sum_
        self.centroid_ = self.linear_sum_ / self.n_samples_
        self.sq_norm_ = np.dot(self.centroid_, self.centroid_)

    def merge_subcluster(self, nom, threshold):
        ss = self.squared_sum_ + nom.squared_sum_
        ls = self.linear_sum_ + nom.linear_sum_
        n = self.n_samples_ + nom.n_samples_
        c = (1 / n) * ls
        sqn = np.dot(c, c)
        if ss / n - sqn <= threshold ** 2:
            self.n_samples_, self.linear_sum_, self.squared_sum_ = n, ls, ss
            self.centroid_, self.sq_norm_ = c, sqn
            return True
        return False

    @property
    def radius(self):
        return np.sqrt(max(0, self.squared_sum_ / self.n_samples_ - self.sq_norm_))


class _CFNode:
    def __init__(self, *, threshold, branching_factor, is_leaf, n_features):
        self.threshold = threshold
        self.branching_factor = branching_factor
        self.is_leaf = is_leaf
        self.n_features = n_features
        self.subclusters_ = []
        self.init_centroids_ = np.zeros((branching_factor + 1, n_features))
        self.init_sq_norm_ = np.zeros(branching_factor + 1)
        self.squared_norm_ = []
        self.prev_leaf_ = None
        self.next_leaf_ = None

    def append_subcluster(self, sub):
        n = len(self.subclusters_)
        self.subclusters_.append(sub)
        self.init_centroids_[n] = sub.centroid_
        self.init_sq_norm_[n] = sub.sq_norm_
        self.centroids_ = self.init_centroids_[:n + 1, :]
        self.squared_norm_ = self.init_sq_norm_[:n + 1]

    def update_split_subclusters(self, sub, new1, new2):
        i = self.subclusters_.index(sub)
        self.subclusters_[i] = new1
        self.init_centroids_[i] = new1.centroid_
        self.init_sq_norm_[i] = new1.sq_norm_
        self.append_subcluster(new2)

    def insert_cf_subcluster(self, sub):
        if not self.subclusters_:
            self.append_subcluster(sub)
            return False
        d = -2.0 * (self.centroids_ @ sub.centroid_) + self.squared_norm_
        ci = int(np.argmin(d))
        closest = self.subclusters_[ci]
        if closest.child_ is not None:
            split = closest.child_.insert_cf_subcluster(sub)
            if not split:
                closest.update(sub)
                self.init_centroids_[ci] = self.subclusters_[ci].centroid_
                self.init_sq_norm_[ci] = self.subclusters_[ci].sq_norm_
                return False
            n1, n2 = _split_node(closest.child_, self.threshold, self.branching_factor)
            self.update_split_subclusters(closest, n1, n2)
            return len(self.subclusters_) > self.branching_factor
        if closest.merge_subcluster(sub, self.threshold):
            self.init_centroids_[ci] = closest.centroid_
            self.init_sq_norm_[ci] = closest.sq_norm_
            return False
        self.append_subcluster(sub)
        return len(self.subclusters_) > self.branching_factor


def _split_node(node, threshold, branching_factor):
    s1, s2 = _CFSubcluster(), _CFSubcluster()
    kw = dict(threshold=threshold, branching_factor=branching_factor, is_leaf=node.is_leaf,
              n_features=node.n_features)
    n1, n2 = _CFNode(**kw), _CFNode(**kw)
    s1.child_, s2.child_ = n1, n2
    if node.is_leaf:
        if node.prev_leaf_ is not None:
            node.prev_leaf_.next_leaf_ = n1
        n1.prev_leaf_, n1.next_leaf_ = node.prev_leaf_, n2
        n2.prev_leaf_, n2.next_leaf_ = n1, node.next_leaf_
        if node.next_leaf_ is not None:
            node.next_leaf_.prev_leaf_ = n2
    C = node.centroids_
    sq = node.squared_norm_
    D = sq[:, None] - 2.0 * (C @ C.T) + sq[None, :]
    np.maximum(D, 0, out=D)
    np.fill_diagonal(D, 0)
    far = np.unravel_index(D.argmax(), D.shape)
    d1, d2 = D[(far,)]
    closer1 = d1 < d2
    for i, sub in enumerate(node.subclusters_):
        if closer1[i]:
            n1.append_subcluster(sub)
            s1.update(sub)
        else:
            n2.append_subcluster(sub)
            s2.update(sub)
    return s1, s2


class Birch(ClusterMixin, TransformerMixin, BaseEstimator):
    """Balanced iterative reducing and clustering using hierarchies."""

    def __init__(self, *, threshold=0.5, branching_factor=50, n_clusters=3,
                 compute_labels=True, copy=True):
        self.threshold = threshold
        self.branching_factor = branching_factor
        self.n_clusters = n_clusters
        self.compute_labels = compute_labels
        self.copy = copy

    def _fit(self, X, partial):
        first = not (partial and hasattr(self, "root_"))
        X = X.tocsr() if sp.issparse(X) else _dense(X)
        if first:
            self.n_features_in_ = X.shape[1]
        elif X.shape[1] != self.n_features_in_:
            raise ValueError("Training data and predicted data do not have same number of "
                             "features.")
        if self.branching_factor <= 1:
            raise ValueError("Branching_factor should be greater than one.")
        d = X.shape[1]
        if first:
            kw = dict(threshold=self.threshold, branching_factor=self.branching_factor,
                      n_features=d)
            self.root_ = _CFNode(is_leaf=True, **kw)
            self.dummy_leaf_ = _CFNode(is_leaf=True, **kw)
            self.dummy_leaf_.next_leaf_ = self.root_
            self.root_.prev_leaf_ = self.dummy_leaf_
        rows = (X[i].toarray().ravel() for i in range(X.shape[0])) if sp.issparse(X) else iter(X)
        for row in rows:
            split = self.root_.insert_cf_subcluster(_CFSubcluster(linear_sum=row))
            if split:
                s1, s2 = _split_node(self.root_, self.threshold, self.branching_factor)
                self.root_ = _CFNode(threshold=self.threshold,
                                     branching_factor=self.branching_factor, is_leaf=False,
                                     n_features=d)
                self.root_.append_subcluster(s1)
                self.root_.append_subcluster(s2)
        self.subcluster_centers_ = np.concatenate([lf.centroids_ for lf in self._get_leaves()])
        self._subcluster_norms = (self.subcluster_centers_ ** 2).sum(1)
        self._global_clustering(X)
        return self

    def _get_leaves(self):
        p = self.dummy_leaf_.next_leaf_
        out = []
        while p is not None:
            out.append(p)
            p = p.next_leaf_
        return out

    def fit(self, X, y=None):
        return self._fit(X, partial=False)

    def partial_fit(self, X=None, y=None):
        if X is None:
            self._global_clustering()
            return self
        return self._fit(X, partial=True)

    def _global_clustering(self, X=None):
        from .hierarchical import AgglomerativeClustering
        clusterer = self.n_clusters
        C = self.subcluster_centers_
        too_few = False
        if isinstance(clusterer, numbers.Integral):
            clusterer = AgglomerativeClustering(n_clusters=self.n_clusters)
            too_few = len(C) < self.n_clusters
        elif clusterer is not None and not hasattr(clusterer, "fit_predict"):
            raise ValueError("n_clusters should be an instance of ClusterMixin or an int")
        if clusterer is None or too_few:
            self.subcluster_labels_ = np.arange(len(C))
            if too_few:
                warnings.warn("Number of subclusters found (%d) by BIRCH is less than "
                              "(%d). Decrease the threshold." % (len(C), self.n_clusters),
                              ConvergenceWarning)
        else:
            self.subcluster_labels_ = np.asarray(clusterer.fit_predict(C))
        if X is not None and self.compute_labels:
            self.labels_ = self.predict(X)

    def predict(self, X):
        check_is_fitted(self, "subcluster_centers_")
        X = _dense(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError("X has %d features, but Birch is expecting %d features as input."
                             % (X.shape[1], self.n_features_in_))
        D = -2.0 * X @ self.subcluster_centers_.T + self._subcluster_norms[None, :]
        return self.subcluster_labels_[np.argmin(D, axis=1)]

    def transform(self, X):
        check_is_fitted(self, "subcluster_centers_")
        X = _dense(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError("X has %d features, but Birch is expecting %d features as input."
                             % (X.shape[1], self.n_features_in_))
        return np.sqrt(_sq_dists(X, self.subcluster_centers_))


# ------------------------------------------------------------------- OPTICS
def _validate_size(size, n, name):
    if size <= 0 or (size != int(size) and size > 1):
        raise ValueError("%s must be a positive integer or a float between 0 and 1. Got %r"
                         % (name, size))
    if size > n:
        raise ValueError("%s must be no greater than the number of samples (%d). Got %d"
                         % (name, n, size))


def compute_optics_graph(X, *, min_samples, max_eps, metric, p, metric_params, algorithm,
                         leaf_size, n_jobs):
    from ..neighbors import NearestNeighbors
    X = _dense(X)
    n = X.shape[0]
    _validate_size(min_samples, n, "min_samples")
    if min_samples <= 1:
        min_samples = max(2, int(min_samples * n))
    # core distances: trees compute direct differences (as the reference's
    # auto/kd_tree choice for low dimension does); brute uses the GEMM form
    algo = "kd_tree" if algorithm == "auto" else algorithm
    nn = NearestNeighbors(n_neighbors=min_samples, algorithm=algo, leaf_size=leaf_size,
                          metric=metric, metric_params=metric_params, p=p).fit(X)
    core = np.asarray(nn.kneighbors(X, min_samples)[0], dtype=np.float64)[:, -1].copy()
    core[core > max_eps] = np.inf
    np.around(core, decimals=np.finfo(core.dtype).precision, out=core)
    from ..neighbors._extra import _tree_p
    pp = _tree_p(metric, p, metric_params)
    if pp is None:
        raise ValueError("OPTICS supports minkowski-family metrics (got %r)" % metric)
    reach = np.empty(n)
    pred = np.empty(n, dtype=np.int64)
    order = np.empty(n, dtype=np.int64)
    Xc = np.ascontiguousarray(X)
    core = np.ascontiguousarray(core)
    _host.lib().sqh_optics_order(_c(Xc), n, X.shape[1], _c(core), float(max_eps), float(pp),
                                 _c(reach), _c(pred), _c(order))
    if np.all(np.isinf(reach)):
        warnings.warn("All reachability values are inf. Set a larger max_eps or all data will "
                      "be considered outliers.", UserWarning)
    return order, core, reach, pred


def cluster_optics_dbscan(*, reachability, core_distances, ordering, eps):
    n = len(core_distances)
    labels = np.zeros(n, dtype=int)
    far = reachability > eps
    near = core_distances <= eps
    labels[ordering] = np.cumsum(far[ordering] & near[ordering]) - 1
    labels[far & ~near] = -1
    return labels


def _extend_region(steep, xward, start, min_samples):
    n = len(steep)
    non = 0
    end = start
    for i in range(start, n):
        if steep[i]:
            non = 0
            end = i
        elif not xward[i]:
            non += 1
            if non > min_samples:
                break
        else:
            return end
    return end


def _filter_sdas(sdas, mib, xc, rp):
    if np.isinf(mib):
        return []
    keep = [s for s in sdas if mib <= rp[s["start"]] * xc]
    for s in keep:
        s["mib"] = max(s["mib"], mib)
    return keep


def _correct_predecessor(rp, pp, ordering, s, e):
    while s < e:
        if rp[s] > rp[e]:
            return s, e
        pe = ordering[pp[e]]
        if any(pe == ordering[i] for i in range(s, e)):
            return s, e
        e -= 1
    return None, None


def _xi_cluster(rp, pp, ordering, xi, min_samples, min_cluster_size, correction):
    rp = np.hstack((rp, np.inf))
    xc = 1 - xi
    sdas, clusters = [], []
    index, mib = 0, 0.0
    with np.errstate(invalid="ignore"):
        ratio = rp[:-1] / rp[1:]
        up_steep = ratio <= xc
        down_steep = ratio >= 1 / xc
        down = ratio > 1
        up = ratio < 1
    for si in np.flatnonzero(up_steep | down_steep):
        if si < index:
            continue
        mib = max(mib, np.max(rp[index:si + 1]))
        if down_steep[si]:
            sdas = _filter_sdas(sdas, mib, xc, rp)
            d_end = _extend_region(down_steep, up, si, min_samples)
            sdas.append({"start": si, "end": d_end, "mib": 0.0})
            index = d_end + 1
            mib = rp[index]
            continue
        sdas = _filter_sdas(sdas, mib, xc, rp)
        u_start = si
        u_end = _extend_region(up_steep, down, si, min_samples)
        index = u_end + 1
        mib = rp[index]
        found = []
        for D in sdas:
            cs, ce = D["start"], u_end
            if rp[ce + 1] * xc < D["mib"]:
                continue
            dmax = rp[D["start"]]
            if dmax * xc >= rp[ce + 1]:
                while rp[cs + 1] > rp[ce + 1] and cs < D["end"]:
                    cs += 1
            elif rp[ce + 1] * xc >= dmax:
                while rp[ce - 1] > dmax and ce > u_start:
                    ce -= 1
            if correction:
                cs, ce = _correct_predecessor(rp, pp, ordering, cs, ce)
            if cs is None or ce - cs + 1 < min_cluster_size or cs > D["end"] or ce < u_start:
                continue
            found.append((cs, ce))
        clusters.extend(found[::-1])
    return np.array(clusters)


def _extract_xi_labels(ordering, clusters):
    labels = np.full(len(ordering), -1, dtype=int)
    lab = 0
    for c in clusters:
        if not np.any(labels[c[0]:c[1] + 1] != -1):
            labels[c[0]:c[1] + 1] = lab
            lab += 1
    out = np.empty_like(labels)
    out[ordering] = labels
    return out


def cluster_optics_xi(*, reachability, predecessor, ordering, min_samples,
                      min_cluster_size=None, xi=0.05, predecessor_correction=True):
    n = len(reachability)
    _validate_size(min_samples, n, "min_samples")
    if min_samples <= 1:
        min_samples = max(2, int(min_samples * n))
    if min_cluster_size is None:
        min_cluster_size = min_samples
    _validate_size(min_cluster_size, n, "min_cluster_size")
    if min_cluster_size <= 1:
        min_cluster_size = max(2, int(min_cluster_size * n))
    clusters = _xi_cluster(reachability[ordering], predecessor[ordering], ordering, xi,
                           min_samples, min_cluster_size, predecessor_correction)
    return _extract_xi_labels(ordering, clusters), clusters


class OPTICS(ClusterMixin, BaseEstimator):
    """Ordering points to identify the clustering structure."""

    def __init__(self, *, min_samples=5, max_eps=np.inf, metric="minkowski", p=2,
                 metric_params=None, cluster_method="xi", eps=None, xi=0.05,
                 predecessor_correction=True, min_cluster_size=None, algorithm="auto",
                 leaf_size=30, memory=None, n_jobs=None):
        self.max_eps = max_eps
        self.min_samples = min_samples
        self.min_cluster_size = min_cluster_size
        self.algorithm = algorithm
        self.metric = metric
        self.metric_params = metric_params
        self.p = p
        self.leaf_size = leaf_size
        self.cluster_method = cluster_method
        self.eps = eps
        self.xi = xi
        self.predecessor_correction = predecessor_correction
        self.memory = memory
        self.n_jobs = n_jobs

    def fit(self, X, y=None):
        X = _dense(X)
        self.n_features_in_ = X.shape[1]
        if self.cluster_method not in ("dbscan", "xi"):
            raise ValueError("cluster_method should be one of 'dbscan' or 'xi' but is %s"
                             % self.cluster_method)
        self.ordering_, self.core_distances_, self.reachability_, self.predecessor_ = \
            compute_optics_graph(X, min_samples=self.min_samples, algorithm=self.algorithm,
                                 leaf_size=self.leaf_size, metric=self.metric,
                                 metric_params=self.metric_params, p=self.p, n_jobs=self.n_jobs,
                                 max_eps=self.max_eps)
        if self.cluster_method == "xi":
            self.labels_, self.cluster_hierarchy_ = cluster_optics_xi(
                reachability=self.reachability_, predecessor=self.predecessor_,
                ordering=self.ordering_, min_samples=self.min_samples,
                min_cluster_size=self.min_cluster_size, xi=self.xi,
                predecessor_correction=self.predecessor_correction)
        else:
            eps = self.max_eps if self.eps is None else self.eps
            if eps > self.max_eps:
                raise ValueError("Specify an epsilon smaller than %s. Got %s."
                                 % (self.max_eps, eps))
            self.labels_ = cluster_optics_dbscan(reachability=self.reachability_,
                                                 core_distances=self.core_distances_,
                                                 ordering=self.ordering_, eps=eps)
        return self


# -------------------------------------------------------- SpectralClustering
def discretize(vectors, *, copy=True, max_svd_restarts=30, n_iter_max=20, random_state=None):
    from scipy.sparse import csc_matrix
    rs = check_random_state(random_state)
    V = np.array(vectors, dtype=np.float64, copy=True)
    eps = np.finfo(float).eps
    n, k = V.shape
    for i in range(k):
        V[:, i] = V[:, i] / np.linalg.norm(V[:, i]) * np.sqrt(n)
        if V[0, i] != 0:
            V[:, i] = -1 * V[:, i] * np.sign(V[0, i])
    V = V / np.sqrt((V ** 2).sum(axis=1))[:, np.newaxis]
    restarts, converged = 0, False
    labels = None
    while restarts < max_svd_restarts and not converged:
        rot = np.zeros((k, k))
        rot[:, 0] = V[rs.randint(n), :].T
        c = np.zeros(n)
        for j in range(1, k):
            c += np.abs(V @ rot[:, j - 1])
            rot[:, j] = V[c.argmin(), :].T
        last, it = 0.0, 0
        while not converged:
            it += 1
            labels = (V @ rot).argmax(axis=1)
            Vd = csc_matrix((np.ones(len(labels)), (np.arange(n), labels)), shape=(n, k))
            try:
                U, S, Vh = np.linalg.svd(Vd.T @ V)
                restarts += 1
            except np.linalg.LinAlgError:
                break
            ncut = 2.0 * (n - S.sum())
            if abs(ncut - last) < eps or it > n_iter_max:
                converged = True
            else:
                last = ncut
                rot = Vh.T @ U.T
    if not converged:
        raise np.linalg.LinAlgError("SVD did not converge")
    return labels


def spectral_clustering(affinity, *, n_clusters=8, n_components=None, eigen_solver=None,
                        random_state=None, n_init=10, eigen_tol=0.0, assign_labels="kmeans",
                        verbose=False):
    from ..manifold._spectral import spectral_embedding
    from .kmeans import k_means
    if assign_labels not in ("kmeans", "discretize"):
        raise ValueError("The 'assign_labels' parameter should be 'kmeans' or 'discretize', but "
                         "'%s' was given" % assign_labels)
    rs = check_random_state(random_state)
    nc = n_clusters if n_components is None else n_components
    maps = spectral_embedding(affinity, n_components=nc, eigen_solver=eigen_solver,
                              random_state=rs, eigen_tol=eigen_tol, drop_first=False)
    if assign_labels == "kmeans":
        _, labels, _ = k_means(maps, n_clusters, random_state=rs, n_init=n_init)
        return np.asarray(labels)
    return discretize(maps, random_state=rs)


class SpectralClustering(ClusterMixin, BaseEstimator):
    def __init__(self, n_clusters=8, *, eigen_solver=None, n_components=None, random_state=None,
                 n_init=10, gamma=1.0, affinity="rbf", n_neighbors=10, eigen_tol=0.0,
                 assign_labels="kmeans", degree=3, coef0=1, kernel_params=None, n_jobs=None,
                 verbose=False):
        self.n_clusters = n_clusters
        self.eigen_solver = eigen_solver
        self.n_components = n_components
        self.random_state = random_state
        self.n_init = n_init
        self.gamma = gamma
        self.affinity = affinity
        self.n_neighbors = n_neighbors
        self.eigen_tol = eigen_tol
        self.assign_labels = assign_labels
        self.degree = degree
        self.coef0 = coef0
        self.kernel_params = kernel_params
        self.n_jobs = n_jobs
        self.verbose = verbose

    def fit(self, X, y=None):
        Xd = X if sp.issparse(X) else _dense(X)
        self.n_features_in_ = Xd.shape[1]
        if self.affinity == "nearest_neighbors":
            from ..neighbors import kneighbors_graph
            c = kneighbors_graph(Xd, n_neighbors=self.n_neighbors, include_self=True)
            self.affinity_matrix_ = 0.5 * (c + c.T)
        elif self.affinity == "precomputed_nearest_neighbors":
            from ..neighbors import NearestNeighbors
            nn = NearestNeighbors(n_neighbors=self.n_neighbors, metric="precomputed").fit(Xd)
            c = nn.kneighbors_graph(Xd, mode="connectivity")
            self.affinity_matrix_ = 0.5 * (c + c.T)
        elif self.affinity == "precomputed":
            self.affinity_matrix_ = Xd
        else:
            from ...metrics import pairwise_kernels
            params = dict(self.kernel_params or {})
            if not callable(self.affinity):
                params.update(gamma=self.gamma, degree=self.degree, coef0=self.coef0)
                from ..decomposition._extra import _KERNEL_PARAMS
                params = {k: v for k, v in params.items()
                          if k in _KERNEL_PARAMS.get(self.affinity, ())}
            K = pairwise_kernels(Xd, metric=self.affinity, **params)
            self.affinity_matrix_ = np.asarray(K.detach().cpu().numpy() if hasattr(K, "detach")
                                               else K)
        rs = check_random_state(self.random_state)
        self.labels_ = spectral_clustering(self.affinity_matrix_, n_clusters=self.n_clusters,
                                           n_components=self.n_components,
                                           eigen_solver=self.eigen_solver, random_state=rs,
                                           n_init=self.n_init, eigen_tol=self.eigen_tol,
                                           assign_labels=self.assign_labels)
        return self

    def fit_predict(self, X, y=None):
        return self.fit(X).labels_


__all__ = ["AffinityPropagation", "affinity_propagation", "MeanShift", "mean_shift",
           "estimate_bandwidth", "get_bin_seeds", "Birch", "OPTICS", "compute_optics_graph",
           "cluster_optics_dbscan", "cluster_optics_xi", "SpectralClustering",
           "spectral_clustering"]
