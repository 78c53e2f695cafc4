"""Neighbour trees, metrics and the remaining neighbours estimators
(reference ``sklearn/neighbors``: ``_binary_tree.pxi`` / ``_kd_tree.pyx`` /
``_ball_tree.pyx`` (N12), ``_dist_metrics.pyx``, ``_base.py``
radius/graph methods, ``_regression.py`` / ``_classification.py`` radius
estimators, ``_graph.py``, ``_kde.py``, ``_lof.py``,
``_nearest_centroid.py``, ``_nca.py``).

* ``KDTree`` / ``BallTree`` are host C++ (``csrc/host/binary_tree.cpp``,
  OpenMP over query rows) with the reference's node layout.
* Euclidean brute force stays on the GPU (distance GEMM + top-k kernel,
  ``knn.py``); other metrics use the trees or a pairwise matrix.
* ``KernelDensity`` evaluates exactly (atol = rtol = 0 semantics) with a
  chunked device log-sum-exp; ``NeighborhoodComponentsAnalysis`` computes
  its softmax loss/gradient on the device and drives scipy L-BFGS-B.
"""

import ctypes
import os
import warnings
from math import lgamma, log, pi

import numpy as np
import scipy.sparse as sp
import torch
from scipy.optimize import minimize
from scipy.spatial.distance import cdist
from scipy.special import gammainc

from ...base import (BaseEstimator, ClassifierMixin, OutlierMixin, RegressorMixin,
                     TransformerMixin)
from ...ops import _host
from ...runtime.device import resolve_device, to_numpy
from ...utils.validation import check_array, check_is_fitted, check_random_state

_P_OF = {"euclidean": 2.0, "l2": 2.0, "manhattan": 1.0, "cityblock": 1.0, "l1": 1.0,
         "chebyshev": np.inf, "infinity": np.inf}
_SCIPY = {"l2": "euclidean", "l1": "cityblock", "manhattan": "cityblock",
          "infinity": "chebyshev", "p": "minkowski"}


def _is_euclidean(metric, p=2, metric_params=None):
    if metric_params and "p" in metric_params:
        p = metric_params["p"]
    return metric in ("euclidean", "l2") or (metric == "minkowski" and p == 2)


def _tree_p(metric, p, metric_params):
    if metric_params and "p" in metric_params:
        p = metric_params["p"]
    if metric == "minkowski":
        return float(p)
    return _P_OF.get(metric)


def _c(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def _nthreads():
    return int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))


class DistanceMetric:
    """Pairwise distances by metric name (reference _dist_metrics.pyx)."""

    def __init__(self, metric, **kwargs):
        self.metric = metric
        self.kwargs = kwargs

    @classmethod
    def get_metric(cls, metric, **kwargs):
        return cls(metric, **kwargs)

    def pairwise(self, X, Y=None):
        X = np.asarray(X, dtype=np.float64)
        Y = X if Y is None else np.asarray(Y, dtype=np.float64)
        m = _SCIPY.get(self.metric, self.metric)
        kw = dict(self.kwargs)
        if m == "haversine":
            s1 = np.sin(0.5 * (Y[None, :, 0] - X[:, None, 0]))
            s2 = np.sin(0.5 * (Y[None, :, 1] - X[:, None, 1]))
            return 2 * np.arcsin(np.sqrt(s1 ** 2 + np.cos(X[:, None, 0]) * np.cos(Y[None, :, 0])
                                         * s2 ** 2))
        if m == "minkowski" and "p" not in kw:
            kw["p"] = 2
        if m == "mahalanobis" and "V" in kw and "VI" not in kw:
            kw["VI"] = np.linalg.inv(kw.pop("V"))
        return cdist(X, Y, metric=m, **kw)

    def rdist_to_dist(self, rdist):
        p = _tree_p(self.metric, self.kwargs.get("p", 2), None)
        if p is None or np.isinf(p) or p == 1:
            return rdist
        return rdist ** (1.0 / p)

    def dist_to_rdist(self, dist):
        p = _tree_p(self.metric, self.kwargs.get("p", 2), None)
        if p is None or np.isinf(p) or p == 1:
            return dist
        return dist ** p


# --------------------------------------------------------- binary trees
def _log_vn(n):
    return 0.5 * n * log(pi) - lgamma(0.5 * n + 1)


def _log_sn(n):
    return log(2 * pi) + _log_vn(n - 1)


def _log_kernel_norm(h, d, kernel):
    if kernel == "gaussian":
        f = 0.5 * d * log(2 * pi)
    elif kernel == "tophat":
        f = _log_vn(d)
    elif kernel == "epanechnikov":
        f = _log_vn(d) + log(2.0 / (d + 2.0))
    elif kernel == "exponential":
        f = _log_sn(d - 1) + lgamma(d)
    elif kernel == "linear":
        f = _log_vn(d) - log(d + 1.0)
    elif kernel == "cosine":
        f, tmp = 0.0, 2.0 / pi
        for k in range(1, d + 1, 2):
            f += tmp
            tmp *= -(d - k) * (d - k - 1) * (2.0 / pi) ** 2
        with np.errstate(invalid="ignore"):
            f = float(np.log(f)) + _log_sn(d - 1)
    else:
        raise ValueError("kernel = '%s' not recognized" % kernel)
    return -f - d * log(h)


def _log_kernel(D, h, kernel):
    """log K(d/h) elementwise on a torch tensor of distances."""
    u = D / h
    neg = torch.full_like(D, -np.inf)
    if kernel == "gaussian":
        return -0.5 * u * u
    if kernel == "tophat":
        return torch.where(u < 1, torch.zeros_like(D), neg)
    if kernel == "epanechnikov":
        return torch.where(u < 1, torch.log((1 - u * u).clamp(min=1e-300)), neg)
    if kernel == "exponential":
        return -u
    if kernel == "linear":
        return torch.where(u < 1, torch.log((1 - u).clamp(min=1e-300)), neg)
    if kernel == "cosine":
        return torch.where(u < 1, torch.log(torch.cos(0.5 * pi * u).clamp(min=1e-300)), neg)
    raise ValueError("kernel = '%s' not recognized" % kernel)


class _BinaryTree:
    _kind = 0
    valid_metrics = ["euclidean", "l2", "minkowski", "p", "manhattan", "cityblock", "l1",
                     "chebyshev", "infinity"]

    def __init__(self, X, leaf_size=40, metric="minkowski", sample_weight=None, **kwargs):
        self.data = np.ascontiguousarray(check_array(X), dtype=np.float64)
        self.leaf_size = leaf_size
        self.metric = metric
        self.kwargs = kwargs
        self.sample_weight = None if sample_weight is None else \
            np.asarray(sample_weight, dtype=np.float64)
        p = kwargs.get("p", 2)
        self._p = _tree_p("minkowski" if metric == "p" else metric, p, None)
        if self._p is None:
            raise ValueError("metric %r is not valid for %s" % (metric, type(self).__name__))
        if leaf_size < 1:
            raise ValueError("leaf_size must be greater than or equal to 1")
        self._build()

    def _build(self):
        n, d = self.data.shape
        self._h = _host.lib().sqh_btree_build(_c(self.data), n, d, int(self.leaf_size),
                                              self._kind, float(self._p))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                _host.lib().sqh_btree_free(h)
            except Exception:  # interpreter shutdown
                pass
            self._h = None

    def __getstate__(self):
        return {k: v for k, v in self.__dict__.items() if k != "_h"}

    def __setstate__(self, state):
        self.__dict__.update(state)
        self._build()

    def get_arrays(self):
        lib = _host.lib()
        info = np.zeros(2, dtype=np.int64)
        lib.sqh_btree_info(self._h, _c(info))
        nn, nb = int(info[0]), int(info[1])
        idx = np.empty(self.data.shape[0], dtype=np.int64)
        start, end = np.empty(nn, np.int64), np.empty(nn, np.int64)
        leaf, rad = np.empty(nn, np.uint8), np.empty(nn)
        bounds = np.empty(nb)
        lib.sqh_btree_copy(self._h, _c(idx), _c(start), _c(end), _c(leaf), _c(rad), _c(bounds))
        d = self.data.shape[1]
        node_data = np.zeros(nn, dtype=[("idx_start", np.intp), ("idx_end", np.intp),
                                        ("is_leaf", np.intp), ("radius", np.float64)])
        node_data["idx_start"], node_data["idx_end"] = start, end
        node_data["is_leaf"], node_data["radius"] = leaf, rad
        nb_shape = (2, nn, d) if self._kind == 0 else (1, nn, d)
        if self._kind == 0:
            b = bounds.reshape(nn, 2, d).transpose(1, 0, 2)
        else:
            b = bounds.reshape(1, nn, d)
        return self.data, idx, node_data, b.reshape(nb_shape)

    def query(self, X, k=1, return_distance=True, dualtree=False, breadth_first=False,
              sort_results=True):
        X = np.ascontiguousarray(check_array(X), dtype=np.float64)
        if X.shape[1] != self.data.shape[1]:
            raise ValueError("query data dimension must match training data dimension")
        if self.data.shape[0] < k:
            raise ValueError("k must be less than or equal to the number of training points")
        m = X.shape[0]
        dist = np.empty((m, k))
        ind = np.empty((m, k), dtype=np.int64)
        _host.lib().sqh_btree_knn(self._h, _c(X), m, int(k), _c(dist), _c(ind), _nthreads())
        return (dist, ind) if return_distance else ind

    def query_radius(self, X, r, return_distance=False, count_only=False, sort_results=False):
        if count_only and return_distance:
            raise ValueError("count_only and return_distance cannot both be true")
        if sort_results and not return_distance:
            raise ValueError("return_distance must be True if sort_results is True")
        X = np.ascontiguousarray(check_array(X), dtype=np.float64)
        m = X.shape[0]
        r = np.ascontiguousarray(np.broadcast_to(np.asarray(r, dtype=np.float64), (m,)))
        counts = np.empty(m, dtype=np.int64)
        lib = _host.lib()
        res = lib.sqh_btree_radius(self._h, _c(X), m, _c(r), int(count_only),
                                   int(return_distance), int(sort_results), _c(counts),
                                   _nthreads())
        if count_only:
            return counts
        total = int(counts.sum())
        ind = np.empty(total, dtype=np.int64)
        dist = np.empty(total) if return_distance else None
        lib.sqh_radius_copy(res, _c(ind), _c(dist))
        lib.sqh_radius_free(res)
        splits = np.cumsum(counts)[:-1]
        ind_o = np.empty(m, dtype=object)
        ind_o[:] = np.split(ind, splits)
        if return_distance:
            dist_o = np.empty(m, dtype=object)
            dist_o[:] = np.split(dist, splits)
            return ind_o, dist_o
        return ind_o

    def kernel_density(self, X, h, kernel="gaussian", atol=0, rtol=1e-8, breadth_first=True,
                       return_log=False):
        X = np.asarray(check_array(X), dtype=np.float64)
        logd = _exact_log_density(X, self.data, self.sample_weight, h, kernel,
                                  self.metric, self.kwargs)
        logd += _log_kernel_norm(h, self.data.shape[1], kernel)
        return logd if return_log else np.exp(logd)

    def two_point_correlation(self, X, r, dualtree=False):
        r = np.atleast_1d(np.asarray(r, dtype=np.float64))
        X = np.asarray(check_array(X), dtype=np.float64)
        return np.array([int(self.query_radius(X, ri, count_only=True).sum()) for ri in r])

    def get_n_calls(self):
        return 0


class KDTree(_BinaryTree):
    """KD-tree for fast nearest-neighbour queries."""
    _kind = 0


class BallTree(_BinaryTree):
    """Ball tree for fast nearest-neighbour queries."""
    _kind = 1


def _exact_log_density(Q, Xd, sw, h, kernel, metric="euclidean", kwargs=None):
    dev = resolve_device(None)
    Xt = torch.as_tensor(Xd, dtype=torch.float64, device=dev)
    lw = None if sw is None else torch.log(torch.as_tensor(sw, dtype=torch.float64, device=dev))
    out = np.empty(Q.shape[0])
    rows = max(1, int(2 ** 26 // max(1, Xd.shape[0])))
    euclid = _is_euclidean(metric, (kwargs or {}).get("p", 2))
    for s in range(0, Q.shape[0], rows):
        q = Q[s:s + rows]
        if euclid:
            qt = torch.as_tensor(q, dtype=torch.float64, device=dev)
            D = torch.cdist(qt, Xt)
        else:
            D = torch.as_tensor(DistanceMetric(metric, **(kwargs or {})).pairwise(q, Xd),
                                device=dev)
        L = _log_kernel(D, h, kernel)
        if lw is not None:
            L = L + lw[None, :]
        out[s:s + rows] = torch.logsumexp(L, dim=1).cpu().numpy()
    return out


# ----------------------------------------------------- host engine for knn.py
class _HostEngine:
    """kneighbors / radius_neighbors on the host for non-euclidean metrics
    or explicit tree algorithms."""

    def __init__(self, X, algorithm, metric, p, metric_params, leaf_size):
        self.X = np.ascontiguousarray(X, dtype=np.float64)
        self.metric, self.p, self.metric_params = metric, p, metric_params
        tp = _tree_p(metric, p, metric_params)
        if algorithm in ("kd_tree", "ball_tree") and tp is None and algorithm == "kd_tree":
            raise ValueError("Metric '%s' not valid for algorithm 'kd_tree'" % metric)
        if algorithm == "brute" or (algorithm == "auto" and tp is None) or tp is None:
            self.method, self.tree = "brute", None
        else:
            cls = BallTree if algorithm == "ball_tree" else KDTree
            self.method = "ball_tree" if cls is BallTree else "kd_tree"
            self.tree = cls(self.X, leaf_size=leaf_size,
                            metric="minkowski", p=tp if not np.isinf(tp) else np.inf)

    def _pairwise(self, Q):
        kw = dict(self.metric_params or {})
        if self.metric == "minkowski":
            kw.setdefault("p", self.p)
        return DistanceMetric(self.metric, **kw).pairwise(Q, self.X)

    def kneighbors(self, X, k, return_distance):
        train = X is None
        Q = self.X if train else np.asarray(to_numpy(X), dtype=np.float64)
        kk = k + 1 if train else k
        if kk > self.X.shape[0]:
            raise ValueError(f"Expected n_neighbors <= n_samples, but n_samples = "
                             f"{self.X.shape[0]}, n_neighbors = {kk}")
        if self.tree is not None:
            dist, ind = self.tree.query(Q, kk)
        else:
            D = self._pairwise(Q)
            ind = np.argsort(D, axis=1, kind="stable")[:, :kk]
            dist = np.take_along_axis(D, ind, axis=1)
        if train:
            keep = np.ones_like(ind, dtype=bool)
            selfpos = ind == np.arange(ind.shape[0])[:, None]
            first = np.where(selfpos.any(1), selfpos.argmax(1), kk - 1)
            keep[np.arange(ind.shape[0]), first] = False
            ind = ind[keep].reshape(ind.shape[0], k)
            dist = dist[keep].reshape(dist.shape[0], k)
        return (dist, ind) if return_distance else ind

    def radius(self, X, r, return_distance, sort_results):
        train = X is None
        Q = self.X if train else np.asarray(to_numpy(X), dtype=np.float64)
        if self.tree is not None:
            ind, dist = self.tree.query_radius(Q, r, return_distance=True,
                                               sort_results=sort_results)
        else:
            D = self._pairwise(Q)
            ind = np.empty(Q.shape[0], dtype=object)
            dist = np.empty(Q.shape[0], dtype=object)
            for i in range(Q.shape[0]):
                sel = np.flatnonzero(D[i] <= r)
                if sort_results:
                    sel = sel[np.argsort(D[i, sel], kind="stable")]
                ind[i], dist[i] = sel, D[i, sel]
        if train:
            for i in range(len(ind)):
                m = ind[i] != i
                ind[i], dist[i] = ind[i][m], dist[i][m]
        return (dist, ind) if return_distance else ind


def _radius_neighbors(est, X=None, radius=None, return_distance=True, sort_results=False):
    check_is_fitted(est, "_X")
    radius = est.radius if radius is None else radius
    host = getattr(est, "_host", None)
    if host is None:
        est._host = host = _HostEngine(to_numpy(est._X).astype(np.float64), "brute", "euclidean",
                                       2, None, getattr(est, "leaf_size", 30))
    return host.radius(X, radius, return_distance, sort_results)


def _graph(n_query, n_fit, dist, ind, mode):
    counts = np.array([len(i) for i in ind]) if ind.dtype == object else \
        np.full(n_query, ind.shape[1])
    indptr = np.concatenate([[0], np.cumsum(counts)])
    cols = np.concatenate(list(ind)) if ind.dtype == object else ind.ravel()
    if mode == "connectivity":
        data = np.ones(len(cols))
    elif mode == "distance":
        data = np.concatenate(list(dist)) if dist.dtype == object else dist.ravel()
    else:
        raise ValueError('Unsupported mode, must be one of "connectivity" or "distance" but got '
                         '"%s" instead' % mode)
    return sp.csr_matrix((data, cols.astype(np.int64), indptr), shape=(n_query, n_fit))


class _GraphMixin:
    def radius_neighbors(self, X=None, radius=None, return_distance=True, sort_results=False):
        return _radius_neighbors(self, X, radius, return_distance, sort_results)

    def kneighbors_graph(self, X=None, n_neighbors=None, mode="connectivity"):
        k = self.n_neighbors if n_neighbors is None else n_neighbors
        nq = self.n_samples_fit_ if X is None else np.asarray(to_numpy(X)).shape[0]
        if mode == "connectivity":
            ind = self.kneighbors(X, k, return_distance=False)
            return _graph(nq, self.n_samples_fit_, None, np.asarray(ind), mode)
        dist, ind = self.kneighbors(X, k, return_distance=True)
        return _graph(nq, self.n_samples_fit_, np.asarray(dist), np.asarray(ind), mode)

    def radius_neighbors_graph(self, X=None, radius=None, mode="connectivity",
                               sort_results=False):
        nq = self.n_samples_fit_ if X is None else np.asarray(to_numpy(X)).shape[0]
        dist, ind = self.radius_neighbors(X, radius, return_distance=True,
                                          sort_results=sort_results)
        return _graph(nq, self.n_samples_fit_, dist, ind, mode)


def _install_graph_methods():
    from .knn import _NeighborsBase
    for name in ("radius_neighbors", "kneighbors_graph", "radius_neighbors_graph"):
        if not hasattr(_NeighborsBase, name):
            setattr(_NeighborsBase, name, getattr(_GraphMixin, name))


_install_graph_methods()


def kneighbors_graph(X, n_neighbors, *, mode="connectivity", metric="minkowski", p=2,
                     metric_params=None, include_self=False, n_jobs=None):
    from .knn import NearestNeighbors
    nn = NearestNeighbors(n_neighbors=n_neighbors, metric=metric, p=p,
                          metric_params=metric_params).fit(X)
    return nn.kneighbors_graph(X if include_self else None, n_neighbors, mode=mode)


def radius_neighbors_graph(X, radius, *, mode="connectivity", metric="minkowski", p=2,
                           metric_params=None, include_self=False, n_jobs=None):
    from .knn import NearestNeighbors
    nn = NearestNeighbors(radius=radius, metric=metric, p=p, metric_params=metric_params).fit(X)
    return nn.radius_neighbors_graph(X if include_self else None, radius, mode=mode)


# ---------------------------------------------------------- radius models
def _weights(dist, weights):
    if weights in (None, "uniform"):
        return None
    if weights == "distance":
        if dist.dtype == object:
            out = np.empty_like(dist)
            for i, d in enumerate(dist):
                with np.errstate(divide="ignore"):
                    w = 1.0 / d
                if np.isinf(w).any():
                    w = np.isinf(w).astype(float)
                out[i] = w
            return out
        with np.errstate(divide="ignore"):
            w = 1.0 / dist
        inf = np.isinf(w)
        w[inf.any(1)] = inf[inf.any(1)].astype(float)
        return w
    if callable(weights):
        return weights(dist)
    raise ValueError("weights not recognized: should be 'uniform', 'distance', or a callable "
                     "function")


class _RadiusBase(BaseEstimator):
    def _init(self, radius, weights, algorithm, leaf_size, p, metric, metric_params, n_jobs,
              device):
        self.radius = radius
        self.weights = weights
        self.algorithm = algorithm
        self.leaf_size = leaf_size
        self.p = p
        self.metric = metric
        self.metric_params = metric_params
        self.n_jobs = n_jobs
        self.device = device

    def _fitX(self, X):
        from .knn import NearestNeighbors
        self._nn = NearestNeighbors(radius=self.radius, algorithm=self.algorithm,
                                    leaf_size=self.leaf_size, metric=self.metric, p=self.p,
                                    metric_params=self.metric_params, device=self.device).fit(X)
        self.n_features_in_ = self._nn.n_features_in_
        self.n_samples_fit_ = self._nn.n_samples_fit_
        self.effective_metric_ = self._nn.effective_metric_

    def radius_neighbors(self, X=None, radius=None, return_distance=True, sort_results=False):
        return self._nn.radius_neighbors(X, radius, return_distance, sort_results)


class RadiusNeighborsRegressor(RegressorMixin, _RadiusBase):
    def __init__(self, radius=1.0, *, weights="uniform", algorithm="auto", leaf_size=30, p=2,
                 metric="minkowski", metric_params=None, n_jobs=None, device=None):
        self._init(radius, weights, algorithm, leaf_size, p, metric, metric_params, n_jobs,
                   device)

    def fit(self, X, y):
        self._fitX(X)
        self._y = np.asarray(y, dtype=np.float64)
        return self

    def predict(self, X):
        check_is_fitted(self, "_nn")
        dist, ind = self.radius_neighbors(X)
        w = _weights(dist, self.weights)
        y = self._y if self._y.ndim > 1 else self._y[:, None]
        empty = np.array([len(i) == 0 for i in ind])
        if empty.any():
            warnings.warn("One or more samples have no neighbors within specified radius; "
                          "predicting NaN.")
        out = np.full((len(ind), y.shape[1]), np.nan)
        for i, idx in enumerate(ind):
            if len(idx) == 0:
                continue
            out[i] = np.mean(y[idx], axis=0) if w is None else \
                np.average(y[idx], axis=0, weights=w[i])
        return out.ravel() if self._y.ndim == 1 else out


class RadiusNeighborsClassifier(ClassifierMixin, _RadiusBase):
    def __init__(self, radius=1.0, *, weights="uniform", algorithm="auto", leaf_size=30, p=2,
                 metric="minkowski", outlier_label=None, metric_params=None, n_jobs=None,
                 device=None):
        self._init(radius, weights, algorithm, leaf_size, p, metric, metric_params, n_jobs,
                   device)
        self.outlier_label = outlier_label

    def fit(self, X, y):
        self._fitX(X)
        y = np.asarray(y)
        self.classes_, self._y = np.unique(y, return_inverse=True)
        self.outputs_2d_ = False
        if self.outlier_label is None:
            self.outlier_label_ = None
        elif self.outlier_label == "most_frequent":
            self.outlier_label_ = self.classes_[np.bincount(self._y).argmax()]
        else:
            self.outlier_label_ = self.outlier_label
        return self

    def predict_proba(self, X):
        check_is_fitted(self, "_nn")
        dist, ind = self.radius_neighbors(X)
        w = _weights(dist, self.weights)
        nc = len(self.classes_)
        P = np.zeros((len(ind), nc))
        outliers = []
        for i, idx in enumerate(ind):
            if len(idx) == 0:
                outliers.append(i)
                continue
            ww = np.ones(len(idx)) if w is None else w[i]
            P[i] = np.bincount(self._y[idx], weights=ww, minlength=nc)
        if outliers:
            if self.outlier_label_ is None:
                raise ValueError("No neighbors found for test samples %r, you can try using "
                                 "larger radius, giving a label for outliers, or considering "
                                 "removing them from your dataset." % outliers)
            if self.outlier_label_ in self.classes_:
                P[outliers, np.searchsorted(self.classes_, self.outlier_label_)] = 1.0
            else:
                warnings.warn("Outlier label {} is not in training classes. All class "
                              "probabilities of outliers will be assigned with 0."
                              .format(self.outlier_label_))
        norm = P.sum(axis=1, keepdims=True)
        norm[norm == 0.0] = 1.0
        return P / norm

    def predict(self, X):
        P = self.predict_proba(X)
        pred = self.classes_[P.argmax(axis=1)].astype(object if self.outlier_label_ is not None
                                                      and self.outlier_label_ not in
                                                      self.classes_ else self.classes_.dtype)
        zero = P.sum(axis=1) == 0
        if zero.any():
            pred[zero] = self.outlier_label_
        return pred


class KNeighborsTransformer(TransformerMixin, BaseEstimator):
    """Sparse k-nearest-neighbours graph of X (with n_neighbors + 1 in
    'distance' mode, as the reference)."""

    def __init__(self, *, mode="distance", n_neighbors=5, algorithm="auto", leaf_size=30,
                 metric="minkowski", p=2, metric_params=None, n_jobs=1, device=None):
        self.mode = mode
        self.n_neighbors = n_neighbors
        self.algorithm = algorithm
        self.leaf_size = leaf_size
        self.metric = metric
        self.p = p
        self.metric_params = metric_params
        self.n_jobs = n_jobs
        self.device = device

    def fit(self, X, y=None):
        from .knn import NearestNeighbors
        self._nn = NearestNeighbors(n_neighbors=self.n_neighbors, algorithm=self.algorithm,
                                    leaf_size=self.leaf_size, metric=self.metric, p=self.p,
                                    metric_params=self.metric_params, device=self.device).fit(X)
        self.n_features_in_ = self._nn.n_features_in_
        self.n_samples_fit_ = self._nn.n_samples_fit_
        return self

    def transform(self, X):
        check_is_fitted(self, "_nn")
        k = self.n_neighbors + (self.mode == "distance")
        return self._nn.kneighbors_graph(X, n_neighbors=k, mode=self.mode)

    def fit_transform(self, X, y=None):
        return self.fit(X).transform(X)


class RadiusNeighborsTransformer(TransformerMixin, BaseEstimator):
    def __init__(self, *, mode="distance", radius=1.0, algorithm="auto", leaf_size=30,
                 metric="minkowski", p=2, metric_params=None, n_jobs=1, device=None):
        self.mode = mode
        self.radius = radius
        self.algorithm = algorithm
        self.leaf_size = leaf_size
        self.metric = metric
        self.p = p
        self.metric_params = metric_params
        self.n_jobs = n_jobs
        self.device = device

    def fit(self, X, y=None):
        from .knn import NearestNeighbors
        self._nn = NearestNeighbors(radius=self.radius, algorithm=self.algorithm,
                                    leaf_size=self.leaf_size, metric=self.metric, p=self.p,
                                    metric_params=self.metric_params, device=self.device).fit(X)
        self.n_features_in_ = self._nn.n_features_in_
        self.n_samples_fit_ = self._nn.n_samples_fit_
        return self

    def transform(self, X):
        check_is_fitted(self, "_nn")
        return self._nn.radius_neighbors_graph(X, mode=self.mode, sort_results=True)

    def fit_transform(self, X, y=None):
        return self.fit(X).transform(X)


# ---------------------------------------------------------------- KDE
class KernelDensity(BaseEstimator):
    """Kernel density estimation (exact evaluation)."""

    def __init__(self, *, bandwidth=1.0, algorithm="auto", kernel="gaussian",
                 metric="euclidean", atol=0, rtol=0, breadth_first=True, leaf_size=40,
                 metric_params=None):
        self.algorithm = algorithm
        self.bandwidth = bandwidth
        self.kernel = kernel
        self.metric = metric
        self.atol = atol
        self.rtol = rtol
        self.breadth_first = breadth_first
        self.leaf_size = leaf_size
        self.metric_params = metric_params

    def fit(self, X, y=None, sample_weight=None):
        if self.bandwidth <= 0:
            raise ValueError("bandwidth must be positive")
        if self.kernel not in ("gaussian", "tophat", "epanechnikov", "exponential", "linear",
                               "cosine"):
            raise ValueError("invalid kernel: '{0}'".format(self.kernel))
        X = np.asarray(check_array(X), dtype=np.float64)
        if sample_weight is not None:
            sample_weight = np.asarray(sample_weight, dtype=np.float64)
            if sample_weight.shape != (X.shape[0],) or (sample_weight <= 0).any():
                raise ValueError("sample_weight must have positive values and shape (n,)")
        self.X_ = X
        self.sample_weight_ = sample_weight
        self.n_features_in_ = X.shape[1]
        return self

    def score_samples(self, X):
        check_is_fitted(self, "X_")
        X = np.asarray(check_array(X), dtype=np.float64)
        if X.shape[1] != self.n_features_in_:
            raise ValueError("X has %d features, but KernelDensity is expecting %d features as "
                             "input." % (X.shape[1], self.n_features_in_))
        N = self.X_.shape[0] if self.sample_weight_ is None else self.sample_weight_.sum()
        logd = _exact_log_density(X, self.X_, self.sample_weight_, self.bandwidth, self.kernel,
                                  self.metric, self.metric_params)
        return logd + _log_kernel_norm(self.bandwidth, X.shape[1], self.kernel) - np.log(N)

    def score(self, X, y=None):
        return np.sum(self.score_samples(X))

    def sample(self, n_samples=1, random_state=None):
        check_is_fitted(self, "X_")
        if self.kernel not in ["gaussian", "tophat"]:
            raise NotImplementedError()
        data = self.X_
        rng = check_random_state(random_state)
        u = rng.uniform(0, 1, size=n_samples)
        if self.sample_weight_ is None:
            i = (u * data.shape[0]).astype(np.int64)
        else:
            cw = np.cumsum(self.sample_weight_)
            i = np.searchsorted(cw, u * cw[-1])
        if self.kernel == "gaussian":
            return np.atleast_2d(rng.normal(data[i], self.bandwidth))
        dim = data.shape[1]
        Xn = rng.normal(size=(n_samples, dim))
        s_sq = (Xn * Xn).sum(1)
        corr = gammainc(0.5 * dim, 0.5 * s_sq) ** (1.0 / dim) * self.bandwidth / np.sqrt(s_sq)
        return data[i] + Xn * corr[:, np.newaxis]


# ---------------------------------------------------------------- LOF
class LocalOutlierFactor(OutlierMixin, BaseEstimator):
    """Local outlier factor (outlier detection, or novelty detection with
    ``novelty=True``)."""

    def __init__(self, n_neighbors=20, *, algorithm="auto", leaf_size=30, metric="minkowski",
                 p=2, metric_params=None, contamination="auto", novelty=False, n_jobs=None,
                 device=None):
        self.n_neighbors = n_neighbors
        self.algorithm = algorithm
        self.leaf_size = leaf_size
        self.metric = metric
        self.p = p
        self.metric_params = metric_params
        self.contamination = contamination
        self.novelty = novelty
        self.n_jobs = n_jobs
        self.device = device

    def _lrd(self, dist, ind):
        dist_k = self._distances_fit_X_[ind, self.n_neighbors_ - 1]
        reach = np.maximum(dist, dist_k)
        return 1.0 / (np.mean(reach, axis=1) + 1e-10)

    def fit(self, X, y=None):
        from .knn import NearestNeighbors
        if self.contamination != "auto" and not (0.0 < self.contamination <= 0.5):
            raise ValueError("contamination must be in (0, 0.5], got: %f" % self.contamination)
        self._nn = NearestNeighbors(n_neighbors=self.n_neighbors, algorithm=self.algorithm,
                                    leaf_size=self.leaf_size, metric=self.metric, p=self.p,
                                    metric_params=self.metric_params, device=self.device).fit(X)
        n = self._nn.n_samples_fit_
        self.n_samples_fit_, self.n_features_in_ = n, self._nn.n_features_in_
        if self.n_neighbors > n:
            warnings.warn("n_neighbors (%s) is greater than the total number of samples (%s). "
                          "n_neighbors will be set to (n_samples - 1) for estimation."
                          % (self.n_neighbors, n))
        self.n_neighbors_ = max(1, min(self.n_neighbors, n - 1))
        self.effective_metric_ = self._nn.effective_metric_
        self._distances_fit_X_, ind = self._nn.kneighbors(n_neighbors=self.n_neighbors_)
        self._distances_fit_X_ = np.asarray(self._distances_fit_X_)
        ind = np.asarray(ind)
        self._lrd_ = self._lrd(self._distances_fit_X_, ind)
        self.negative_outlier_factor_ = -np.mean(self._lrd_[ind] / self._lrd_[:, None], axis=1)
        self.offset_ = -1.5 if self.contamination == "auto" else \
            np.percentile(self.negative_outlier_factor_, 100.0 * self.contamination)
        return self

    def fit_predict(self, X, y=None):
        if self.novelty:
            raise AttributeError("fit_predict is not available when novelty=True. Use "
                                 "novelty=False if you want to predict on the training set.")
        self.fit(X)
        out = np.ones(self.n_samples_fit_, dtype=int)
        out[self.negative_outlier_factor_ < self.offset_] = -1
        return out

    def _check_novelty(self, name):
        if not self.novelty:
            raise AttributeError("%s is not available when novelty=False, use novelty=True if "
                                 "you want to use LOF for novelty detection and %s on new unseen "
                                 "data." % (name, name))

    def score_samples(self, X):
        self._check_novelty("score_samples")
        check_is_fitted(self, "_nn")
        dist, ind = self._nn.kneighbors(X, n_neighbors=self.n_neighbors_)
        lrd = self._lrd(np.asarray(dist), np.asarray(ind))
        return -np.mean(self._lrd_[np.asarray(ind)] / lrd[:, None], axis=1)

    def decision_function(self, X):
        self._check_novelty("decision_function")
        return self.score_samples(X) - self.offset_

    def predict(self, X):
        self._check_novelty("predict")
        out = np.ones(np.asarray(X).shape[0], dtype=int)
        out[self.decision_function(X) < 0] = -1
        return out


# ---------------------------------------------------------- NearestCentroid
class NearestCentroid(ClassifierMixin, BaseEstimator):
    def __init__(self, metric="euclidean", *, shrink_threshold=None):
        self.metric = metric
        self.shrink_threshold = shrink_threshold

    def fit(self, X, y):
        X = np.asarray(check_array(X), dtype=np.float64)
        y = np.asarray(y)
        n, d = X.shape
        self.n_features_in_ = d
        self.classes_, y_ind = np.unique(y, return_inverse=True)
        nc = len(self.classes_)
        if nc < 2:
            raise ValueError("The number of classes has to be greater than one; got %d class"
                             % nc)
        self.centroids_ = np.empty((nc, d))
        nk = np.zeros(nc)
        for c in range(nc):
            m = y_ind == c
            nk[c] = m.sum()
            self.centroids_[c] = np.median(X[m], axis=0) if self.metric == "manhattan" else \
                X[m].mean(axis=0)
        if self.shrink_threshold:
            if np.all(np.ptp(X, axis=0) == 0):
                raise ValueError("All features have zero variance. Division by zero.")
            dc = np.mean(X, axis=0)
            m = np.sqrt((1.0 / nk) - (1.0 / n))
            var = ((X - self.centroids_[y_ind]) ** 2).sum(axis=0)
            s = np.sqrt(var / (n - nc))
            s += np.median(s)
            ms = m.reshape(len(m), 1) * s
            dev_ = (self.centroids_ - dc) / ms
            signs = np.sign(dev_)
            dev_ = np.clip(np.abs(dev_) - self.shrink_threshold, 0, None) * signs
            self.centroids_ = dc[np.newaxis, :] + ms * dev_
        return self

    def predict(self, X):
        check_is_fitted(self, "centroids_")
        X = np.asarray(check_array(X), dtype=np.float64)
        D = DistanceMetric(self.metric).pairwise(X, self.centroids_)
        return self.classes_[D.argmin(axis=1)]


# -------------------------------------------------------------------- NCA
class NeighborhoodComponentsAnalysis(TransformerMixin, BaseEstimator):
    """Learn a linear map maximising the leave-one-out soft nearest-
    neighbour accuracy; loss and gradient evaluated on the device."""

    def __init__(self, n_components=None, *, init="auto", warm_start=False, max_iter=50,
                 tol=1e-5, callback=None, verbose=0, random_state=None):
        self.n_components = n_components
        self.init = init
        self.warm_start = warm_start
        self.max_iter = max_iter
        self.tol = tol
        self.callback = callback
        self.verbose = verbose
        self.random_state = random_state

    def _initialize(self, X, y, init):
        n_comp = self.n_components or X.shape[1]
        if isinstance(init, np.ndarray):
            return np.asarray(init, dtype=np.float64)
        if init == "auto":
            nc = len(np.unique(y))
            init = "lda" if n_comp <= min(X.shape[1], nc - 1) else \
                ("pca" if n_comp < X.shape[1] else "identity")
        if init == "identity":
            return np.eye(n_comp, X.shape[1])
        if init == "random":
            return self.random_state_.randn(n_comp, X.shape[1])
        if init == "pca":
            from ...decomposition import PCA
            return PCA(n_components=n_comp, random_state=self.random_state_).fit(X).components_
        if init == "lda":
            from ...discriminant_analysis import LinearDiscriminantAnalysis
            lda = LinearDiscriminantAnalysis(n_components=n_comp).fit(X, y)
            return lda.scalings_.T[:n_comp]
        raise ValueError("`init` must be 'auto', 'pca', 'identity', 'random', 'lda' or a numpy "
                         "array of shape (n_components, n_features).")

    def fit(self, X, y):
        X = np.asarray(check_array(X), dtype=np.float64)
        y = np.asarray(y)
        self.n_features_in_ = X.shape[1]
        if self.n_components is not None and self.n_components > X.shape[1]:
            raise ValueError("The preferred dimensionality of the projected space "
                             "`n_components` ({}) cannot be greater than the given data "
                             "dimensionality ({})!".format(self.n_components, X.shape[1]))
        self.random_state_ = check_random_state(self.random_state)
        _, yi = np.unique(y, return_inverse=True)
        init = self.components_ if self.warm_start and hasattr(self, "components_") else self.init
        A0 = self._initialize(X, yi, init)
        dev = resolve_device(None)
        Xt = torch.as_tensor(X, device=dev)
        mask = torch.as_tensor(yi[:, None] == yi[None, :], device=dev, dtype=torch.float64)
        self.n_iter_ = 0

        def fun(a):
            A = torch.as_tensor(a.reshape(-1, X.shape[1]), device=dev)
            E = Xt @ A.T
            sq = (E * E).sum(1)
            P = sq[:, None] + sq[None, :] - 2 * E @ E.T
            P.fill_diagonal_(float("inf"))
            P = torch.softmax(-P, dim=1)
            mp = P * mask
            p = mp.sum(1, keepdim=True)
            loss = p.sum()
            W = mp - P * p
            Ws = W + W.T
            Ws.fill_diagonal_(0.0)
            Ws.diagonal().copy_(-W.sum(0))
            g = 2 * (E.T @ Ws) @ Xt
            return -float(loss), -g.reshape(-1).cpu().numpy()

        def cb(xk):
            self.n_iter_ += 1
            if self.callback is not None:
                self.callback(xk, self.n_iter_)

        res = minimize(fun, A0.ravel(), method="L-BFGS-B", jac=True, tol=self.tol,
                       options=dict(maxiter=self.max_iter, disp=False), callback=cb)
        self.components_ = res.x.reshape(-1, X.shape[1])
        self.n_iter_ = res.nit
        return self

    def transform(self, X):
        check_is_fitted(self, "components_")
        X = np.asarray(check_array(X), dtype=np.float64)
        if X.shape[1] != self.n_features_in_:
            raise ValueError("X has %d features, but NeighborhoodComponentsAnalysis is expecting "
                             "%d features as input." % (X.shape[1], self.n_features_in_))
        return X @ self.components_.T


VALID_METRICS = {"ball_tree": BallTree.valid_metrics, "kd_tree": KDTree.valid_metrics,
                 "brute": ["euclidean", "l2", "l1", "manhattan", "cityblock", "chebyshev",
                           "minkowski", "cosine", "correlation", "hamming", "canberra",
                           "braycurtis", "seuclidean", "mahalanobis", "haversine", "jaccard"]}

__all__ = ["KDTree", "BallTree", "DistanceMetric", "RadiusNeighborsClassifier",
           "RadiusNeighborsRegressor", "KNeighborsTransformer", "RadiusNeighborsTransformer",
           "KernelDensity", "LocalOutlierFactor", "NearestCentroid",
           "NeighborhoodComponentsAnalysis", "kneighbors_graph", "radius_neighbors_graph",
           "VALID_METRICS", "VALID_METRICS_SPARSE"]

VALID_METRICS_SPARSE = {"ball_tree": [], "kd_tree": [],
                        "brute": sorted({"cityblock", "cosine", "euclidean", "l1", "l2",
                                         "manhattan", "precomputed"})}
