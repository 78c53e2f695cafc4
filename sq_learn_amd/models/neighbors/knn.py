"""Brute-force k-nearest neighbours on MI355X.

Reference: ``sklearn/neighbors/_classification.py`` (``KNeighborsClassifier``)
and ``_base.py`` (``kneighbors``).  The reference chooses KD/Ball trees or
brute force on the CPU; on the GPU brute force wins for the dimensions of
the reference pipelines (MNIST-shape, d = 61-784): query tiles x reference
set distances by one library GEMM, then the per-row top-k selection kernel
(``csrc/knn.hip``).  Tiles are sized by ``working_memory``.
"""

import numpy as np
import torch

from ...base import BaseEstimator, ClassifierMixin, RegressorMixin
from ...utils.validation import check_is_fitted, check_array
from ...utils.pairwise import get_chunk_n_rows
from ...runtime.device import resolve_device, to_numpy
from ...ops import _native as nat


def _topk_rows(D, k, col_offset=0):
    """(dist, idx) of the k smallest entries per row of D."""
    if nat.use_native(D) and k <= 32:
        m, nref = D.shape
        D = D.contiguous()
        od = torch.empty((m, k), dtype=torch.float32, device=D.device)
        oi = torch.empty((m, k), dtype=torch.int64, device=D.device)
        nat.native().knn_topk(D.data_ptr(), od.data_ptr(), oi.data_ptr(), m, nref, D.stride(0), k,
                              int(col_offset), nat.stream_handle(D.device))
        return od, oi
    v, i = torch.topk(D, k, dim=1, largest=False, sorted=True)
    return v, i + col_offset


class _NeighborsBase(BaseEstimator):
    def _fit(self, X, y=None):
        dev = resolve_device(self.device)
        if isinstance(X, torch.Tensor):
            Xt = X.to(dev)
        else:
            Xt = torch.as_tensor(np.asarray(check_array(X), dtype=np.float64)).to(dev)
        self._dt = torch.float64 if dev.type == "cpu" else torch.float32
        self._X = Xt.to(self._dt).contiguous()
        self._xn = (self._X * self._X).sum(1)
        self.n_features_in_ = self._X.shape[1]
        self.n_samples_fit_ = self._X.shape[0]
        # euclidean + auto/brute -> device GEMM + top-k; anything else (other
        # metrics, explicit kd_tree / ball_tree) -> host trees / pairwise
        from ._extra import _HostEngine, _is_euclidean
        euclid = _is_euclidean(self.metric, getattr(self, "p", 2), self.metric_params)
        algo = getattr(self, "algorithm", "auto")
        self._host = None
        if not euclid or algo in ("kd_tree", "ball_tree"):
            self._host = _HostEngine(to_numpy(Xt).astype(np.float64), algo, self.metric,
                                     getattr(self, "p", 2), self.metric_params,
                                     getattr(self, "leaf_size", 30))
        self._fit_method = self._host.method if self._host is not None else "brute"
        self.effective_metric_ = "euclidean" if euclid else self.metric
        return self

    def kneighbors(self, X=None, n_neighbors=None, return_distance=True):
        check_is_fitted(self, "_X")
        if X is not None and np.shape(X)[-1] != self.n_features_in_:
            raise ValueError(f"X has {np.shape(X)[-1]} features, but {type(self).__name__} is "
                             f"expecting {self.n_features_in_} features as input.")
        if getattr(self, "_host", None) is not None:
            k = self.n_neighbors if n_neighbors is None else n_neighbors
            return self._host.kneighbors(X, k, return_distance)
        k = self.n_neighbors if n_neighbors is None else n_neighbors
        dev = self._X.device
        query_is_train = X is None
        Q = self._X if query_is_train else torch.as_tensor(
            np.asarray(to_numpy(X), dtype=np.float64)).to(dev).to(self._dt)
        kk = k + 1 if query_is_train else k
        if kk > self.n_samples_fit_:
            raise ValueError(f"Expected n_neighbors <= n_samples, but n_samples = "
                             f"{self.n_samples_fit_}, n_neighbors = {kk}")
        rows = get_chunk_n_rows(4 * self.n_samples_fit_)
        dists, idxs = [], []
        for s in range(0, Q.shape[0], rows):
            q = Q[s:s + rows]
            D = ((q * q).sum(1)[:, None] + self._xn[None, :] - 2.0 * (q @ self._X.T)).clamp_(min=0)
            if D.dtype != torch.float32 and nat.use_native(D):
                D = D.float()
            v, i = _topk_rows(D, kk)
            dists.append(v.to(torch.float64))
            idxs.append(i)
        dist = torch.sqrt(torch.cat(dists)).cpu().numpy()
        ind = torch.cat(idxs).cpu().numpy()
        if query_is_train:
            # drop each sample itself (first occurrence of its own index)
            keep = np.ones_like(ind, dtype=bool)
            self_pos = (ind == np.arange(ind.shape[0])[:, None])
            first = np.where(self_pos.any(1), self_pos.argmax(1), kk - 1)
            keep[np.arange(ind.shape[0]), first] = False
            ind = ind[keep].reshape(ind.shape[0], k)
            dist = dist[keep].reshape(dist.shape[0], k)
        return (dist, ind) if return_distance else ind


class KNeighborsClassifier(ClassifierMixin, _NeighborsBase):
    def __init__(self, n_neighbors=5, *, weights="uniform", algorithm="auto", leaf_size=30, p=2,
                 metric="minkowski", metric_params=None, n_jobs=None, device=None):
        self.n_neighbors = n_neighbors
        self.weights = weights
        self.algorithm = algorithm
        self.leaf_size = leaf_size
        self.p = p
        self.metric = metric
        self.metric_params = metric_params
        self.n_jobs = n_jobs
        self.device = device

    def fit(self, X, y):
        X, y = self._validate_data(X, y) if not isinstance(X, torch.Tensor) else (X, y)
        self._fit(X)
        y = np.asarray(to_numpy(y))
        self.classes_, self._y = np.unique(y, return_inverse=True)
        self.outputs_2d_ = False
        return self

    def _weights(self, dist):
        if self.weights == "uniform":
            return np.ones_like(dist)
        if self.weights == "distance":
            with np.errstate(divide="ignore"):
                w = 1.0 / dist
            inf = np.isinf(w)
            w[inf.any(1)] = inf[inf.any(1)].astype(float)
            return w
        if callable(self.weights):
            return self.weights(dist)
        raise ValueError("weights not recognized")

    def predict_proba(self, X):
        dist, ind = self.kneighbors(X)
        w = self._weights(dist)
        lab = self._y[ind]
        P = np.zeros((ind.shape[0], len(self.classes_)))
        for c in range(len(self.classes_)):
            P[:, c] = (w * (lab == c)).sum(1)
        P /= P.sum(1, keepdims=True)
        return P

    def predict(self, X):
        return self.classes_[np.argmax(self.predict_proba(X), axis=1)]


class KNeighborsRegressor(RegressorMixin, _NeighborsBase):
    def __init__(self, n_neighbors=5, *, weights="uniform", algorithm="auto", leaf_size=30, p=2,
                 metric="minkowski", metric_params=None, n_jobs=None, device=None):
        self.n_neighbors = n_neighbors
        self.weights = weights
        self.algorithm = algorithm
        self.leaf_size = leaf_size
        self.p = p
        self.metric = metric
        self.metric_params = metric_params
        self.n_jobs = n_jobs
        self.device = device

    def fit(self, X, y):
        self._fit(X)
        self._yv = np.asarray(to_numpy(y), dtype=np.float64)
        return self

    def predict(self, X):
        dist, ind = self.kneighbors(X)
        if self.weights == "distance":
            with np.errstate(divide="ignore"):
                w = 1.0 / dist
            w[np.isinf(w).any(1)] = np.isinf(w[np.isinf(w).any(1)]).astype(float)
        else:
            w = np.ones_like(dist)
        return (w * self._yv[ind]).sum(1) / w.sum(1)


class NearestNeighbors(_NeighborsBase):
    def __init__(self, n_neighbors=5, *, radius=1.0, algorithm="auto", leaf_size=30,
                 metric="minkowski", p=2, metric_params=None, n_jobs=None, device=None):
        self.n_neighbors = n_neighbors
        self.radius = radius
        self.algorithm = algorithm
        self.leaf_size = leaf_size
        self.metric = metric
        self.p = p
        self.metric_params = metric_params
        self.n_jobs = n_jobs
        self.device = device

    def fit(self, X, y=None):
        return self._fit(X)
