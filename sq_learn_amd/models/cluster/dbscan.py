"""DBSCAN (reference ``cluster/_dbscan.py`` + ``_dbscan_inner.pyx``;
SURVEY.md N24).

Radius neighbourhoods come from chunked distance GEMMs on the data's device
(hipBLASLt on MI355X: ||x||^2 + ||y||^2 - 2 x.y, thresholded at eps^2 inside
each chunk, so only the CSR neighbour lists reach the host); the cluster
expansion is the host-native depth-first pass ``sqh_dbscan_inner``
(``csrc/host/cluster_host.cpp``).  ``metric='precomputed'`` takes a dense or
sparse distance matrix; other metrics go through ``torch.cdist``
(minkowski family)."""

import numpy as np
import scipy.sparse as sp
import torch

from ...base import BaseEstimator, ClusterMixin
from ...ops import _host
from ...runtime.device import resolve_device, to_tensor
from ...utils.pairwise import get_chunk_n_rows

_P_OF = {"euclidean": 2.0, "l2": 2.0, "manhattan": 1.0, "cityblock": 1.0, "l1": 1.0,
         "chebyshev": float("inf")}


def radius_neighbors_graph(X, eps, *, metric="euclidean", p=None, device=None):
    """CSR (indptr, indices) of {j : d(x_i, x_j) <= eps} for every row (self
    included), computed chunk by chunk on the device."""
    Xt = X if isinstance(X, torch.Tensor) else to_tensor(np.asarray(X), resolve_device(device))
    if not Xt.is_floating_point() or Xt.dtype == torch.bfloat16:
        Xt = Xt.float()
    if Xt.device.type == "cpu":
        Xt = Xt.double()
    n = Xt.shape[0]
    rows = get_chunk_n_rows(max(n, 1) * 8)
    indptr = [np.zeros(1, dtype=np.int64)]
    indices = []
    total = 0
    euclid = metric in ("euclidean", "l2") and p in (None, 2)
    if euclid:
        xn = (Xt * Xt).sum(1)
        thr = eps * eps
    for s in range(0, n, rows):
        e = min(n, s + rows)
        if euclid:
            D2 = (xn[s:e, None] + xn[None, :] - 2.0 * (Xt[s:e] @ Xt.T)).clamp_(min=0)
            # expansion error ~ machine eps * (|x|^2 + |y|^2): widen, then
            # decide the candidates with the exact difference
            tol = 16 * torch.finfo(Xt.dtype).eps
            cand = D2 <= thr * (1 + tol) + tol * (xn[s:e, None] + xn[None, :])
            r, c = torch.nonzero(cand, as_tuple=True)
            if r.numel():
                exact = ((Xt[s + r] - Xt[c]) ** 2).sum(1) <= thr
                r, c = r[exact], c[exact]
        else:
            pp = _P_OF.get(metric, p if p is not None else 2.0) if metric != "minkowski" else (
                p if p is not None else 2.0)
            D = torch.cdist(Xt[s:e], Xt, p=pp)
            r, c = torch.nonzero(D <= eps, as_tuple=True)
        counts = torch.bincount(r, minlength=e - s).cpu().numpy().astype(np.int64)
        indices.append(c.cpu().numpy().astype(np.int64))
        indptr.append(total + np.cumsum(counts))
        total += int(counts.sum())
    return np.concatenate(indptr), (np.concatenate(indices) if indices else
                                    np.zeros(0, dtype=np.int64))


def _precomputed_neighbors(X, eps):
    if sp.issparse(X):
        X = X.tocsr()
        X.sort_indices()
        n = X.shape[0]
        indptr = [0]
        indices = []
        for i in range(n):
            sl = slice(X.indptr[i], X.indptr[i + 1])
            cols = X.indices[sl][X.data[sl] <= eps]
            if i not in set(cols.tolist()):
                cols = np.sort(np.append(cols, i))   # self is a neighbour (distance 0)
            indices.append(cols)
            indptr.append(indptr[-1] + len(cols))
        return np.asarray(indptr, np.int64), np.concatenate(indices).astype(np.int64)
    D = np.asarray(X)
    r, c = np.nonzero(D <= eps)
    counts = np.bincount(r, minlength=D.shape[0])
    return np.concatenate([[0], np.cumsum(counts)]).astype(np.int64), c.astype(np.int64)


def dbscan(X, eps=0.5, *, min_samples=5, metric="minkowski", metric_params=None,
           algorithm="auto", leaf_size=30, p=2, sample_weight=None, n_jobs=None):
    """Functional interface: (core_sample_indices, labels)."""
    est = DBSCAN(eps=eps, min_samples=min_samples, metric=metric, metric_params=metric_params,
                 algorithm=algorithm, leaf_size=leaf_size, p=p, n_jobs=n_jobs)
    est.fit(X, sample_weight=sample_weight)
    return est.core_sample_indices_, est.labels_


class DBSCAN(ClusterMixin, BaseEstimator):
    """Density-based clustering (eps, min_samples, metric, ...: reference
    parameters; ``algorithm`` / ``leaf_size`` are accepted - the
    neighbourhoods are always brute-force GEMMs on the device)."""

    def __init__(self, eps=0.5, *, min_samples=5, metric="euclidean", metric_params=None,
                 algorithm="auto", leaf_size=30, p=None, n_jobs=None, device=None):
        self.eps = eps
        self.min_samples = min_samples
        self.metric = metric
        self.metric_params = metric_params
        self.algorithm = algorithm
        self.leaf_size = leaf_size
        self.p = p
        self.n_jobs = n_jobs
        self.device = device

    def fit(self, X, y=None, sample_weight=None):
        if not self.eps > 0.0:
            raise ValueError("eps must be positive.")
        if self.metric == "precomputed":
            indptr, indices = _precomputed_neighbors(X, self.eps)
            n = indptr.shape[0] - 1
            Xd = None
        else:
            Xd = X if (sp.issparse(X) is False and isinstance(X, torch.Tensor)) else (
                np.asarray(X.toarray() if sp.issparse(X) else X))
            indptr, indices = radius_neighbors_graph(Xd, self.eps, metric=self.metric, p=self.p,
                                                     device=self.device)
            n = indptr.shape[0] - 1
        if sample_weight is None:
            n_neighbors = np.diff(indptr)
        else:
            w = np.asarray(sample_weight, dtype=np.float64)
            if w.shape != (n,):
                raise ValueError("sample_weight has the wrong shape")
            n_neighbors = np.add.reduceat(w[indices], indptr[:-1]) if len(indices) else np.zeros(n)
            n_neighbors[np.diff(indptr) == 0] = 0
        labels = np.full(n, -1, dtype=np.int64)
        core = np.ascontiguousarray(np.asarray(n_neighbors) >= self.min_samples, dtype=np.uint8)
        ip = np.ascontiguousarray(indptr, dtype=np.int64)
        ix = np.ascontiguousarray(indices, dtype=np.int64)
        if n:
            _host.lib().sqh_dbscan_inner(_host.ptr(core), _host.ptr(ip), _host.ptr(ix), n,
                                         _host.ptr(labels))
        self.core_sample_indices_ = np.where(core)[0]
        self.labels_ = labels
        if len(self.core_sample_indices_) and Xd is not None:
            Xn = Xd.cpu().numpy() if isinstance(Xd, torch.Tensor) else Xd
            self.components_ = Xn[self.core_sample_indices_].copy()
        else:
            self.components_ = np.empty((0, 0 if Xd is None else Xd.shape[1]))
        return self

    def fit_predict(self, X, y=None, sample_weight=None):
        self.fit(X, sample_weight=sample_weight)
        return self.labels_
