"""Mini-batch k-means (reference ``cluster/_kmeans.py:1254-1723``: ``_mini_batch_step``
:1064, ``_mini_batch_convergence`` :1188, ``fit`` :1456, ``partial_fit`` :1620).

Semantics follow the reference: per-centre streaming means with
accumulated weight sums (the per-centre learning rate), random reassignment
of centres whose weight falls below ``reassignment_ratio * max`` every
``10 + min(count)`` steps, EWA-smoothed inertia / centre-shift early stopping
(``tol``, ``max_no_improvement``), best of ``n_init`` initialisations judged on
a common validation subset, and mini-batch label computation at the end.

The per-step update is vectorised (one GEMM for the batch distances,
``index_add_`` for the per-centre sums) instead of the reference's Python
loop over centres, so a step is a handful of device kernels; the host RNG
(``RandomState``) draws the same batch indices as the reference.
"""

import numpy as np
import torch

from ...base import BaseEstimator, ClusterMixin, TransformerMixin
from ...runtime.device import resolve_device, to_numpy
from ...utils.validation import check_array, check_is_fitted, check_random_state
from ._init import kmeans_plusplus as _kpp
from .._data import as_data


def _labels_inertia(X, w, C, xn=None):
    xn = (X * X).sum(1) if xn is None else xn
    D = xn[:, None] - 2.0 * (X @ C.T) + (C * C).sum(1)[None, :]
    mind, lab = D.min(1)
    mind = mind.clamp_(min=0)
    return lab, float((mind * w).sum())


class MiniBatchKMeans(TransformerMixin, ClusterMixin, BaseEstimator):
    def __init__(self, n_clusters=8, *, init="k-means++", max_iter=100, batch_size=100,
                 verbose=0, compute_labels=True, random_state=None, tol=0.0,
                 max_no_improvement=10, init_size=None, n_init=3, reassignment_ratio=0.01,
                 device=None):
        self.n_clusters = n_clusters
        self.init = init
        self.max_iter = max_iter
        self.batch_size = batch_size
        self.verbose = verbose
        self.compute_labels = compute_labels
        self.random_state = random_state
        self.tol = tol
        self.max_no_improvement = max_no_improvement
        self.init_size = init_size
        self.n_init = n_init
        self.reassignment_ratio = reassignment_ratio
        self.device = device

    # ------------------------------------------------------------ helpers
    def _tensor(self, X):
        dev = resolve_device(self.device)
        if isinstance(X, torch.Tensor):
            X = X.to(dev)
        else:
            X = torch.as_tensor(np.asarray(check_array(X), dtype=np.float64), device=dev)
        return X.to(torch.float64 if dev.type == "cpu" else torch.float32).contiguous()

    def _check_params(self, n):
        if self.n_clusters <= 0:
            raise ValueError(f"n_clusters should be > 0, got {self.n_clusters} instead.")
        if self.batch_size <= 0:
            raise ValueError(f"batch_size should be > 0, got {self.batch_size} instead.")
        if self.max_no_improvement is not None and self.max_no_improvement < 0:
            raise ValueError("max_no_improvement should be >= 0")
        if self.reassignment_ratio < 0:
            raise ValueError("reassignment_ratio should be >= 0")
        init_size = self.init_size
        if init_size is None:
            init_size = 3 * self.batch_size
        if init_size < self.n_clusters:
            init_size = 3 * self.n_clusters
        self._init_size = min(init_size, n)
        self._n_init = 1 if hasattr(self.init, "__array__") else self.n_init

    def _init_centers(self, X, rs):
        n = X.shape[0]
        if hasattr(self.init, "__array__"):
            return torch.as_tensor(np.asarray(self.init, dtype=np.float64), device=X.device).to(X.dtype)
        idx = rs.randint(0, n, self._init_size)
        Xi = X[torch.as_tensor(idx, device=X.device)]
        if isinstance(self.init, str) and self.init == "k-means++":
            C, _ = _kpp(as_data(Xi), self.n_clusters, rs)
            return C.to(X.dtype)
        if isinstance(self.init, str) and self.init == "random":
            sel = rs.permutation(Xi.shape[0])[: self.n_clusters]
            return Xi[torch.as_tensor(sel, device=X.device)].clone()
        if callable(self.init):
            return torch.as_tensor(np.asarray(self.init(to_numpy(Xi), self.n_clusters, rs)),
                                   device=X.device).to(X.dtype)
        raise ValueError(f"init should be 'k-means++', 'random' or an ndarray, got {self.init!r}")

    def _step(self, Xb, wb, C, counts, rs, random_reassign, compute_diff):
        lab, inertia = _labels_inertia(Xb, wb, C)
        if random_reassign and self.reassignment_ratio > 0:
            to_reassign = counts < self.reassignment_ratio * counts.max()
            if int(to_reassign.sum()) > 0.5 * Xb.shape[0]:
                keep = torch.argsort(counts)[int(0.5 * Xb.shape[0]):]
                to_reassign[keep] = False
            nre = int(to_reassign.sum())
            if nre:
                new = rs.choice(Xb.shape[0], replace=False, size=nre)
                C[to_reassign] = Xb[torch.as_tensor(new, device=Xb.device)]
                counts[to_reassign] = counts[~to_reassign].min()
        k = C.shape[0]
        wsum = torch.zeros(k, dtype=C.dtype, device=C.device).index_add_(0, lab, wb)
        xsum = torch.zeros_like(C).index_add_(0, lab, Xb * wb[:, None])
        upd = wsum > 0
        old = C.clone() if compute_diff else None
        new_counts = counts + wsum
        C[upd] = (C[upd] * counts[upd, None] + xsum[upd]) / new_counts[upd, None]
        counts.copy_(new_counts)
        diff = float(((C - old) ** 2).sum()) if compute_diff else 0.0
        return inertia, diff

    def _converged(self, it, n_iter, tol, n, diff, inertia, ctx):
        inertia /= self.batch_size
        diff /= self.batch_size
        if ctx.get("ewa_diff") is None:
            ctx["ewa_diff"], ctx["ewa_inertia"] = diff, inertia
        else:
            alpha = min(self.batch_size * 2.0 / (n + 1), 1.0)
            ctx["ewa_diff"] = ctx["ewa_diff"] * (1 - alpha) + diff * alpha
            ctx["ewa_inertia"] = ctx["ewa_inertia"] * (1 - alpha) + inertia * alpha
        if self.verbose:
            print(f"Minibatch iteration {it + 1}/{n_iter}: mean batch inertia: {inertia}, "
                  f"ewa inertia: {ctx['ewa_inertia']}")
        if tol > 0.0 and ctx["ewa_diff"] <= tol:
            return True
        if ctx.get("ewa_inertia_min") is None or ctx["ewa_inertia"] < ctx["ewa_inertia_min"]:
            ctx["no_improvement"] = 0
            ctx["ewa_inertia_min"] = ctx["ewa_inertia"]
        else:
            ctx["no_improvement"] = ctx.get("no_improvement", 0) + 1
        return (self.max_no_improvement is not None
                and ctx["no_improvement"] >= self.max_no_improvement)

    def _weights(self, X, sample_weight):
        if sample_weight is None:
            return torch.ones(X.shape[0], dtype=X.dtype, device=X.device)
        return torch.as_tensor(np.asarray(to_numpy(sample_weight), dtype=np.float64),
                               device=X.device).to(X.dtype)

    # ---------------------------------------------------------------- fit
    def fit(self, X, y=None, sample_weight=None):
        X = self._tensor(X)
        n, d = X.shape
        self._check_params(n)
        self.n_features_in_ = d
        rs = check_random_state(self.random_state)
        w = self._weights(X, sample_weight)
        tol = 0.0
        if self.tol > 0.0:
            tol = float(X.var(0, unbiased=False).mean()) * self.tol
        n_batches = int(np.ceil(n / self.batch_size))
        n_iter = int(self.max_iter * n_batches)
        vidx = torch.as_tensor(rs.randint(0, n, self._init_size), device=X.device)
        Xv, wv = X[vidx], w[vidx]
        best = None
        for _ in range(self._n_init):
            counts = torch.zeros(self.n_clusters, dtype=X.dtype, device=X.device)
            C = self._init_centers(X, rs)
            self._step(Xv, wv, C, counts, rs, False, False)
            _, inertia = _labels_inertia(Xv, wv, C)
            if best is None or inertia < best:
                best = inertia
                self._C, self._counts = C, counts
        ctx = {}
        it = 0
        for it in range(n_iter):
            bidx = torch.as_tensor(rs.randint(0, n, self.batch_size), device=X.device)
            reassign = (it + 1) % (10 + int(self._counts.min())) == 0
            inertia, diff = self._step(X[bidx], w[bidx], self._C, self._counts, rs, reassign,
                                       tol > 0.0)
            if self._converged(it, n_iter, tol, n, diff, inertia, ctx):
                break
        self.n_iter_ = it + 1
        self.n_steps_ = it + 1
        self._publish()
        if self.compute_labels:
            self.labels_, self.inertia_ = self._labels_inertia_batched(X, w)
        return self

    def partial_fit(self, X, y=None, sample_weight=None):
        X = self._tensor(X)
        n, d = X.shape
        w = self._weights(X, sample_weight)
        if not hasattr(self, "_rs"):
            self._rs = check_random_state(self.random_state)
        if not hasattr(self, "_C"):
            self._check_params(n)
            self.n_features_in_ = d
            self._counts = torch.zeros(self.n_clusters, dtype=X.dtype, device=X.device)
            self._C = self._init_centers(X, self._rs)
            self.n_steps_ = 0
            random_reassign = False
        else:
            if d != self.n_features_in_:
                raise ValueError(f"X has {d} features, but MiniBatchKMeans is expecting "
                                 f"{self.n_features_in_} features as input.")
            self._C = self._C.to(X.device, X.dtype)
            self._counts = self._counts.to(X.device, X.dtype)
            random_reassign = self._rs.randint(10 * (1 + int(self._counts.min()))) == 0
        self._step(X, w, self._C, self._counts, self._rs, random_reassign, False)
        self.n_steps_ += 1
        self._publish()
        if self.compute_labels:
            self.labels_, self.inertia_ = self._labels_inertia_batched(X, w)
        return self

    def _publish(self):
        self.cluster_centers_ = self._C.detach().cpu().numpy().astype(np.float64)
        self.counts_ = self._counts.detach().cpu().numpy()

    def _labels_inertia_batched(self, X, w):
        labs, tot = [], 0.0
        C = torch.as_tensor(self.cluster_centers_, device=X.device).to(X.dtype)
        for s in range(0, X.shape[0], max(self.batch_size, 65536)):
            lab, inertia = _labels_inertia(X[s:s + 65536], w[s:s + 65536], C)
            labs.append(lab)
            tot += inertia
        return torch.cat(labs).cpu().numpy().astype(np.int32), tot

    # ------------------------------------------------------------ predict
    def _check_nf(self, X):
        if X.shape[1] != self.n_features_in_:
            raise ValueError(f"X has {X.shape[1]} features, but MiniBatchKMeans is expecting "
                             f"{self.n_features_in_} features as input.")

    def predict(self, X, sample_weight=None):
        check_is_fitted(self, "cluster_centers_")
        X = self._tensor(X)
        self._check_nf(X)
        return self._labels_inertia_batched(X, self._weights(X, sample_weight))[0]

    def transform(self, X):
        check_is_fitted(self, "cluster_centers_")
        X = self._tensor(X)
        self._check_nf(X)
        C = torch.as_tensor(self.cluster_centers_, device=X.device).to(X.dtype)
        D = (X * X).sum(1)[:, None] - 2 * X @ C.T + (C * C).sum(1)[None]
        return torch.sqrt(D.clamp(min=0)).cpu().numpy()

    def score(self, X, y=None, sample_weight=None):
        X = self._tensor(X)
        return -self._labels_inertia_batched(X, self._weights(X, sample_weight))[1]
