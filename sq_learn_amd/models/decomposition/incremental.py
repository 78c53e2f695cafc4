"""Incremental PCA (reference ``decomposition/_incremental_pca.py``, 358 LoC).

Each ``partial_fit`` folds a batch into the running factorisation: the
stacked matrix ``[diag(S) Vt ; X_b - mean_b ; sqrt(n n_b / (n + n_b)) (mean - mean_b)]``
has the same right singular vectors / values as the centred union of all
rows seen so far, so its thin SVD (small: (k + n_b + 1) x d) updates the
model.  Means/variances use the streaming (Chan) combination.  Runs on the
data's device in fp64 (CPU) / fp32 (GPU).
"""

import numpy as np
import torch

from ...runtime.device import resolve_device
from ...utils.extmath import svd_flip
from ...utils.pairwise import gen_batches
from ...utils.validation import check_array
from ._base import _BasePCA


class IncrementalPCA(_BasePCA):
    def __init__(self, n_components=None, *, whiten=False, copy=True, batch_size=None,
                 device=None):
        self.n_components = n_components
        self.whiten = whiten
        self.copy = copy
        self.batch_size = batch_size
        self.device = device

    def _np(self, X):
        if isinstance(X, torch.Tensor):
            return X.detach().cpu().numpy().astype(np.float64)
        return np.asarray(check_array(X), dtype=np.float64)

    def fit(self, X, y=None):
        for a in ("components_", "n_samples_seen_", "mean_", "var_"):
            if hasattr(self, a):
                delattr(self, a)
        X = self._np(X)
        n, d = X.shape
        self.batch_size_ = 5 * d if self.batch_size is None else self.batch_size
        for sl in gen_batches(n, self.batch_size_, min_batch_size=self.n_components or 0):
            self.partial_fit(X[sl], check_input=False)
        return self

    def partial_fit(self, X, y=None, check_input=True):
        X = self._np(X) if check_input or not isinstance(X, np.ndarray) else X
        n_b, d = X.shape
        first = not hasattr(self, "components_")
        if first:
            self.n_features_in_ = d
        elif d != self.components_.shape[1]:
            raise ValueError("Number of features of the new batch does not match the number "
                             "of features of the first batch.")
        if self.n_components is None:
            k = d if first else self.components_.shape[0]
        elif not 1 <= self.n_components <= d:
            raise ValueError(f"n_components={self.n_components} invalid for n_features={d}, "
                             "need more rows than columns for IncrementalPCA processing")
        elif self.n_components > n_b:
            raise ValueError(f"n_components={self.n_components} must be less or equal to the "
                             f"batch number of samples {n_b}.")
        else:
            k = self.n_components
        if not first and self.components_.shape[0] != k:
            raise ValueError(f"Number of input features has changed from "
                             f"{self.components_.shape[0]} to {k} between calls to partial_fit!")
        if first:
            self.n_samples_seen_ = 0
            self.mean_ = np.zeros(d)
            self.var_ = np.zeros(d)

        dev = resolve_device(self.device)
        dt = torch.float64 if dev.type == "cpu" else torch.float32
        Xt = torch.as_tensor(X, device=dev, dtype=dt)
        n_a = self.n_samples_seen_
        mean_b = Xt.mean(0).double().cpu().numpy()
        m2_b = ((Xt - Xt.mean(0)) ** 2).sum(0).double().cpu().numpy()
        n_tot = n_a + n_b
        delta = mean_b - self.mean_
        col_mean = self.mean_ + delta * (n_b / n_tot)
        col_var = (self.var_ * n_a + m2_b + delta * delta * (n_a * n_b / n_tot)) / n_tot

        Xc = Xt - torch.as_tensor(mean_b, device=dev, dtype=dt)
        if first:
            M = Xc
        else:
            corr = np.sqrt((n_a / n_tot) * n_b) * (self.mean_ - mean_b)
            M = torch.cat([
                torch.as_tensor(self.singular_values_[:, None] * self.components_, device=dev,
                                dtype=dt),
                Xc,
                torch.as_tensor(corr[None, :], device=dev, dtype=dt)])
        U, S, Vt = torch.linalg.svd(M, full_matrices=False)
        U, Vt = svd_flip(U.double().cpu().numpy(), Vt.double().cpu().numpy(),
                         u_based_decision=False)
        S = S.double().cpu().numpy()
        ev = S ** 2 / (n_tot - 1)
        evr = S ** 2 / np.sum(col_var * n_tot)

        self.n_samples_seen_ = n_tot
        self.components_ = Vt[:k]
        self.singular_values_ = S[:k]
        self.mean_ = col_mean
        self.var_ = col_var
        self.explained_variance_ = ev[:k]
        self.explained_variance_ratio_ = evr[:k]
        self.n_components_ = k
        if k not in (n_tot, d):
            self.noise_variance_ = float(ev[k:].mean()) if ev.size > k else 0.0
        else:
            self.noise_variance_ = 0.0
        return self
