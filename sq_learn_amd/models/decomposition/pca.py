"""Classical PCA and TruncatedSVD on the MI355X SVD back-ends (parity oracles
for QPCA; reference ``sklearn/decomposition/_pca.py:114-623``,
``_truncated_svd.py``)."""

import numbers
import warnings

import numpy as np
import torch

from ...runtime.device import to_numpy
from ...utils.extmath import stable_cumsum, _infer_dimension, fast_logdet
from ...utils.validation import check_is_fitted, seed_from_random_state
from ...base import BaseEstimator, TransformerMixin
from .._data import as_data, global_mean_var
from ._base import _BasePCA, _as_out
from ._svd import full_svd, truncated_svd


class PCA(_BasePCA):
    """Principal component analysis (sklearn semantics)."""

    def __init__(self, n_components=None, *, copy=True, whiten=False, svd_solver="auto", tol=0.0,
                 iterated_power="auto", random_state=None, device=None):
        self.n_components = n_components
        self.copy = copy
        self.whiten = whiten
        self.svd_solver = svd_solver
        self.tol = tol
        self.iterated_power = iterated_power
        self.random_state = random_state
        self.device = device

    def fit(self, X, y=None):
        self._fit(X)
        return self

    def fit_transform(self, X, y=None):
        U, S = self._fit(X)
        U = U[:, :self.n_components_]
        if self.whiten:
            U = U * np.sqrt(self.n_samples_ - 1) if isinstance(U, np.ndarray) else U * (self.n_samples_ - 1) ** 0.5
        else:
            U = U * (S[:self.n_components_] if isinstance(U, np.ndarray)
                     else torch.as_tensor(S[:self.n_components_], dtype=U.dtype, device=U.device))
        return U

    def _fit(self, X):
        data = as_data(X, device=self.device, copy=self.copy)
        self.n_features_in_ = data.d
        n_samples, n_features = data.n_global, data.d
        n_components = min(n_samples, n_features) if self.n_components is None else self.n_components
        if self.n_components is None and self.svd_solver == "arpack":
            n_components = min(n_samples, n_features) - 1
        solver = self.svd_solver
        if solver == "auto":
            if max(n_samples, n_features) <= 500 or n_components == "mle":
                solver = "full"
            elif 1 <= n_components < 0.8 * min(n_samples, n_features):
                solver = "randomized"
            else:
                solver = "full"
        self._fit_svd_solver = solver
        mean, var = global_mean_var(data)
        self.mean_ = to_numpy(mean)
        self.n_samples_, self.n_features_ = n_samples, n_features
        if solver == "full":
            if n_components == "mle":
                if n_samples < n_features:
                    raise ValueError("n_components='mle' is only supported if n_samples >= n_features")
            elif not 0 <= n_components <= min(n_samples, n_features):
                raise ValueError(f"n_components={n_components!r} must be between 0 and "
                                 f"min(n_samples, n_features)={min(n_samples, n_features)!r} with "
                                 "svd_solver='full'")
            elif n_components >= 1 and not isinstance(n_components, numbers.Integral):
                raise ValueError(f"n_components={n_components!r} must be of type int when greater "
                                 f"than or equal to 1, was of type={type(n_components)!r}")
            k_left = min(n_samples, n_features)
            res = full_svd(data, mean, k_left)
            S, Vt = res.S, res.Vt
            ev = (S ** 2) / (n_samples - 1)
            ratio = ev / ev.sum()
            if n_components == "mle":
                n_components = _infer_dimension(ev, n_samples)
            elif 0 < n_components < 1.0:
                n_components = int(np.searchsorted(stable_cumsum(ratio), n_components, side="right") + 1)
            self.noise_variance_ = float(ev[n_components:].mean()) if n_components < min(n_features, n_samples) else 0.0
            self.components_ = Vt[:n_components]
            self.n_components_ = int(n_components)
            self.explained_variance_ = ev[:n_components]
            self.explained_variance_ratio_ = ratio[:n_components]
            self.singular_values_ = S[:n_components].copy()
            U = res.U_local
            return (to_numpy(U) if data.source_kind == "numpy" else U), S
        if isinstance(n_components, str) or not 1 <= n_components <= min(n_samples, n_features):
            raise ValueError(f"n_components={n_components!r} must be between 1 and "
                             f"min(n_samples, n_features)={min(n_samples, n_features)!r} with "
                             f"svd_solver='{solver}'")
        res = truncated_svd(data, mean, n_components, n_iter=self.iterated_power,
                            seed=seed_from_random_state(self.random_state))
        S, Vt = res.S, res.Vt
        self.components_ = Vt
        self.n_components_ = n_components
        self.explained_variance_ = (S ** 2) / (n_samples - 1)
        total_var = to_numpy(var) * n_samples / (n_samples - 1)
        self.explained_variance_ratio_ = self.explained_variance_ / total_var.sum()
        self.singular_values_ = S.copy()
        if n_components < min(n_features, n_samples):
            self.noise_variance_ = (total_var.sum() - self.explained_variance_.sum()) / (
                min(n_features, n_samples) - n_components)
        else:
            self.noise_variance_ = 0.0
        U = res.U_local
        return (to_numpy(U) if data.source_kind == "numpy" else U), S

    def score_samples(self, X):
        check_is_fitted(self)
        X = np.asarray(to_numpy(X), dtype=np.float64)
        Xr = X - self.mean_
        precision = self.get_precision()
        ll = -0.5 * (Xr * (Xr @ precision)).sum(axis=1)
        ll -= 0.5 * (X.shape[1] * np.log(2.0 * np.pi) - fast_logdet(precision))
        return ll

    def score(self, X, y=None):
        return float(np.mean(self.score_samples(X)))

    def _more_tags(self):
        return {"preserves_dtype": [np.float64, np.float32]}


class TruncatedSVD(TransformerMixin, BaseEstimator):
    """Truncated SVD without centring (randomized, fused power iteration)."""

    def __init__(self, n_components=2, *, algorithm="randomized", n_iter=5, random_state=None,
                 tol=0.0, device=None):
        self.n_components = n_components
        self.algorithm = algorithm
        self.n_iter = n_iter
        self.random_state = random_state
        self.tol = tol
        self.device = device

    def fit(self, X, y=None):
        self.fit_transform(X)
        return self

    def fit_transform(self, X, y=None):
        data = as_data(X, device=self.device)
        self.n_features_in_ = data.d
        zero = torch.zeros(data.d, dtype=torch.float64, device=data.device)
        if self.algorithm == "arpack" or data.n_global * data.d <= 4e6 and data.comm.world_size == 1:
            Xd = data.X.double()
            U, S, Vt = torch.linalg.svd(Xd, full_matrices=False)
            from ...utils.extmath import svd_flip
            U, Vt = svd_flip(U, Vt)
            U, S, Vt = U[:, :self.n_components], S[:self.n_components], Vt[:self.n_components]
            S, Vt = S.cpu().numpy(), Vt.cpu().numpy()
        else:
            res = truncated_svd(data, zero, self.n_components, n_iter=self.n_iter,
                                seed=seed_from_random_state(self.random_state))
            U, S, Vt = res.U_local, res.S, res.Vt
        self.components_ = Vt
        X_t = U * torch.as_tensor(S, dtype=U.dtype, device=U.device)
        # variances over all shards (one collective each)
        from .._data import Data
        tdata = Data(X_t.double(), data.n_global, data.row_offset, data.comm, data.source_kind)
        self.explained_variance_ = to_numpy(global_mean_var(tdata)[1])
        full_var = float(global_mean_var(data)[1].sum())
        self.explained_variance_ratio_ = self.explained_variance_ / full_var
        self.singular_values_ = S
        return _as_out(X_t, data.source_kind)

    def transform(self, X):
        check_is_fitted(self)
        data = as_data(X, device=self.device)
        if data.d != self.n_features_in_:
            raise ValueError(f"X has {data.d} features, but TruncatedSVD is expecting "
                             f"{self.n_features_in_} features as input.")
        out = data.X.double() @ torch.as_tensor(self.components_.T, dtype=torch.float64, device=data.device)
        return _as_out(out, data.source_kind)

    def inverse_transform(self, X):
        return np.asarray(X) @ self.components_
