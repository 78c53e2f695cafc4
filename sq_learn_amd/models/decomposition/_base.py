"""PCA base class (reference ``sklearn/decomposition/_base.py`` incl. the
fork's ``use_classical_components`` switch at :97-164).

``transform`` / ``inverse_transform`` project on ``components_`` (classical)
or on ``estimate_right_sv`` (the tomography estimates of the right singular
vectors produced by ``QPCA(estimate_all=True)``).  Inputs may be numpy,
tensors (any device) or row-sharded arrays; outputs follow the input kind
(numpy in -> numpy out).
"""

import numpy as np
import torch
from scipy import linalg

from ...base import BaseEstimator, TransformerMixin
from ...utils.validation import check_is_fitted
from ...runtime.device import to_numpy, resolve_device
from .._data import as_data


def _as_out(t, kind):
    return to_numpy(t) if kind == "numpy" else t


class _BasePCA(TransformerMixin, BaseEstimator):

    def get_covariance(self):
        components_ = self.components_
        exp_var = self.explained_variance_
        if self.whiten:
            components_ = components_ * np.sqrt(exp_var[:, np.newaxis])
        exp_var_diff = np.maximum(exp_var - self.noise_variance_, 0.0)
        cov = np.dot(components_.T * exp_var_diff, components_)
        cov.flat[:: len(cov) + 1] += self.noise_variance_
        return cov

    def get_precision(self):
        n_features = self.components_.shape[1]
        if self.n_components_ == 0:
            return np.eye(n_features) / self.noise_variance_
        if self.n_components_ == n_features:
            return linalg.inv(self.get_covariance())
        components_ = self.components_
        exp_var = self.explained_variance_
        if self.whiten:
            components_ = components_ * np.sqrt(exp_var[:, np.newaxis])
        exp_var_diff = np.maximum(exp_var - self.noise_variance_, 0.0)
        precision = np.dot(components_, components_.T) / self.noise_variance_
        precision.flat[:: len(precision) + 1] += 1.0 / exp_var_diff
        precision = np.dot(components_.T, np.dot(linalg.inv(precision), components_))
        precision /= -(self.noise_variance_ ** 2)
        precision.flat[:: len(precision) + 1] += 1.0 / self.noise_variance_
        return precision

    def _projection_basis(self, use_classical_components):
        if use_classical_components:
            return self.components_
        if not hasattr(self, "estimate_right_sv"):
            raise AttributeError("estimate_right_sv is not available: fit with estimate_all=True")
        return to_numpy(self.estimate_right_sv)

    def transform(self, X, use_classical_components=True):
        """(X - mean_) @ basis^T (``_base.py:97-128``)."""
        check_is_fitted(self)
        data = as_data(X, device=getattr(self, "device", None))
        if data.d != self.n_features_in_:
            raise ValueError(f"X has {data.d} features, but {type(self).__name__} is expecting "
                             f"{self.n_features_in_} features as input.")
        dt = torch.float64 if data.device.type == "cpu" else torch.float32
        basis = torch.as_tensor(np.asarray(self._projection_basis(use_classical_components)),
                                dtype=dt, device=data.device)
        Xt = data.X.to(dt)
        if self.mean_ is not None:
            Xt = Xt - torch.as_tensor(self.mean_, dtype=dt, device=data.device)
        out = Xt @ basis.T
        if self.whiten and use_classical_components:
            out = out / torch.sqrt(torch.as_tensor(self.explained_variance_, dtype=dt,
                                                   device=data.device))
        return _as_out(out, data.source_kind)

    def inverse_transform(self, X, use_classical_components=True):
        """X @ basis + mean_ (``_base.py:130-164``)."""
        check_is_fitted(self)
        basis = np.asarray(self._projection_basis(use_classical_components))
        if isinstance(X, torch.Tensor):
            dt = X.dtype if X.dtype in (torch.float32, torch.float64) else torch.float32
            B = torch.as_tensor(basis, dtype=dt, device=X.device)
            if self.whiten and use_classical_components:
                B = B * torch.sqrt(torch.as_tensor(self.explained_variance_, dtype=dt,
                                                   device=X.device))[:, None]
            return X.to(dt) @ B + torch.as_tensor(self.mean_, dtype=dt, device=X.device)
        X = np.asarray(X)
        if self.whiten and use_classical_components:
            return np.dot(X, np.sqrt(self.explained_variance_[:, np.newaxis]) * basis) + self.mean_
        return np.dot(X, basis) + self.mean_
