"""Shared linear-model machinery (reference ``linear_model/_base.py``):
centring / rescaling of the design (``_preprocess_data``,
``_rescale_data``), intercept recovery, the linear decision function and
the classifier mixin.  Heavy products run on the resolved device in fp64
(MI355X fp64 matrix cores); results come back as numpy arrays."""

import numbers

import numpy as np
import scipy.sparse as sp
import torch

from ...base import BaseEstimator, ClassifierMixin, RegressorMixin
from ...runtime.device import resolve_device
from ...utils.validation import check_array, check_is_fitted


def _as_dense64(X, copy=False):
    if isinstance(X, torch.Tensor):
        return X.detach().cpu().numpy().astype(np.float64)
    if sp.issparse(X):
        return np.asarray(X.toarray(), dtype=np.float64)
    X = check_array(X, dtype=[np.float64, np.float32], copy=copy)
    return X


def _preprocess_data(X, y, fit_intercept, normalize=False, copy=True, sample_weight=None):
    """Center X and y (weighted means) when fitting an intercept; returns
    X, y, X_offset, y_offset, X_scale."""
    if isinstance(sample_weight, numbers.Number):
        sample_weight = None
    X = np.array(X, dtype=X.dtype, copy=True) if copy else X
    y = np.asarray(y, dtype=X.dtype)
    if fit_intercept:
        X_offset = np.average(X, axis=0, weights=sample_weight)
        X = X - X_offset
        if normalize:
            X_scale = np.sqrt((X ** 2).sum(0))
            X_scale[X_scale == 0] = 1
            X = X / X_scale
        else:
            X_scale = np.ones(X.shape[1], dtype=X.dtype)
        y_offset = np.average(y, axis=0, weights=sample_weight)
        y = y - y_offset
    else:
        X_offset = np.zeros(X.shape[1], dtype=X.dtype)
        X_scale = np.ones(X.shape[1], dtype=X.dtype)
        y_offset = X.dtype.type(0) if y.ndim == 1 else np.zeros(y.shape[1], dtype=X.dtype)
    return X, y, X_offset, y_offset, X_scale


def _rescale_data(X, y, sample_weight):
    """Rows scaled by sqrt(sample_weight) (weighted least squares)."""
    sw = np.sqrt(np.asarray(sample_weight, dtype=X.dtype))
    return X * sw[:, None], (y * sw if y.ndim == 1 else y * sw[:, None])


def _check_sample_weight(sample_weight, n, dtype=np.float64):
    if sample_weight is None:
        return None
    if isinstance(sample_weight, numbers.Number):
        return np.full(n, sample_weight, dtype=dtype)
    sw = np.asarray(sample_weight, dtype=dtype)
    if sw.ndim != 1 or sw.shape[0] != n:
        raise ValueError("sample_weight.shape == {}, expected {}!".format(sw.shape, (n,)))
    return sw


def _device_tensor(a, device):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=device)


class LinearModel(BaseEstimator):
    """predict = X coef^T + intercept."""

    def _device(self):
        return resolve_device(getattr(self, "device", None))

    def _decision_function(self, X):
        check_is_fitted(self)
        X = _as_dense64(X)
        if X.shape[1] != np.atleast_2d(self.coef_).shape[-1]:
            raise ValueError(f"X has {X.shape[1]} features, but {type(self).__name__} is "
                             f"expecting {np.atleast_2d(self.coef_).shape[-1]} features as input.")
        return X @ np.asarray(self.coef_).T + self.intercept_

    def predict(self, X):
        return self._decision_function(X)

    def _set_intercept(self, X_offset, y_offset, X_scale):
        if self.fit_intercept:
            self.coef_ = self.coef_ / X_scale
            self.intercept_ = y_offset - np.dot(X_offset, self.coef_.T)
        else:
            self.intercept_ = 0.0


class LinearClassifierMixin(ClassifierMixin):
    """decision_function / predict for linear classifiers with classes_."""

    def decision_function(self, X):
        check_is_fitted(self)
        X = _as_dense64(X)
        n_features = self.coef_.shape[1]
        if X.shape[1] != n_features:
            raise ValueError("X has %d features per sample; expecting %d" % (X.shape[1], n_features))
        scores = X @ self.coef_.T + self.intercept_
        return scores.ravel() if scores.shape[1] == 1 else scores

    def predict(self, X):
        scores = self.decision_function(X)
        if scores.ndim == 1:
            idx = (scores > 0).astype(int)
        else:
            idx = scores.argmax(axis=1)
        return self.classes_[idx]

    def _predict_proba_lr(self, X):
        prob = self.decision_function(X)
        prob = 1.0 / (1.0 + np.exp(-prob))
        if prob.ndim == 1:
            return np.vstack([1 - prob, prob]).T
        prob /= prob.sum(axis=1).reshape((prob.shape[0], -1))
        return prob


class SparseCoefMixin:
    def densify(self):
        if sp.issparse(self.coef_):
            self.coef_ = self.coef_.toarray()
        return self

    def sparsify(self):
        self.coef_ = sp.csr_matrix(self.coef_)
        return self


def label_binarize_pm1(y, classes):
    """{-1, +1} indicator matrix (n, n_classes); a single column for 2 classes."""
    y = np.asarray(y)
    if len(classes) == 2:
        return np.where(y == classes[1], 1.0, -1.0)[:, None]
    Y = -np.ones((len(y), len(classes)))
    Y[np.arange(len(y)), np.searchsorted(classes, y)] = 1.0
    return Y


class LinearRegression(RegressorMixin, LinearModel):
    """Ordinary least squares (reference ``LinearRegression``): minimum-norm
    solution from the SVD of the centred design on the device; ``positive``
    -> non-negative least squares (scipy nnls on the host)."""

    def __init__(self, *, fit_intercept=True, normalize=False, copy_X=True, n_jobs=None,
                 positive=False, device=None):
        self.fit_intercept = fit_intercept
        self.normalize = normalize
        self.copy_X = copy_X
        self.n_jobs = n_jobs
        self.positive = positive
        self.device = device

    def fit(self, X, y, sample_weight=None):
        X = _as_dense64(X)
        y = np.asarray(y, dtype=X.dtype)
        self.n_features_in_ = X.shape[1]
        sw = _check_sample_weight(sample_weight, X.shape[0], X.dtype)
        X, y, X_offset, y_offset, X_scale = _preprocess_data(
            X, y, self.fit_intercept, self.normalize, copy=self.copy_X, sample_weight=sw)
        if sw is not None:
            X, y = _rescale_data(X, y, sw)
        if self.positive:
            from scipy.optimize import nnls
            if y.ndim < 2:
                self.coef_, self._residues = nnls(X, y)
            else:
                outs = [nnls(X, y[:, j]) for j in range(y.shape[1])]
                self.coef_ = np.vstack([o[0] for o in outs])
                self._residues = np.array([o[1] for o in outs])
        else:
            dev = self._device()
            Xt, yt = _device_tensor(X, dev), _device_tensor(y, dev)
            U, S, Vh = torch.linalg.svd(Xt, full_matrices=False)
            cut = torch.finfo(torch.float64).eps * (S[0] if S.numel() else 0)
            keep = S > cut
            Sinv = torch.where(keep, 1.0 / torch.where(keep, S, torch.ones_like(S)),
                               torch.zeros_like(S))
            yy = yt if yt.ndim == 2 else yt[:, None]
            coef = Vh.T @ (Sinv[:, None] * (U.T @ yy))
            self.rank_ = int(keep.sum())
            self.singular_ = S.cpu().numpy()
            resid = yy - Xt @ coef
            n, d = X.shape
            self._residues = ((resid ** 2).sum(0).cpu().numpy() if self.rank_ == d and n > d
                              else np.array([]))
            self.coef_ = coef.T.cpu().numpy()
            if y.ndim == 1:
                self._residues = self._residues.ravel()
        if y.ndim == 1:
            self.coef_ = np.ravel(self.coef_)
        self._set_intercept(X_offset, y_offset, X_scale)
        return self
