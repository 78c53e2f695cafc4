"""Partial least squares and CCA (reference ``cross_decomposition/_pls.py``:
NIPALS power method ``_get_first_singular_vectors_power_method`` :45,
``_PLS.fit`` :185, ``PLSRegression`` :490, ``PLSCanonical`` :620, ``CCA``
:740, ``PLSSVD`` :860).

Deflation is rank-1 updates of the (n x p) residual; X^T y products and
the final rotations use host BLAS (the matrices are small), while
``PLSSVD`` takes its cross-covariance SVD on the resolved device."""

import warnings

import numpy as np
import scipy.linalg
import torch

from .base import (BaseEstimator, MultiOutputMixin, RegressorMixin, TransformerMixin)
from .exceptions import ConvergenceWarning
from .runtime.device import resolve_device
from .utils.validation import check_is_fitted


def _pinv2_old(a):
    u, s, vh = scipy.linalg.svd(a, full_matrices=False, check_finite=False)
    t = u.dtype.char.lower()
    cond = np.max(s) * {"f": 1e3, "d": 1e6}[t] * np.finfo(t).eps
    rank = np.sum(s > cond)
    u = u[:, :rank] / s[:rank]
    return np.transpose(np.conjugate(np.dot(u, vh[:rank])))


def _first_singular_vectors_power(X, Y, mode="A", max_iter=500, tol=1e-06, norm_y_weights=False):
    eps = np.finfo(X.dtype).eps
    try:
        y_score = next(col for col in Y.T if np.any(np.abs(col) > eps))
    except StopIteration as e:
        raise StopIteration("Y residual is constant") from e
    x_old = 100
    if mode == "B":
        X_pinv, Y_pinv = _pinv2_old(X), _pinv2_old(Y)
    for i in range(max_iter):
        if mode == "B":
            xw = X_pinv @ y_score
        else:
            xw = X.T @ y_score / (y_score @ y_score)
        xw /= np.sqrt(xw @ xw) + eps
        x_score = X @ xw
        if mode == "B":
            yw = Y_pinv @ x_score
        else:
            yw = Y.T @ x_score / (x_score @ x_score)
        if norm_y_weights:
            yw /= np.sqrt(yw @ yw) + eps
        y_score = Y @ yw / (yw @ yw + eps)
        diff = xw - x_old
        if diff @ diff < tol or Y.shape[1] == 1:
            break
        x_old = xw
    n_iter = i + 1
    if n_iter == max_iter:
        warnings.warn("Maximum number of iterations reached", ConvergenceWarning)
    return xw, yw, n_iter


def _first_singular_vectors_svd(X, Y):
    U, _, Vt = scipy.linalg.svd(X.T @ Y, full_matrices=False)
    return U[:, 0], Vt[0, :]


def _center_scale_xy(X, Y, scale=True):
    xm, ym = X.mean(axis=0), Y.mean(axis=0)
    X, Y = X - xm, Y - ym
    if scale:
        xs = X.std(axis=0, ddof=1)
        xs[xs == 0.0] = 1.0
        X = X / xs
        ys = Y.std(axis=0, ddof=1)
        ys[ys == 0.0] = 1.0
        Y = Y / ys
    else:
        xs, ys = np.ones(X.shape[1]), np.ones(Y.shape[1])
    return X, Y, xm, ym, xs, ys


def _svd_flip_1d(u, v):
    i = np.argmax(np.abs(u))
    s = np.sign(u[i])
    u *= s
    v *= s


def _arr(X):
    X = X.detach().cpu().numpy() if hasattr(X, "detach") else X
    return np.array(X, dtype=np.float64)


class _PLS(TransformerMixin, RegressorMixin, MultiOutputMixin, BaseEstimator):
    def __init__(self, n_components=2, *, scale=True, deflation_mode="regression", mode="A",
                 algorithm="nipals", max_iter=500, tol=1e-06, copy=True):
        self.n_components = n_components
        self.deflation_mode = deflation_mode
        self.mode = mode
        self.scale = scale
        self.algorithm = algorithm
        self.max_iter = max_iter
        self.tol = tol
        self.copy = copy

    def fit(self, X, Y):
        X, Y = _arr(X), _arr(Y)
        if Y.ndim == 1:
            Y = Y.reshape(-1, 1)
        n, p = X.shape
        q = Y.shape[1]
        self.n_features_in_ = p
        nc = self.n_components
        ub = p if self.deflation_mode == "regression" else min(n, p, q)
        if not 1 <= nc <= ub:
            raise ValueError(f"`n_components` upper bound is {ub}. Got {nc} instead. Reduce "
                             "`n_components`.")
        if self.algorithm not in ("svd", "nipals"):
            raise ValueError("algorithm should be 'svd' or 'nipals', got %s." % self.algorithm)
        self._norm_y_weights = self.deflation_mode == "canonical"
        Xk, Yk, self._x_mean, self._y_mean, self._x_std, self._y_std = \
            _center_scale_xy(X, Y, self.scale)
        self.x_weights_ = np.zeros((p, nc))
        self._y_weights = np.zeros((q, nc))
        self._x_scores = np.zeros((n, nc))
        self._y_scores = np.zeros((n, nc))
        self.x_loadings_ = np.zeros((p, nc))
        self._y_loadings = np.zeros((q, nc))
        self.n_iter_ = []
        yeps = np.finfo(Yk.dtype).eps
        for k in range(nc):
            if self.algorithm == "nipals":
                mask = np.all(np.abs(Yk) < 10 * yeps, axis=0)
                Yk[:, mask] = 0.0
                try:
                    xw, yw, it = _first_singular_vectors_power(
                        Xk, Yk, mode=self.mode, max_iter=self.max_iter, tol=self.tol,
                        norm_y_weights=self._norm_y_weights)
                except StopIteration as e:
                    if str(e) != "Y residual is constant":
                        raise
                    warnings.warn(f"Y residual is constant at iteration {k}")
                    break
                self.n_iter_.append(it)
            else:
                xw, yw = _first_singular_vectors_svd(Xk, Yk)
            _svd_flip_1d(xw, yw)
            xs = Xk @ xw
            yss = 1 if self._norm_y_weights else yw @ yw
            ys = Yk @ yw / yss
            xl = xs @ Xk / (xs @ xs)
            Xk -= np.outer(xs, xl)
            if self.deflation_mode == "canonical":
                yl = ys @ Yk / (ys @ ys)
                Yk -= np.outer(ys, yl)
            else:
                yl = xs @ Yk / (xs @ xs)
                Yk -= np.outer(xs, yl)
            self.x_weights_[:, k], self._y_weights[:, k] = xw, yw
            self._x_scores[:, k], self._y_scores[:, k] = xs, ys
            self.x_loadings_[:, k], self._y_loadings[:, k] = xl, yl
        self.x_rotations_ = self.x_weights_ @ scipy.linalg.pinv(
            self.x_loadings_.T @ self.x_weights_, check_finite=False)
        self.y_rotations_ = self._y_weights @ scipy.linalg.pinv(
            self._y_loadings.T @ self._y_weights, check_finite=False)
        self.coef_ = (self.x_rotations_ @ self._y_loadings.T) * self._y_std
        self.x_scores_, self.y_scores_ = self._x_scores, self._y_scores
        return self

    @property
    def y_weights_(self):
        return self._y_weights

    @property
    def y_loadings_(self):
        return self._y_loadings

    def transform(self, X, Y=None, copy=True):
        check_is_fitted(self)
        X = (_arr(X) - self._x_mean) / self._x_std
        if X.shape[1] != self.n_features_in_:
            raise ValueError("X has %d features, but %s is expecting %d features as input."
                             % (X.shape[1], type(self).__name__, self.n_features_in_))
        xs = X @ self.x_rotations_
        if Y is not None:
            Y = _arr(Y)
            if Y.ndim == 1:
                Y = Y.reshape(-1, 1)
            Y = (Y - self._y_mean) / self._y_std
            return xs, Y @ self.y_rotations_
        return xs

    def inverse_transform(self, X):
        check_is_fitted(self)
        return (_arr(X) @ self.x_loadings_.T) * self._x_std + self._x_mean

    def predict(self, X, copy=True):
        check_is_fitted(self)
        X = (_arr(X) - self._x_mean) / self._x_std
        Yp = X @ self.coef_ + self._y_mean
        return Yp

    def fit_transform(self, X, y=None):
        return self.fit(X, y).transform(X, y)

    def _more_tags(self):
        return {"poor_score": True, "requires_y": False}


class PLSRegression(_PLS):

    def _more_tags(self):
        return {"multioutput_only": True}

    def __init__(self, n_components=2, *, scale=True, max_iter=500, tol=1e-06, copy=True):
        super().__init__(n_components=n_components, scale=scale, deflation_mode="regression",
                         mode="A", algorithm="nipals", max_iter=max_iter, tol=tol, copy=copy)


class PLSCanonical(_PLS):

    def _more_tags(self):
        return {"multioutput_only": True}

    def __init__(self, n_components=2, *, scale=True, algorithm="nipals", max_iter=500, tol=1e-06,
                 copy=True):
        super().__init__(n_components=n_components, scale=scale, deflation_mode="canonical",
                         mode="A", algorithm=algorithm, max_iter=max_iter, tol=tol, copy=copy)


class CCA(_PLS):

    def _more_tags(self):
        return {"multioutput_only": True}

    def __init__(self, n_components=2, *, scale=True, max_iter=500, tol=1e-06, copy=True):
        super().__init__(n_components=n_components, scale=scale, deflation_mode="canonical",
                         mode="B", algorithm="nipals", max_iter=max_iter, tol=tol, copy=copy)


class PLSSVD(TransformerMixin, BaseEstimator):
    """SVD of the cross-covariance X^T Y (on the device)."""

    def _more_tags(self):
        return {"multioutput_only": True}


    def __init__(self, n_components=2, *, scale=True, copy=True):
        self.n_components = n_components
        self.scale = scale
        self.copy = copy

    def fit(self, X, Y):
        X, Y = _arr(X), _arr(Y)
        if Y.ndim == 1:
            Y = Y.reshape(-1, 1)
        self.n_features_in_ = X.shape[1]
        ub = min(X.shape[0], X.shape[1], Y.shape[1])
        if not 1 <= self.n_components <= ub:
            raise ValueError(f"`n_components` upper bound is {ub}. Got {self.n_components} "
                             "instead. Reduce `n_components`.")
        X, Y, self._x_mean, self._y_mean, self._x_std, self._y_std = \
            _center_scale_xy(X, Y, self.scale)
        dev = resolve_device(None)
        C = torch.as_tensor(X.T @ Y, dtype=torch.float64, device=dev)
        U, s, Vt = torch.linalg.svd(C, full_matrices=False)
        U = U[:, :self.n_components].cpu().numpy()
        Vt = Vt[:self.n_components].cpu().numpy()
        mx = np.argmax(np.abs(U), axis=0)
        signs = np.sign(U[mx, range(U.shape[1])])
        U *= signs
        Vt *= signs[:, np.newaxis]
        self.x_weights_ = U
        self.y_weights_ = Vt.T
        self._x_scores = X @ self.x_weights_
        self._y_scores = Y @ self.y_weights_
        return self

    def transform(self, X, Y=None):
        check_is_fitted(self)
        X = (_arr(X) - self._x_mean) / self._x_std
        xs = X @ self.x_weights_
        if Y is not None:
            Y = _arr(Y)
            if Y.ndim == 1:
                Y = Y.reshape(-1, 1)
            return xs, ((Y - self._y_mean) / self._y_std) @ self.y_weights_
        return xs

    def fit_transform(self, X, y=None):
        return self.fit(X, y).transform(X, y)


__all__ = ["PLSRegression", "PLSCanonical", "CCA", "PLSSVD"]

from .utils._aliases import alias_submodules  # noqa: E402
alias_submodules(__name__, "_pls")
