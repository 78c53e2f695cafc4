"""Bayesian linear regression (reference ``linear_model/_bayes.py``).

``BayesianRidge`` (reference _bayes.py:176-300): evidence maximisation
(MacKay 1992) over the thin SVD of the centred design.  The SVD is taken
once on the device in fp64; each iteration is then an O(d^2) update of
the posterior mean in the SVD basis, so the loop never re-touches X.

``ARDRegression`` (reference _bayes.py:528-640): per-feature precisions
with pruning; sigma is the pseudo-inverse of the (kept) posterior
precision (Gram form when n >= d, Woodbury form otherwise).
"""

from math import log

import numpy as np
import torch

from ...base import RegressorMixin
from ._base import (LinearModel, _as_dense64, _check_sample_weight, _device_tensor,
                    _preprocess_data, _rescale_data)


def _pinvh(A):
    """Pseudo-inverse of a symmetric matrix via its eigendecomposition
    (cutoff as scipy.linalg.pinvh: largest |eig| * max(shape) * eps)."""
    w, V = np.linalg.eigh(A)
    cut = np.abs(w).max() * max(A.shape) * np.finfo(A.dtype).eps if w.size else 0.0
    keep = np.abs(w) > cut
    return (V[:, keep] / w[keep]) @ V[:, keep].T


def _fast_logdet(A):
    sign, ld = np.linalg.slogdet(A)
    return ld if sign > 0 else -np.inf


class BayesianRidge(RegressorMixin, LinearModel):
    """Bayesian ridge regression with evidence-maximised alpha/lambda."""

    def __init__(self, *, n_iter=300, tol=1.e-3, alpha_1=1.e-6, alpha_2=1.e-6,
                 lambda_1=1.e-6, lambda_2=1.e-6, alpha_init=None, lambda_init=None,
                 compute_score=False, fit_intercept=True, normalize=False, copy_X=True,
                 verbose=False):
        self.n_iter = n_iter
        self.tol = tol
        self.alpha_1 = alpha_1
        self.alpha_2 = alpha_2
        self.lambda_1 = lambda_1
        self.lambda_2 = lambda_2
        self.alpha_init = alpha_init
        self.lambda_init = lambda_init
        self.compute_score = compute_score
        self.fit_intercept = fit_intercept
        self.normalize = normalize
        self.copy_X = copy_X
        self.verbose = verbose

    def fit(self, X, y, sample_weight=None):
        if self.n_iter < 1:
            raise ValueError("n_iter should be greater than or equal to 1. Got {!r}."
                             .format(self.n_iter))
        X = _as_dense64(X).astype(np.float64)
        y = np.asarray(y, dtype=np.float64).ravel()
        if X.shape[0] != y.shape[0]:
            raise ValueError("Found input variables with inconsistent numbers of samples")
        self.n_features_in_ = X.shape[1]
        sw = _check_sample_weight(sample_weight, X.shape[0])
        X, y, X_offset, y_offset, X_scale = _preprocess_data(
            X, y, self.fit_intercept, self.normalize, True, sample_weight=sw)
        if sw is not None:
            X, y = _rescale_data(X, y, sw)
        self.X_offset_, self.X_scale_ = X_offset, X_scale
        n, d = X.shape
        eps = np.finfo(np.float64).eps
        alpha_ = self.alpha_init if self.alpha_init is not None else 1. / (np.var(y) + eps)
        lambda_ = self.lambda_init if self.lambda_init is not None else 1.

        dev = self._device()
        Xt = _device_tensor(X, dev)
        U, S, Vh = torch.linalg.svd(Xt, full_matrices=False)
        U, S, Vh = U.cpu().numpy(), S.cpu().numpy(), Vh.cpu().numpy()
        ev = S ** 2
        XTy = X.T @ y
        Uty = U.T @ y
        Vty = Vh @ XTy

        def update(a, lam):
            if n > d:
                coef = Vh.T @ (Vty / (ev + lam / a))
            else:
                coef = X.T @ (U @ (Uty / (ev + lam / a)))
            return coef, float(np.sum((y - X @ coef) ** 2))

        self.scores_ = []
        coef_old = None
        for it in range(self.n_iter):
            coef, rmse = update(alpha_, lambda_)
            if self.compute_score:
                self.scores_.append(self._log_ml(n, d, ev, alpha_, lambda_, coef, rmse))
            gamma = np.sum((alpha_ * ev) / (lambda_ + alpha_ * ev))
            lambda_ = (gamma + 2 * self.lambda_1) / (np.sum(coef ** 2) + 2 * self.lambda_2)
            alpha_ = (n - gamma + 2 * self.alpha_1) / (rmse + 2 * self.alpha_2)
            if it != 0 and np.sum(np.abs(coef_old - coef)) < self.tol:
                if self.verbose:
                    print("Convergence after ", str(it), " iterations")
                break
            coef_old = coef.copy()
        self.n_iter_ = it + 1
        self.alpha_, self.lambda_ = alpha_, lambda_
        self.coef_, rmse = update(alpha_, lambda_)
        if self.compute_score:
            self.scores_.append(self._log_ml(n, d, ev, alpha_, lambda_, coef, rmse))
            self.scores_ = np.array(self.scores_)
        self.sigma_ = (1. / alpha_) * (Vh.T @ (Vh / (ev + lambda_ / alpha_)[:, None]))
        self._set_intercept(X_offset, y_offset, X_scale)
        return self

    def _log_ml(self, n, d, ev, alpha_, lambda_, coef, rmse):
        if n > d:
            logdet = -np.sum(np.log(lambda_ + alpha_ * ev))
        else:
            full = np.full(d, lambda_, dtype=np.float64)
            full[:n] += alpha_ * ev
            logdet = -np.sum(np.log(full))
        s = self.lambda_1 * log(lambda_) - self.lambda_2 * lambda_
        s += self.alpha_1 * log(alpha_) - self.alpha_2 * alpha_
        s += 0.5 * (d * log(lambda_) + n * log(alpha_) - alpha_ * rmse
                    - lambda_ * np.sum(coef ** 2) + logdet - n * log(2 * np.pi))
        return s

    def predict(self, X, return_std=False):
        y_mean = self._decision_function(X)
        if not return_std:
            return y_mean
        X = _as_dense64(X)
        if self.normalize:
            X = (X - self.X_offset_) / self.X_scale_
        var = ((X @ self.sigma_) * X).sum(axis=1)
        return y_mean, np.sqrt(var + 1. / self.alpha_)


class ARDRegression(RegressorMixin, LinearModel):
    """Automatic relevance determination regression."""

    def __init__(self, *, n_iter=300, tol=1.e-3, alpha_1=1.e-6, alpha_2=1.e-6,
                 lambda_1=1.e-6, lambda_2=1.e-6, compute_score=False, threshold_lambda=1.e+4,
                 fit_intercept=True, normalize=False, copy_X=True, verbose=False):
        self.n_iter = n_iter
        self.tol = tol
        self.fit_intercept = fit_intercept
        self.normalize = normalize
        self.alpha_1 = alpha_1
        self.alpha_2 = alpha_2
        self.lambda_1 = lambda_1
        self.lambda_2 = lambda_2
        self.compute_score = compute_score
        self.threshold_lambda = threshold_lambda
        self.copy_X = copy_X
        self.verbose = verbose

    def fit(self, X, y):
        X = _as_dense64(X).astype(np.float64)
        y = np.asarray(y, dtype=np.float64).ravel()
        if X.shape[0] < 2:
            raise ValueError("ARDRegression requires at least 2 samples")
        self.n_features_in_ = X.shape[1]
        n, d = X.shape
        coef = np.zeros(d)
        X, y, X_offset, y_offset, X_scale = _preprocess_data(
            X, y, self.fit_intercept, self.normalize, True)
        self.X_offset_, self.X_scale_ = X_offset, X_scale
        keep = np.ones(d, dtype=bool)
        l1, l2, a1, a2 = self.lambda_1, self.lambda_2, self.alpha_1, self.alpha_2
        alpha_ = 1. / (np.var(y) + np.finfo(np.float64).eps)
        lambda_ = np.ones(d)
        gram_full = X.T @ X if n >= d else None

        def update_sigma(a, lam, kp):
            if n >= d:
                G = gram_full[np.ix_(kp, kp)]
                return _pinvh(np.diag(lam[kp]) + a * G)
            Xk = X[:, kp]
            inv = 1. / lam[kp][None, :]
            S = _pinvh(np.eye(n) / a + (Xk * inv) @ Xk.T)
            S = -(inv.T * Xk.T) @ (S @ (Xk * inv))
            S[np.diag_indices(S.shape[1])] += 1. / lam[kp]
            return S

        def update_coef(c, a, kp, sig):
            c[kp] = a * (sig @ (X[:, kp].T @ y))
            return c

        self.scores_ = []
        coef_old = None
        for it in range(self.n_iter):
            sigma = update_sigma(alpha_, lambda_, keep)
            coef = update_coef(coef, alpha_, keep, sigma)
            rmse = np.sum((y - X @ coef) ** 2)
            gamma = 1. - lambda_[keep] * np.diag(sigma)
            lambda_[keep] = (gamma + 2. * l1) / (coef[keep] ** 2 + 2. * l2)
            alpha_ = (n - gamma.sum() + 2. * a1) / (rmse + 2. * a2)
            keep = lambda_ < self.threshold_lambda
            coef[~keep] = 0
            if self.compute_score:
                s = (l1 * np.log(lambda_) - l2 * lambda_).sum()
                s += a1 * log(alpha_) - a2 * alpha_
                s += 0.5 * (_fast_logdet(sigma) + n * log(alpha_) + np.sum(np.log(lambda_)))
                s -= 0.5 * (alpha_ * rmse + (lambda_ * coef ** 2).sum())
                self.scores_.append(s)
            if it > 0 and np.sum(np.abs(coef_old - coef)) < self.tol:
                break
            coef_old = coef.copy()
            if not keep.any():
                break
        if keep.any():
            sigma = update_sigma(alpha_, lambda_, keep)
            coef = update_coef(coef, alpha_, keep, sigma)
        else:
            sigma = np.zeros((0, 0))
        self.n_iter_ = it + 1
        self.coef_, self.alpha_, self.sigma_, self.lambda_ = coef, alpha_, sigma, lambda_
        self._set_intercept(X_offset, y_offset, X_scale)
        return self

    def predict(self, X, return_std=False):
        y_mean = self._decision_function(X)
        if not return_std:
            return y_mean
        X = _as_dense64(X)
        if self.normalize:
            X = (X - self.X_offset_) / self.X_scale_
        X = X[:, self.lambda_ < self.threshold_lambda]
        var = ((X @ self.sigma_) * X).sum(axis=1)
        return y_mean, np.sqrt(var + 1. / self.alpha_)
