"""Remaining decomposition estimators (reference ``sklearn/decomposition``):
``KernelPCA`` (``_kernel_pca.py``), ``FastICA`` / ``fastica``
(``_fastica.py``), ``FactorAnalysis`` (``_factor_analysis.py``), ``NMF`` /
``non_negative_factorization`` (``_nmf.py`` + ``_cdnmf_fast.pyx``, N28)
and ``LatentDirichletAllocation`` (``_lda.py`` + ``_online_lda_fast.pyx``,
N28).

Kernel matrices and eigendecompositions run in fp64 on the resolved
device; the NMF coordinate-descent sweep and the LDA E-step are host C++
(``csrc/host/decomposition_host.cpp``) - both are sequential per column /
per document with tiny inner loops, where a GPU launch per step would cost
more than the work.
"""

import ctypes
import numbers
import os
import warnings

import numpy as np
import scipy.sparse as sp
import torch
from scipy import linalg
from scipy.sparse.linalg import eigsh
from scipy.special import gammaln, logsumexp

from ...base import BaseEstimator, TransformerMixin
from ...exceptions import ConvergenceWarning
from ...ops import _host
from ...runtime.device import resolve_device
from ...utils.extmath import randomized_svd, svd_flip
from ...utils.validation import check_array, check_is_fitted, check_random_state

EPSILON = np.finfo(np.float32).eps


def _c(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def _dense(X):
    if hasattr(X, "detach"):
        X = X.detach().cpu().numpy()
    return np.array(X.toarray() if sp.issparse(X) else X, dtype=np.float64)


# ------------------------------------------------------------------ KernelPCA
class KernelPCA(TransformerMixin, BaseEstimator):
    """Kernel PCA: eigendecomposition of the centred kernel matrix."""

    def __init__(self, n_components=None, *, kernel="linear", gamma=None, degree=3, coef0=1,
                 kernel_params=None, alpha=1.0, fit_inverse_transform=False, eigen_solver="auto",
                 tol=0, max_iter=None, iterated_power="auto", remove_zero_eig=False,
                 random_state=None, copy_X=True, n_jobs=None):
        self.n_components = n_components
        self.kernel = kernel
        self.kernel_params = kernel_params
        self.gamma = gamma
        self.degree = degree
        self.coef0 = coef0
        self.alpha = alpha
        self.fit_inverse_transform = fit_inverse_transform
        self.eigen_solver = eigen_solver
        self.tol = tol
        self.max_iter = max_iter
        self.iterated_power = iterated_power
        self.remove_zero_eig = remove_zero_eig
        self.random_state = random_state
        self.copy_X = copy_X
        self.n_jobs = n_jobs

    def _get_kernel(self, X, Y=None):
        from ...metrics import pairwise_kernels
        if self.kernel == "precomputed":
            return np.asarray(X, dtype=np.float64)
        if callable(self.kernel):
            params = self.kernel_params or {}
        else:
            params = {"gamma": self.gamma, "degree": self.degree, "coef0": self.coef0}
            params = {k: v for k, v in params.items()
                      if k in _KERNEL_PARAMS.get(self.kernel, ())}
        K = pairwise_kernels(X, Y, metric=self.kernel, **params)
        return np.asarray(K.detach().cpu().numpy() if hasattr(K, "detach") else K,
                          dtype=np.float64)

    def _fit_transform(self, K):
        from ...preprocessing import KernelCenterer
        self._centerer = KernelCenterer()
        K = np.asarray(self._centerer.fit_transform(K), dtype=np.float64)
        n = K.shape[0]
        nc = n if self.n_components is None else min(n, self.n_components)
        solver = self.eigen_solver
        if solver == "auto":
            solver = "arpack" if n > 200 and nc < 10 else "dense"
        if solver == "dense":
            dev = resolve_device(None)
            w, V = torch.linalg.eigh(torch.as_tensor(K, device=dev))
            w, V = w[n - nc:].cpu().numpy(), V[:, n - nc:].cpu().numpy()
        elif solver == "arpack":
            v0 = check_random_state(self.random_state).uniform(-1, 1, n)
            w, V = eigsh(K, nc, which="LA", tol=self.tol, maxiter=self.max_iter, v0=v0)
        elif solver == "randomized":
            U, S, Vt = randomized_svd(K, nc, n_iter=4 if self.iterated_power == "auto"
                                      else self.iterated_power,
                                      random_state=self.random_state, flip_sign=False)
            w = S * np.sign(np.sum(U * Vt.T, axis=0))
            V = U
        else:
            raise ValueError("Unsupported value for `eigen_solver`: %r" % solver)
        w = np.where(w < 0, 0.0, w) if (w < 0).any() and np.abs(w[w < 0]).max() < \
            1e-5 * max(np.abs(w).max(), 1e-300) else w
        w = np.maximum(w, 0.0)
        V, _ = svd_flip(V, np.zeros_like(V).T)
        order = w.argsort()[::-1]
        self.eigenvalues_, self.eigenvectors_ = w[order], V[:, order]
        if self.remove_zero_eig or self.n_components is None:
            keep = self.eigenvalues_ > 0
            self.eigenvectors_ = self.eigenvectors_[:, keep]
            self.eigenvalues_ = self.eigenvalues_[keep]
        return K

    @property
    def lambdas_(self):
        return self.eigenvalues_

    @property
    def alphas_(self):
        return self.eigenvectors_

    def fit(self, X, y=None):
        if self.fit_inverse_transform and self.kernel == "precomputed":
            raise ValueError("Cannot fit_inverse_transform with a precomputed kernel.")
        X = _dense(X)
        self.n_features_in_ = X.shape[1]
        self._fit_transform(self._get_kernel(X))
        if self.fit_inverse_transform:
            Xt = self.eigenvectors_ * np.sqrt(self.eigenvalues_)
            K = self._get_kernel(Xt)
            K.flat[::K.shape[0] + 1] += self.alpha
            self.dual_coef_ = linalg.solve(K, X, assume_a="pos", overwrite_a=True)
            self.X_transformed_fit_ = Xt
        self.X_fit_ = X
        return self

    def fit_transform(self, X, y=None, **params):
        self.fit(X, **params)
        return self.eigenvectors_ * np.sqrt(self.eigenvalues_)

    def transform(self, X):
        check_is_fitted(self, "eigenvectors_")
        X = _dense(X)
        if self.kernel != "precomputed" and X.shape[1] != self.n_features_in_:
            raise ValueError("X has %d features, but KernelPCA is expecting %d features as "
                             "input." % (X.shape[1], self.n_features_in_))
        K = self._centerer.transform(self._get_kernel(X, self.X_fit_))
        nz = np.flatnonzero(self.eigenvalues_)
        sa = np.zeros_like(self.eigenvectors_)
        sa[:, nz] = self.eigenvectors_[:, nz] / np.sqrt(self.eigenvalues_[nz])
        return np.asarray(K) @ sa

    def inverse_transform(self, X):
        if not self.fit_inverse_transform:
            raise ValueError("The fit_inverse_transform parameter was not set to True when "
                             "instantiating and hence the inverse transform is not available.")
        return self._get_kernel(_dense(X), self.X_transformed_fit_) @ self.dual_coef_


_KERNEL_PARAMS = {"rbf": ("gamma",), "poly": ("gamma", "degree", "coef0"),
                  "polynomial": ("gamma", "degree", "coef0"), "sigmoid": ("gamma", "coef0"),
                  "laplacian": ("gamma",), "chi2": ("gamma",), "linear": (), "cosine": (),
                  "precomputed": (), "additive_chi2": ()}


# -------------------------------------------------------------------- FastICA
def _logcosh(x, fun_args=None):
    alpha = (fun_args or {}).get("alpha", 1.0)
    x *= alpha
    gx = np.tanh(x, x)
    g_x = np.empty(x.shape[0])
    for i, gxi in enumerate(gx):
        g_x[i] = (alpha * (1 - gxi ** 2)).mean()
    return gx, g_x


def _exp(x, fun_args=None):
    e = np.exp(-(x ** 2) / 2)
    return x * e, ((1 - x ** 2) * e).mean(axis=-1)


def _cube(x, fun_args=None):
    return x ** 3, (3 * x ** 2).mean(axis=-1)


def _sym_decorrelation(W):
    s, u = linalg.eigh(W @ W.T)
    return np.linalg.multi_dot([u * (1.0 / np.sqrt(s)), u.T, W])


def _ica_par(X, tol, g, fun_args, max_iter, w_init):
    W = _sym_decorrelation(w_init)
    p_ = float(X.shape[1])
    for ii in range(max_iter):
        gwtx, g_wtx = g(W @ X, fun_args)
        W1 = _sym_decorrelation(gwtx @ X.T / p_ - g_wtx[:, np.newaxis] * W)
        lim = max(abs(abs(np.diag(W1 @ W.T)) - 1))
        W = W1
        if lim < tol:
            break
    else:
        warnings.warn("FastICA did not converge. Consider increasing tolerance or the maximum "
                      "number of iterations.", ConvergenceWarning)
    return W, ii + 1


def _ica_def(X, tol, g, fun_args, max_iter, w_init):
    nc = w_init.shape[0]
    W = np.zeros((nc, nc), dtype=X.dtype)
    n_iter = []
    for j in range(nc):
        w = w_init[j, :].copy()
        w /= np.sqrt((w ** 2).sum())
        for i in range(max_iter):
            gwtx, g_wtx = g(w.T @ X, fun_args)
            w1 = (X * gwtx).mean(axis=1) - g_wtx.mean() * w
            w1 -= np.linalg.multi_dot([w1, W[:j].T, W[:j]])
            w1 /= np.sqrt((w1 ** 2).sum())
            lim = np.abs(np.abs((w1 * w).sum()) - 1)
            w = w1
            if lim < tol:
                break
        n_iter.append(i + 1)
        W[j, :] = w
    return W, max(n_iter)


class FastICA(TransformerMixin, BaseEstimator):
    """Fast independent component analysis (parallel or deflation)."""

    def __init__(self, n_components=None, *, algorithm="parallel", whiten=True, fun="logcosh",
                 fun_args=None, max_iter=200, tol=1e-4, w_init=None, random_state=None):
        self.n_components = n_components
        self.algorithm = algorithm
        self.whiten = whiten
        self.fun = fun
        self.fun_args = fun_args
        self.max_iter = max_iter
        self.tol = tol
        self.w_init = w_init
        self.random_state = random_state

    def _fit(self, X, compute_sources=False):
        X = _dense(X)
        if X.shape[0] < 2:
            raise ValueError("FastICA requires at least 2 samples")
        self.n_features_in_ = X.shape[1]
        X = X.T
        fun_args = {} if self.fun_args is None else self.fun_args
        rs = check_random_state(self.random_state)
        if self.fun == "logcosh":
            g = _logcosh
        elif self.fun == "exp":
            g = _exp
        elif self.fun == "cube":
            g = _cube
        elif callable(self.fun):
            def g(x, fa):
                return self.fun(x, **fa)
        else:
            raise ValueError("Unknown function %r; should be one of 'logcosh', 'exp', 'cube' or "
                             "callable" % self.fun)
        n_features, n_samples = X.shape
        whiten = self.whiten
        if whiten is True:
            whiten = "arbitrary-variance"
        nc = self.n_components
        if not whiten and nc is not None:
            nc = None
            warnings.warn("Ignoring n_components with whiten=False.")
        if nc is None:
            nc = min(n_samples, n_features)
        if nc > min(n_samples, n_features):
            nc = min(n_samples, n_features)
            warnings.warn("n_components is too large: it will be set to %s" % nc)
        if whiten:
            X_mean = X.mean(axis=-1)
            X = X - X_mean[:, np.newaxis]
            u, d, _ = linalg.svd(X, full_matrices=False, check_finite=False)
            K = (u / d).T[:nc]
            X1 = (K @ X) * np.sqrt(n_samples)
        else:
            X1 = X.copy()
        w_init = self.w_init
        if w_init is None:
            w_init = np.asarray(rs.normal(size=(nc, nc)), dtype=X1.dtype)
        else:
            w_init = np.asarray(w_init)
            if w_init.shape != (nc, nc):
                raise ValueError("w_init has invalid shape -- should be %(shape)s"
                                 % {"shape": (nc, nc)})
        kw = dict(tol=self.tol, g=g, fun_args=fun_args, max_iter=self.max_iter, w_init=w_init)
        if self.algorithm == "parallel":
            W, n_iter = _ica_par(X1, **kw)
        elif self.algorithm == "deflation":
            W, n_iter = _ica_def(X1, **kw)
        else:
            raise ValueError("Invalid algorithm: must be either `parallel` or `deflation`.")
        S = None
        if compute_sources:
            S = (np.linalg.multi_dot([W, K, X]) if whiten else W @ X).T
        self.n_iter_ = n_iter
        if whiten:
            self.components_ = W @ K
            self.mean_ = X_mean
            self.whitening_ = K
        else:
            self.components_ = W
        if whiten == "unit-variance":
            if S is None:
                S = np.linalg.multi_dot([W, K, X]).T
            std = np.std(S, axis=0, keepdims=True)
            S = S / std
            self.components_ = self.components_ / std.T
        self.mixing_ = linalg.pinv(self.components_, check_finite=False)
        self._unmixing = W
        return S

    def fit_transform(self, X, y=None):
        return self._fit(X, compute_sources=True)

    def fit(self, X, y=None):
        self._fit(X, compute_sources=False)
        return self

    def transform(self, X, copy=True):
        check_is_fitted(self, "components_")
        X = _dense(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError("X has %d features, but FastICA is expecting %d features as input."
                             % (X.shape[1], self.n_features_in_))
        if self.whiten:
            X = X - self.mean_
        return X @ self.components_.T

    def inverse_transform(self, X, copy=True):
        check_is_fitted(self, "components_")
        X = _dense(X) @ self.mixing_.T
        if self.whiten:
            X += self.mean_
        return X


def fastica(X, n_components=None, *, algorithm="parallel", whiten=True, fun="logcosh",
            fun_args=None, max_iter=200, tol=1e-04, w_init=None, random_state=None,
            return_X_mean=False, compute_sources=True, return_n_iter=False):
    est = FastICA(n_components=n_components, algorithm=algorithm, whiten=whiten, fun=fun,
                  fun_args=fun_args, max_iter=max_iter, tol=tol, w_init=w_init,
                  random_state=random_state)
    S = est._fit(X, compute_sources=compute_sources)
    if whiten:
        out = [est.whitening_, est._unmixing, S]
        if return_X_mean:
            out.append(est.mean_)
    else:
        out = [None, est._unmixing, S]
        if return_X_mean:
            out.append(None)
    if return_n_iter:
        out.append(est.n_iter_)
    return tuple(out)


# ------------------------------------------------------------ FactorAnalysis
def _ortho_rotation(components, method="varimax", tol=1e-6, max_iter=100):
    nrow, ncol = components.shape
    R = np.eye(ncol)
    var = 0
    for _ in range(max_iter):
        cr = components @ R
        tmp = cr * np.transpose((cr ** 2).sum(axis=0) / nrow) if method == "varimax" else 0
        u, s, v = np.linalg.svd(components.T @ (cr ** 3 - tmp))
        R = u @ v
        var_new = np.sum(s)
        if var != 0 and var_new < var * (1 + tol):
            break
        var = var_new
    return (components @ R).T


class FactorAnalysis(TransformerMixin, BaseEstimator):
    """Gaussian latent factor model fitted by SVD-based EM."""

    def __init__(self, n_components=None, *, tol=1e-2, copy=True, max_iter=1000,
                 noise_variance_init=None, svd_method="randomized", iterated_power=3,
                 rotation=None, random_state=0):
        self.n_components = n_components
        self.copy = copy
        self.tol = tol
        self.max_iter = max_iter
        if svd_method not in ["lapack", "randomized"]:
            raise ValueError("SVD method %s is not supported. Please consider the documentation"
                             % svd_method)
        self.svd_method = svd_method
        self.noise_variance_init = noise_variance_init
        self.iterated_power = iterated_power
        self.random_state = random_state
        self.rotation = rotation

    def fit(self, X, y=None):
        X = _dense(X)
        n, d = X.shape
        self.n_features_in_ = d
        nc = d if self.n_components is None else self.n_components
        self.mean_ = X.mean(axis=0)
        X = X - self.mean_
        nsqrt = np.sqrt(n)
        llconst = d * np.log(2.0 * np.pi) + nc
        var = np.var(X, axis=0)
        psi = np.ones(d) if self.noise_variance_init is None else \
            np.array(self.noise_variance_init, dtype=np.float64)
        if psi.shape != (d,):
            raise ValueError("noise_variance_init dimension does not with number of features : "
                             "%d != %d" % (len(psi), d))
        loglike, old_ll, SMALL = [], -np.inf, 1e-12
        if self.svd_method == "lapack":
            def my_svd(A):
                _, s, Vt = linalg.svd(A, full_matrices=False, check_finite=False)
                return s[:nc], Vt[:nc], np.sum(s[nc:] ** 2)
        else:
            rs = check_random_state(self.random_state)

            def my_svd(A):
                _, s, Vt = randomized_svd(A, nc, random_state=rs, n_iter=self.iterated_power)
                return s, Vt, np.sum(A * A) - np.sum(s * s)
        for i in range(self.max_iter):
            sqrt_psi = np.sqrt(psi) + SMALL
            s, Vt, unexp = my_svd(X / (sqrt_psi * nsqrt))
            s **= 2
            W = np.sqrt(np.maximum(s - 1.0, 0.0))[:, np.newaxis] * Vt
            W *= sqrt_psi
            ll = llconst + np.sum(np.log(s))
            ll += unexp + np.sum(np.log(psi))
            ll *= -n / 2.0
            loglike.append(ll)
            if (ll - old_ll) < self.tol:
                break
            old_ll = ll
            psi = np.maximum(var - np.sum(W ** 2, axis=0), SMALL)
        else:
            warnings.warn("FactorAnalysis did not converge. You might want to increase the "
                          "number of iterations.", ConvergenceWarning)
        self.components_ = W
        if self.rotation is not None:
            if self.rotation not in ("varimax", "quartimax"):
                raise ValueError("'method' must be in %s, not %s"
                                 % (("varimax", "quartimax"), self.rotation))
            self.components_ = _ortho_rotation(W.T, method=self.rotation)[:nc]
        self.noise_variance_ = psi
        self.loglike_ = loglike
        self.n_iter_ = i + 1
        return self

    def transform(self, X):
        check_is_fitted(self, "components_")
        X = _dense(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError("X has %d features, but FactorAnalysis is expecting %d features as "
                             "input." % (X.shape[1], self.n_features_in_))
        Ih = np.eye(len(self.components_))
        Wpsi = self.components_ / self.noise_variance_
        cov_z = linalg.inv(Ih + Wpsi @ self.components_.T)
        return ((X - self.mean_) @ Wpsi.T) @ cov_z

    def get_covariance(self):
        check_is_fitted(self, "components_")
        cov = self.components_.T @ self.components_
        cov.flat[::len(cov) + 1] += self.noise_variance_
        return cov

    def get_precision(self):
        check_is_fitted(self, "components_")
        nf = len(self.components_[0])
        if len(self.components_) == 0:
            return np.diag(1.0 / self.noise_variance_)
        if len(self.components_) == nf:
            return linalg.inv(self.get_covariance())
        c = self.components_
        prec = c / self.noise_variance_
        prec = c @ prec.T
        prec.flat[::len(prec) + 1] += 1.0
        prec = (c.T @ linalg.inv(prec)) @ c
        prec /= self.noise_variance_[:, np.newaxis]
        prec /= -self.noise_variance_[np.newaxis, :]
        prec.flat[::len(prec) + 1] += 1.0 / self.noise_variance_
        return prec

    def score_samples(self, X):
        check_is_fitted(self, "components_")
        Xr = _dense(X) - self.mean_
        P = self.get_precision()
        ll = -0.5 * (Xr * (Xr @ P)).sum(axis=1)
        sign, ld = np.linalg.slogdet(P)
        ll -= 0.5 * (Xr.shape[1] * np.log(2.0 * np.pi) - (ld if sign > 0 else -np.inf))
        return ll

    def score(self, X, y=None):
        return np.mean(self.score_samples(X))


# ------------------------------------------------------------------------ NMF
def _beta_loss_to_float(beta_loss):
    table = {"frobenius": 2, "kullback-leibler": 1, "itakura-saito": 0}
    if isinstance(beta_loss, str) and beta_loss in table:
        return table[beta_loss]
    if not isinstance(beta_loss, numbers.Number):
        raise ValueError("Invalid beta_loss parameter: got %r instead of one of %r, or a float."
                         % (beta_loss, list(table)))
    return beta_loss


def _beta_divergence(X, W, H, beta, square_root=False):
    beta = _beta_loss_to_float(beta)
    WH = W @ H
    if beta == 2:
        res = np.sum((X - WH) ** 2) / 2.0
        return np.sqrt(res * 2) if square_root else res
    Xd, WHd = X.ravel(), WH.ravel()
    idx = Xd > EPSILON
    WHd, Xd = WHd[idx], Xd[idx]
    WHd[WHd == 0] = EPSILON
    if beta == 1:
        res = Xd @ np.log(Xd / WHd) + np.sum(W, axis=0) @ np.sum(H, axis=1) - Xd.sum()
    elif beta == 0:
        div = Xd / WHd
        res = np.sum(div) - np.prod(X.shape) - np.sum(np.log(div))
    else:
        res = (Xd ** beta).sum() - beta * (Xd @ WHd ** (beta - 1))
        res += np.sum(WH ** beta) * (beta - 1)
        res /= beta * (beta - 1)
    return np.sqrt(2 * res) if square_root else res


def _initialize_nmf(X, n_components, init=None, eps=1e-6, random_state=None):
    if init == "warn":
        init = None
    n, d = X.shape
    if init is None:
        init = "nndsvd" if n_components <= min(n, d) else "random"
    if init == "random":
        avg = np.sqrt(X.mean() / n_components)
        rng = check_random_state(random_state)
        H = np.abs(avg * rng.randn(n_components, d))
        W = np.abs(avg * rng.randn(n, n_components))
        return W, H
    U, S, V = randomized_svd(X, n_components, random_state=random_state)
    W, H = np.zeros_like(U), np.zeros_like(V)
    W[:, 0] = np.sqrt(S[0]) * np.abs(U[:, 0])
    H[0, :] = np.sqrt(S[0]) * np.abs(V[0, :])
    for j in range(1, n_components):
        x, y = U[:, j], V[j, :]
        xp, yp = np.maximum(x, 0), np.maximum(y, 0)
        xn, yn = np.abs(np.minimum(x, 0)), np.abs(np.minimum(y, 0))
        xpn, ypn, xnn, ynn = (np.sqrt(np.sum(v * v)) for v in (xp, yp, xn, yn))
        mp, mn = xpn * ypn, xnn * ynn
        if mp > mn:
            u, v, sigma = xp / xpn, yp / ypn, mp
        else:
            u, v, sigma = xn / xnn, yn / ynn, mn
        lbd = np.sqrt(S[j] * sigma)
        W[:, j], H[j, :] = lbd * u, lbd * v
    W[W < eps] = 0
    H[H < eps] = 0
    if init == "nndsvda":
        avg = X.mean()
        W[W == 0] = avg
        H[H == 0] = avg
    elif init == "nndsvdar":
        rng = check_random_state(random_state)
        avg = X.mean()
        W[W == 0] = abs(avg * rng.randn(len(W[W == 0])) / 100)
        H[H == 0] = abs(avg * rng.randn(len(H[H == 0])) / 100)
    elif init != "nndsvd":
        raise ValueError("Invalid init parameter: got %r instead of one of %r"
                         % (init, (None, "random", "nndsvd", "nndsvda", "nndsvdar")))
    return W, H


def _cd_sweep(X, W, Ht, l1, l2, shuffle, rng):
    k = Ht.shape[1]
    HHt = Ht.T @ Ht
    XHt = np.ascontiguousarray(X @ Ht)
    if l2 != 0.0:
        HHt.flat[::k + 1] += l2
    if l1 != 0.0:
        XHt -= l1
    perm = rng.permutation(k) if shuffle else np.arange(k)
    perm = np.ascontiguousarray(perm, dtype=np.int64)
    HHt = np.ascontiguousarray(HHt)
    return _host.lib().sqh_cdnmf_update(_c(W), _c(HHt), _c(XHt), _c(perm), W.shape[0], k)


def _fit_cd(X, W, H, tol, max_iter, l1W, l1H, l2W, l2H, update_H, shuffle, random_state):
    Ht = np.ascontiguousarray(H.T)
    W = np.ascontiguousarray(W)
    rng = check_random_state(random_state)
    XT = np.ascontiguousarray(X.T)
    for n_iter in range(1, max_iter + 1):
        v = _cd_sweep(X, W, Ht, l1W, l2W, shuffle, rng)
        if update_H:
            v += _cd_sweep(XT, Ht, W, l1H, l2H, shuffle, rng)
        if n_iter == 1:
            v0 = v
        if v0 == 0 or v / v0 <= tol:
            break
    return W, Ht.T, n_iter


def _mu_w(X, W, H, beta, l1, l2, gamma, H_sum, HHt, XHt, update_H):
    if beta == 2:
        if XHt is None:
            XHt = X @ H.T
        num = XHt if update_H else XHt.copy()
        if HHt is None:
            HHt = H @ H.T
        den = W @ HHt
    else:
        WH = W @ H
        WHs = WH.copy()
        if beta - 1.0 < 0:
            WH[WH == 0] = EPSILON
        if beta - 2.0 < 0:
            WHs[WHs == 0] = EPSILON
        if beta == 1:
            WHs = X / WHs
        elif beta == 0:
            WHs = X * WHs ** -2
        else:
            WHs = X * WHs ** (beta - 2)
        num = WHs @ H.T
        if beta == 1:
            if H_sum is None:
                H_sum = np.sum(H, axis=1)
            den = H_sum[np.newaxis, :]
        else:
            den = (WH ** (beta - 1)) @ H.T
    if l1 > 0:
        den = den + l1
    if l2 > 0:
        den = den + l2 * W
    den = np.where(den == 0, EPSILON, den)
    delta = num / den
    if gamma != 1:
        delta **= gamma
    return delta, H_sum, HHt, XHt


def _mu_h(X, W, H, beta, l1, l2, gamma):
    if beta == 2:
        num = W.T @ X
        den = np.linalg.multi_dot([W.T, W, H])
    else:
        WH = W @ H
        WHs = WH.copy()
        if beta - 1.0 < 0:
            WH[WH == 0] = EPSILON
        if beta - 2.0 < 0:
            WHs[WHs == 0] = EPSILON
        if beta == 1:
            WHs = X / WHs
        elif beta == 0:
            WHs = X * WHs ** -2
        else:
            WHs = X * WHs ** (beta - 2)
        num = W.T @ WHs
        if beta == 1:
            ws = np.sum(W, axis=0)
            ws[ws == 0] = 1.0
            den = ws[:, np.newaxis]
        else:
            den = W.T @ WH ** (beta - 1)
    if l1 > 0:
        den = den + l1
    if l2 > 0:
        den = den + l2 * H
    den = np.where(den == 0, EPSILON, den)
    delta = num / den
    if gamma != 1:
        delta **= gamma
    return delta


def _fit_mu(X, W, H, beta, max_iter, tol, l1W, l1H, l2W, l2H, update_H):
    beta = _beta_loss_to_float(beta)
    gamma = 1.0 / (2.0 - beta) if beta < 1 else (1.0 / (beta - 1.0) if beta > 2 else 1.0)
    err0 = _beta_divergence(X, W, H, beta, square_root=True)
    prev = err0
    H_sum = HHt = XHt = None
    for n_iter in range(1, max_iter + 1):
        dW, H_sum, HHt, XHt = _mu_w(X, W, H, beta, l1W, l2W, gamma, H_sum, HHt, XHt, update_H)
        W *= dW
        if beta < 1:
            W[W < np.finfo(np.float64).eps] = 0.0
        if update_H:
            H *= _mu_h(X, W, H, beta, l1H, l2H, gamma)
            H_sum = HHt = XHt = None
            if beta <= 1:
                H[H < np.finfo(np.float64).eps] = 0.0
        if tol > 0 and n_iter % 10 == 0:
            err = _beta_divergence(X, W, H, beta, square_root=True)
            if (prev - err) / err0 < tol:
                break
            prev = err
    return W, H, n_iter


class NMF(TransformerMixin, BaseEstimator):
    """Non-negative matrix factorisation X ~ W H (coordinate descent or
    multiplicative updates; Frobenius / KL / IS / beta losses)."""

    def _more_tags(self):
        return {"requires_positive_X": True}


    def __init__(self, n_components=None, *, init="warn", solver="cd", beta_loss="frobenius",
                 tol=1e-4, max_iter=200, random_state=None, alpha=0.0, l1_ratio=0.0, verbose=0,
                 shuffle=False, regularization="both"):
        self.n_components = n_components
        self.init = init
        self.solver = solver
        self.beta_loss = beta_loss
        self.tol = tol
        self.max_iter = max_iter
        self.random_state = random_state
        self.alpha = alpha
        self.l1_ratio = l1_ratio
        self.verbose = verbose
        self.shuffle = shuffle
        self.regularization = regularization

    def _regs(self):
        aH = float(self.alpha) if self.regularization in ("both", "components") else 0.0
        aW = float(self.alpha) if self.regularization in ("both", "transformation") else 0.0
        r = self.l1_ratio
        return aW * r, aH * r, aW * (1.0 - r), aH * (1.0 - r)

    def _fit_transform(self, X, W=None, H=None, update_H=True):
        if (X < 0).any():
            raise ValueError("Negative values in data passed to NMF (input X)")
        if self.solver not in ("cd", "mu"):
            raise ValueError("Invalid solver parameter: got %r instead of one of %r"
                             % (self.solver, ("cd", "mu")))
        beta = _beta_loss_to_float(self.beta_loss)
        if self.solver == "cd" and beta != 2:
            raise ValueError("Invalid beta_loss parameter: solver %r does not handle beta_loss = "
                             "%r" % (self.solver, self.beta_loss))
        if self.solver == "mu" and self.init == "nndsvd":
            warnings.warn("The multiplicative update ('mu') solver cannot update zeros present "
                          "in the initialization, and so leads to poorer results when used "
                          "jointly with init='nndsvd'. You may try init='nndsvda' or "
                          "init='nndsvdar' instead.", UserWarning)
        if X.min() == 0 and beta <= 0:
            raise ValueError("When beta_loss <= 0 and X contains zeros, the solver may diverge. "
                             "Please add small values to X, or use a positive beta_loss.")
        n, d = X.shape
        nc = d if self.n_components is None else self.n_components
        if not isinstance(nc, numbers.Integral) or nc <= 0:
            raise ValueError("Number of components must be a positive integer; got "
                             "(n_components=%r)" % nc)
        self._n_components = nc
        if self.init == "custom" and update_H:
            W, H = np.array(W, dtype=np.float64), np.array(H, dtype=np.float64)
        elif not update_H:
            H = np.asarray(H, dtype=np.float64)
            W = np.full((n, nc), np.sqrt(X.mean() / nc)) if self.solver == "mu" else \
                np.zeros((n, nc))
        else:
            W, H = _initialize_nmf(X, nc, init=self.init, random_state=self.random_state)
        l1W, l1H, l2W, l2H = self._regs()
        if self.solver == "cd":
            W, H, n_iter = _fit_cd(X, W, H, self.tol, self.max_iter, l1W, l1H, l2W, l2H, update_H,
                                   self.shuffle, self.random_state)
        else:
            W, H, n_iter = _fit_mu(X, W, H, beta, self.max_iter, self.tol, l1W, l1H, l2W, l2H,
                                   update_H)
        if n_iter == self.max_iter and self.tol > 0:
            warnings.warn("Maximum number of iterations %d reached. Increase it to improve "
                          "convergence." % self.max_iter, ConvergenceWarning)
        return W, H, n_iter

    def fit_transform(self, X, y=None, W=None, H=None):
        X = _dense(X)
        self.n_features_in_ = X.shape[1]
        W, H, n_iter = self._fit_transform(X, W=W, H=H)
        self.reconstruction_err_ = _beta_divergence(X, W, H, self.beta_loss, square_root=True)
        self.n_components_ = H.shape[0]
        self.components_ = H
        self.n_iter_ = n_iter
        return W

    def fit(self, X, y=None, **params):
        self.fit_transform(X, **params)
        return self

    def transform(self, X):
        check_is_fitted(self, "components_")
        X = _dense(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError("X has %d features, but NMF is expecting %d features as input."
                             % (X.shape[1], self.n_features_in_))
        return self._fit_transform(X, H=self.components_, update_H=False)[0]

    def inverse_transform(self, W):
        check_is_fitted(self, "components_")
        return W @ self.components_


def non_negative_factorization(X, W=None, H=None, n_components=None, *, init="warn",
                               update_H=True, solver="cd", beta_loss="frobenius", tol=1e-4,
                               max_iter=200, alpha=0.0, l1_ratio=0.0, regularization=None,
                               random_state=None, verbose=0, shuffle=False):
    est = NMF(n_components=n_components, init=init, solver=solver, beta_loss=beta_loss, tol=tol,
              max_iter=max_iter, random_state=random_state, alpha=alpha, l1_ratio=l1_ratio,
              verbose=verbose, shuffle=shuffle,
              regularization=regularization if regularization is not None else "both")
    if regularization is None:
        est.alpha = 0.0
    X = _dense(X)
    return est._fit_transform(X, W=W, H=H, update_H=update_H)


# ------------------------------------------------------------------------ LDA
def _dirichlet_expectation_2d(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    out = np.empty_like(a)
    _host.lib().sqh_dirichlet_expectation_2d(_c(a), a.shape[0], a.shape[1], _c(out))
    return out


def _as_csr(X):
    X = sp.csr_matrix(X, dtype=np.float64) if not sp.isspmatrix_csr(X) else X.astype(np.float64)
    X.sort_indices()
    return X


class LatentDirichletAllocation(TransformerMixin, BaseEstimator):
    """Latent Dirichlet allocation with batch or online variational Bayes."""

    def _more_tags(self):
        return {"requires_positive_X": True}


    def __init__(self, n_components=10, *, doc_topic_prior=None, topic_word_prior=None,
                 learning_method="batch", learning_decay=0.7, learning_offset=10.0, max_iter=10,
                 batch_size=128, evaluate_every=-1, total_samples=1e6, perp_tol=1e-1,
                 mean_change_tol=1e-3, max_doc_update_iter=100, n_jobs=None, verbose=0,
                 random_state=None):
        self.n_components = n_components
        self.doc_topic_prior = doc_topic_prior
        self.topic_word_prior = topic_word_prior
        self.learning_method = learning_method
        self.learning_decay = learning_decay
        self.learning_offset = learning_offset
        self.max_iter = max_iter
        self.batch_size = batch_size
        self.evaluate_every = evaluate_every
        self.total_samples = total_samples
        self.perp_tol = perp_tol
        self.mean_change_tol = mean_change_tol
        self.max_doc_update_iter = max_doc_update_iter
        self.n_jobs = n_jobs
        self.verbose = verbose
        self.random_state = random_state

    def _check(self, X, reset):
        X = _as_csr(X.detach().cpu().numpy() if hasattr(X, "detach") else X)
        if X.data.size and X.data.min() < 0:
            raise ValueError("Negative values in data passed to LatentDirichletAllocation")
        if reset:
            self.n_features_in_ = X.shape[1]
        elif X.shape[1] != self.components_.shape[1]:
            raise ValueError("The provided data has %d dimensions while the model was trained "
                             "with feature size %d." % (X.shape[1], self.components_.shape[1]))
        return X

    def _init_latent_vars(self, d):
        self.random_state_ = check_random_state(self.random_state)
        self.n_batch_iter_ = 1
        self.n_iter_ = 0
        self.doc_topic_prior_ = 1.0 / self.n_components if self.doc_topic_prior is None \
            else self.doc_topic_prior
        self.topic_word_prior_ = 1.0 / self.n_components if self.topic_word_prior is None \
            else self.topic_word_prior
        self.components_ = self.random_state_.gamma(100.0, 0.01, (self.n_components, d))
        self.exp_dirichlet_component_ = np.exp(_dirichlet_expectation_2d(self.components_))

    def _e_step(self, X, cal_sstats, random_init):
        n = X.shape[0]
        k = self.n_components
        dt = self.random_state_.gamma(100.0, 0.01, (n, k)) if random_init else np.ones((n, k))
        dt = np.ascontiguousarray(dt)
        ss = np.zeros(self.components_.shape) if cal_sstats else None
        etw = np.ascontiguousarray(self.exp_dirichlet_component_)
        ind = X.indices.astype(np.int64)
        ptr = X.indptr.astype(np.int64)
        nt = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
        _host.lib().sqh_lda_estep(_c(np.ascontiguousarray(X.data)), _c(ind), _c(ptr), n, k,
                                  X.shape[1], _c(etw), float(self.doc_topic_prior_),
                                  int(self.max_doc_update_iter), float(self.mean_change_tol),
                                  _c(dt), _c(ss), nt)
        if cal_sstats:
            ss *= self.exp_dirichlet_component_
        return dt, ss

    def _em_step(self, X, total_samples, batch_update):
        _, ss = self._e_step(X, cal_sstats=True, random_init=True)
        if batch_update:
            self.components_ = self.topic_word_prior_ + ss
        else:
            w = np.power(self.learning_offset + self.n_batch_iter_, -self.learning_decay)
            ratio = float(total_samples) / X.shape[0]
            self.components_ *= 1 - w
            self.components_ += w * (self.topic_word_prior_ + ratio * ss)
        self.exp_dirichlet_component_ = np.exp(_dirichlet_expectation_2d(self.components_))
        self.n_batch_iter_ += 1

    def fit(self, X, y=None):
        if self.learning_method not in ("batch", "online"):
            raise ValueError("Invalid 'learning_method' parameter: %r" % self.learning_method)
        X = self._check(X, reset=True)
        n = X.shape[0]
        self._init_latent_vars(X.shape[1])
        last = None
        for i in range(self.max_iter):
            if self.learning_method == "online":
                for s in range(0, n, self.batch_size):
                    self._em_step(X[s:s + self.batch_size], n, False)
            else:
                self._em_step(X, n, True)
            if self.evaluate_every > 0 and (i + 1) % self.evaluate_every == 0:
                dt, _ = self._e_step(X, False, False)
                bound = self._perplexity_precomp(X, dt, False)
                if last and abs(last - bound) < self.perp_tol:
                    break
                last = bound
            self.n_iter_ += 1
        dt, _ = self._e_step(X, False, False)
        self.bound_ = self._perplexity_precomp(X, dt, False)
        return self

    def partial_fit(self, X, y=None):
        first = not hasattr(self, "components_")
        X = self._check(X, reset=first)
        if first:
            self._init_latent_vars(X.shape[1])
        for s in range(0, X.shape[0], self.batch_size):
            self._em_step(X[s:s + self.batch_size], self.total_samples, False)
        return self

    def _unnormalized_transform(self, X):
        return self._e_step(X, False, False)[0]

    def transform(self, X):
        check_is_fitted(self, "components_")
        X = self._check(X, reset=False)
        dt = self._unnormalized_transform(X)
        return dt / dt.sum(axis=1)[:, np.newaxis]

    def _approx_bound(self, X, dt, sub_sampling):
        def ll(prior, distr, ddistr, size):
            s = np.sum((prior - distr) * ddistr)
            s += np.sum(gammaln(distr) - gammaln(prior))
            s += np.sum(gammaln(prior * size) - gammaln(np.sum(distr, 1)))
            return s
        n = dt.shape[0]
        d = self.components_.shape[1]
        ddt = _dirichlet_expectation_2d(dt)
        dcomp = _dirichlet_expectation_2d(self.components_)
        score = 0.0
        for i in range(n):
            ids = X.indices[X.indptr[i]:X.indptr[i + 1]]
            cnts = X.data[X.indptr[i]:X.indptr[i + 1]]
            score += cnts @ logsumexp(ddt[i, :, None] + dcomp[:, ids], axis=0)
        score += ll(self.doc_topic_prior_, dt, ddt, self.n_components)
        if sub_sampling:
            score *= float(self.total_samples) / n
        score += ll(self.topic_word_prior_, self.components_, dcomp, d)
        return score

    def score(self, X, y=None):
        check_is_fitted(self, "components_")
        X = self._check(X, reset=False)
        return self._approx_bound(X, self._unnormalized_transform(X), False)

    def _perplexity_precomp(self, X, dt, sub_sampling):
        bound = self._approx_bound(X, dt, sub_sampling)
        wc = X.sum() * (float(self.total_samples) / X.shape[0] if sub_sampling else 1.0)
        return np.exp(-1.0 * bound / wc)

    def perplexity(self, X, sub_sampling=False):
        check_is_fitted(self, "components_")
        X = self._check(X, reset=False)
        return self._perplexity_precomp(X, self._unnormalized_transform(X), sub_sampling)


__all__ = ["KernelPCA", "FastICA", "fastica", "FactorAnalysis", "NMF",
           "non_negative_factorization", "LatentDirichletAllocation"]
