"""Remaining linear models (reference ``sklearn/linear_model``):

* least-angle regression - ``lars_path`` / ``lars_path_gram``, ``Lars``,
  ``LassoLars``, ``LarsCV``, ``LassoLarsCV``, ``LassoLarsIC``
  (``_least_angle.py``).  The path is computed in the Gram domain with an
  incrementally grown Cholesky factor of the active set; the equiangular
  step, lasso sign-crossing drops and the alpha_min interpolation follow
  the reference's semantics.
* orthogonal matching pursuit - ``orthogonal_mp(_gram)``,
  ``OrthogonalMatchingPursuit(CV)`` (``_omp.py``).
* robust regression - ``HuberRegressor`` (``_huber.py``),
  ``RANSACRegressor`` (``_ransac.py``), ``TheilSenRegressor``
  (``_theil_sen.py``; the per-subset least squares are one batched
  pseudo-inverse on the device).
* GLMs - ``TweedieRegressor`` / ``PoissonRegressor`` / ``GammaRegressor``
  (``_glm/glm.py``; L-BFGS on the half deviance), ``QuantileRegressor``
  (``_quantile.py``; HiGHS linear program).
* multi-task - ``MultiTaskElasticNet(CV)`` / ``MultiTaskLasso(CV)``
  (``_coordinate_descent.py`` + ``_cd_fast.pyx`` multi-task CD).
* ``LogisticRegressionCV`` (``_logistic.py``).
"""

import warnings
from itertools import combinations
from math import log

import numpy as np
import scipy.sparse as sp
import torch
from scipy import interpolate, linalg, optimize
from scipy.special import binom, xlogy

from ...base import BaseEstimator, MetaEstimatorMixin, MultiOutputMixin, RegressorMixin, clone
from ...exceptions import ConvergenceWarning
from ...runtime.device import resolve_device
from ...utils.random import sample_without_replacement
from ...utils.validation import check_is_fitted, check_random_state
from ._base import (LinearClassifierMixin, LinearModel, _as_dense64, _check_sample_weight,
                    _preprocess_data)

_EPS64 = np.finfo(np.float64).eps


def _norm_flag(normalize, default):
    if isinstance(normalize, str) and normalize == "deprecated":
        return default
    return bool(normalize)


# ===================================================================== LARS
def _min_pos(a):
    a = a[a > 0]
    return a.min() if a.size else np.finfo(np.float64).max


def _lars_gram(Gram, Xy, n_samples, max_iter, alpha_min, method, eps, positive, return_path):
    """Least-angle / lasso path in the Gram domain."""
    if method == "lar" and positive:
        raise ValueError("Positive constraint not supported for 'lar' coding method.")
    p = Gram.shape[0]
    C = np.array(Xy, dtype=np.float64)
    max_features = min(max_iter, p)
    tiny32 = np.finfo(np.float32).tiny
    eq_tol = np.finfo(np.float32).eps
    coef = np.zeros(p)
    prev_coef = np.zeros(p)
    alphas, coefs = [], []
    active, signs = [], []
    L = np.zeros((max_features + 1, max_features + 1))
    in_active = np.zeros(p, dtype=bool)
    excluded = np.zeros(p, dtype=bool)
    n_iter = 0
    drop = False
    prev_alpha = 0.0
    while True:
        cand = ~in_active & ~excluded
        if cand.any():
            cc = np.where(cand, C, -np.inf if positive else 0.0)
            j = int(np.argmax(cc) if positive else np.argmax(np.abs(np.where(cand, C, 0.0))))
            Cj = C[j]
            Cmax = Cj if positive else abs(Cj)
        elif active:
            j, Cj = -1, 0.0
            Cmax = abs(C[active[0]]) if not positive else C[active[0]]
        else:
            j, Cj, Cmax = -1, 0.0, 0.0
        alpha = Cmax / n_samples
        if alpha <= alpha_min + eq_tol:
            if abs(alpha - alpha_min) > eq_tol:
                if n_iter > 0:
                    ss = (prev_alpha - alpha_min) / (prev_alpha - alpha)
                    coef = prev_coef + ss * (coef - prev_coef)
                alpha = alpha_min
            alphas.append(alpha)
            coefs.append(coef.copy())
            break
        if n_iter >= max_iter or len(active) >= p:
            alphas.append(alpha)
            coefs.append(coef.copy())
            break
        if not drop:
            if j < 0:
                alphas.append(alpha)
                coefs.append(coef.copy())
                break
            k = len(active)
            g = Gram[j, active] if k else np.zeros(0)
            if k:
                g = linalg.solve_triangular(L[:k, :k], g, lower=True)
            diag = max(np.sqrt(abs(Gram[j, j] - g @ g)), eps)
            if diag < 1e-7:
                # degenerate direction: never select this feature again
                excluded[j] = True
                C[j] = 0.0
                continue
            L[k, :k] = g
            L[k, k] = diag
            active.append(j)
            in_active[j] = True
            signs.append(1.0 if positive else float(np.sign(Cj)))
        if method == "lasso" and n_iter > 0 and prev_alpha < alpha:
            break
        k = len(active)
        s = np.asarray(signs)
        ls = linalg.cho_solve((L[:k, :k], True), s)
        if ls.size == 1 and ls[0] == 0:
            ls[0] = 1.0
            AA = 1.0
        else:
            AA = 1.0 / np.sqrt(np.sum(ls * s))
            i = 0
            while not np.isfinite(AA):
                Lp = L[:k, :k].copy()
                Lp.flat[::k + 1] += 2 ** i * eps
                ls = linalg.cho_solve((Lp, True), s)
                AA = 1.0 / np.sqrt(max(np.sum(ls * s), eps))
                i += 1
            ls = ls * AA
        a = Gram[:, active] @ ls
        inact = ~in_active & ~excluded
        Ci, ai = C[inact], a[inact]
        g1 = _min_pos((Cmax - Ci) / (AA - ai + tiny32))
        if positive:
            gamma = min(g1, Cmax / AA)
        else:
            g2 = _min_pos((Cmax + Ci) / (AA + ai + tiny32))
            gamma = min(g1, g2, Cmax / AA)
        drop = False
        z = -coef[active] / (ls + tiny32)
        zpos = _min_pos(z)
        if zpos < gamma:
            idx = np.where(z == zpos)[0][::-1]
            for ii in idx:
                signs[ii] = -signs[ii]
            if method == "lasso":
                gamma = zpos
            drop = True
        n_iter += 1
        alphas.append(alpha)
        coefs.append(coef.copy())
        prev_coef = coef.copy()
        prev_alpha = alpha
        coef = coef.copy()
        coef[active] = prev_coef[active] + gamma * ls
        C = C - gamma * a
        if drop and method == "lasso":
            for ii in sorted(idx, reverse=True):
                jj = active.pop(ii)
                signs.pop(ii)
                in_active[jj] = False
                coef[jj] = 0.0
            # refactor the active Gram (drops are rare; exactness over speed)
            k = len(active)
            L[:, :] = 0.0
            if k:
                L[:k, :k] = linalg.cholesky(Gram[np.ix_(active, active)], lower=True)
    alphas = np.asarray(alphas)
    coefs = np.asarray(coefs).T
    if return_path:
        return alphas, list(active), coefs, n_iter
    return alphas[-1:], list(active), coefs[:, -1], n_iter


def lars_path(X, y, Xy=None, *, Gram=None, max_iter=500, alpha_min=0, method="lar",
              copy_X=True, eps=_EPS64, copy_Gram=True, verbose=0, return_path=True,
              return_n_iter=False, positive=False):
    """Least-angle (method='lar') or lasso (method='lasso') path."""
    if X is None and Gram is not None:
        raise ValueError("X cannot be None if Gram is not NoneUse lars_path_gram to avoid "
                         "passing X and y.")
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    G = X.T @ X if (Gram is None or isinstance(Gram, (str, bool))) else np.asarray(Gram)
    Xy = X.T @ y if Xy is None else np.asarray(Xy)
    a, act, c, n = _lars_gram(G, Xy, y.size, max_iter, alpha_min, method, eps, positive,
                              return_path)
    return (a, act, c, n) if return_n_iter else (a, act, c)


def lars_path_gram(Xy, Gram, *, n_samples, max_iter=500, alpha_min=0, method="lar",
                   copy_X=True, eps=_EPS64, copy_Gram=True, verbose=0, return_path=True,
                   return_n_iter=False, positive=False):
    a, act, c, n = _lars_gram(np.asarray(Gram, dtype=np.float64), np.asarray(Xy), n_samples,
                              max_iter, alpha_min, method, eps, positive, return_path)
    return (a, act, c, n) if return_n_iter else (a, act, c)


class Lars(MultiOutputMixin, RegressorMixin, LinearModel):
    method = "lar"
    positive = False

    def __init__(self, *, fit_intercept=True, verbose=False, normalize="deprecated",
                 precompute="auto", n_nonzero_coefs=500, eps=_EPS64, copy_X=True, fit_path=True,
                 jitter=None, random_state=None):
        self.fit_intercept = fit_intercept
        self.verbose = verbose
        self.normalize = normalize
        self.precompute = precompute
        self.n_nonzero_coefs = n_nonzero_coefs
        self.eps = eps
        self.copy_X = copy_X
        self.fit_path = fit_path
        self.jitter = jitter
        self.random_state = random_state

    def _fit(self, X, y, max_iter, alpha, fit_path, Xy=None):
        n_features = X.shape[1]
        X, y, X_offset, y_offset, X_scale = _preprocess_data(
            X, y, self.fit_intercept, _norm_flag(self.normalize, True), True)
        if y.ndim == 1:
            y = y[:, np.newaxis]
        n_targets = y.shape[1]
        G = X.T @ X
        self.alphas_, self.n_iter_, self.active_, self.coef_path_ = [], [], [], []
        self.coef_ = np.empty((n_targets, n_features))
        for k in range(n_targets):
            xy = X.T @ y[:, k] if Xy is None else Xy[:, k]
            a, act, path, it = _lars_gram(G, xy, X.shape[0], max_iter, alpha, self.method,
                                          self.eps, self.positive, True)
            self.alphas_.append(a if fit_path else a[-1:])
            self.active_.append(act)
            self.n_iter_.append(it)
            self.coef_path_.append(path)
            self.coef_[k] = path[:, -1]
        if n_targets == 1:
            self.alphas_, self.active_, self.coef_path_, self.coef_ = [
                v[0] for v in (self.alphas_, self.active_, self.coef_path_, self.coef_)]
            self.n_iter_ = self.n_iter_[0]
        if not fit_path:
            del self.coef_path_
        self._set_intercept(X_offset, y_offset, X_scale)
        return self

    def fit(self, X, y, Xy=None):
        X = _as_dense64(X).astype(np.float64)
        y = np.asarray(y, dtype=np.float64)
        self.n_features_in_ = X.shape[1]
        alpha = getattr(self, "alpha", 0.0)
        if hasattr(self, "n_nonzero_coefs"):
            alpha = 0.0
            max_iter = self.n_nonzero_coefs
        else:
            max_iter = self.max_iter
        if self.jitter is not None:
            rng = check_random_state(self.random_state)
            y = y + rng.uniform(high=self.jitter, size=len(y))
        return self._fit(X, y, max_iter, alpha, self.fit_path, Xy)


class LassoLars(Lars):

    def _more_tags(self):
        return {"poor_score": True}

    method = "lasso"

    def __init__(self, alpha=1.0, *, fit_intercept=True, verbose=False, normalize="deprecated",
                 precompute="auto", max_iter=500, eps=_EPS64, copy_X=True, fit_path=True,
                 positive=False, jitter=None, random_state=None):
        self.alpha = alpha
        self.fit_intercept = fit_intercept
        self.max_iter = max_iter
        self.verbose = verbose
        self.normalize = normalize
        self.positive = positive
        self.precompute = precompute
        self.copy_X = copy_X
        self.eps = eps
        self.fit_path = fit_path
        self.jitter = jitter
        self.random_state = random_state


def _lars_residues(Xtr, ytr, Xte, yte, method, fit_intercept, normalize, max_iter, eps,
                   positive):
    Xtr, Xte = Xtr.copy(), Xte.copy()
    ytr, yte = ytr.astype(np.float64).copy(), yte.astype(np.float64).copy()
    if fit_intercept:
        xm = Xtr.mean(axis=0)
        Xtr -= xm
        Xte -= xm
        ym = ytr.mean(axis=0)
        ytr -= ym
        yte -= ym
    if normalize:
        norms = np.sqrt(np.sum(Xtr ** 2, axis=0))
        nz = np.flatnonzero(norms)
        Xtr[:, nz] /= norms[nz]
    a, act, coefs, _ = _lars_gram(Xtr.T @ Xtr, Xtr.T @ ytr, ytr.size, max_iter, 0, method, eps,
                                  positive, True)
    if normalize:
        coefs[nz] /= norms[nz][:, np.newaxis]
    return a, act, coefs, (Xte @ coefs - yte[:, np.newaxis]).T


class LarsCV(Lars):
    method = "lar"

    def __init__(self, *, fit_intercept=True, verbose=False, max_iter=500,
                 normalize="deprecated", precompute="auto", cv=None, max_n_alphas=1000,
                 n_jobs=None, eps=_EPS64, copy_X=True):
        self.max_iter = max_iter
        self.cv = cv
        self.max_n_alphas = max_n_alphas
        self.n_jobs = n_jobs
        self.fit_intercept = fit_intercept
        self.verbose = verbose
        self.normalize = normalize
        self.precompute = precompute
        self.eps = eps
        self.copy_X = copy_X
        self.fit_path = True

    def fit(self, X, y):
        from ...model_selection import check_cv
        X = _as_dense64(X).astype(np.float64)
        y = np.asarray(y, dtype=np.float64)
        self.n_features_in_ = X.shape[1]
        cv = check_cv(self.cv, classifier=False)
        norm = _norm_flag(self.normalize, True)
        paths = [_lars_residues(X[tr], y[tr], X[te], y[te], self.method, self.fit_intercept,
                                norm, self.max_iter, self.eps, getattr(self, "positive", False))
                 for tr, te in cv.split(X, y)]
        all_alphas = np.unique(np.concatenate([p[0] for p in paths]))
        stride = int(max(1, int(len(all_alphas) / float(self.max_n_alphas))))
        all_alphas = all_alphas[::stride]
        mse = np.empty((len(all_alphas), len(paths)))
        for i, (a, _, _, res) in enumerate(paths):
            a, res = a[::-1], res[::-1]
            if a[0] != 0:
                a = np.r_[0, a]
                res = np.r_[res[0, np.newaxis], res]
            if a[-1] != all_alphas[-1]:
                a = np.r_[a, all_alphas[-1]]
                res = np.r_[res, res[-1, np.newaxis]]
            r = interpolate.interp1d(a, res, axis=0)(all_alphas) ** 2
            mse[:, i] = np.mean(r, axis=-1)
        ok = np.all(np.isfinite(mse), axis=-1)
        all_alphas, mse = all_alphas[ok], mse[ok]
        best = all_alphas[np.argmin(mse.mean(axis=-1))]
        self.alpha_ = best
        self.cv_alphas_ = all_alphas
        self.mse_path_ = mse
        self._fit(X, y, self.max_iter, best, True)
        return self


class LassoLarsCV(LarsCV):
    method = "lasso"

    def __init__(self, *, fit_intercept=True, verbose=False, max_iter=500,
                 normalize="deprecated", precompute="auto", cv=None, max_n_alphas=1000,
                 n_jobs=None, eps=_EPS64, copy_X=True, positive=False):
        super().__init__(fit_intercept=fit_intercept, verbose=verbose, max_iter=max_iter,
                         normalize=normalize, precompute=precompute, cv=cv,
                         max_n_alphas=max_n_alphas, n_jobs=n_jobs, eps=eps, copy_X=copy_X)
        self.positive = positive


class LassoLarsIC(LassoLars):
    """Lasso-LARS with the alpha picked by AIC / BIC."""

    def __init__(self, criterion="aic", *, fit_intercept=True, verbose=False,
                 normalize="deprecated", precompute="auto", max_iter=500, eps=_EPS64,
                 copy_X=True, positive=False):
        self.criterion = criterion
        self.fit_intercept = fit_intercept
        self.positive = positive
        self.max_iter = max_iter
        self.verbose = verbose
        self.normalize = normalize
        self.copy_X = copy_X
        self.precompute = precompute
        self.eps = eps
        self.fit_path = True

    def fit(self, X, y, copy_X=None):
        X = _as_dense64(X).astype(np.float64)
        y = np.asarray(y, dtype=np.float64)
        self.n_features_in_ = X.shape[1]
        X, y, xm, ym, xs = _preprocess_data(X, y, self.fit_intercept,
                                            _norm_flag(self.normalize, True), True)
        a, act, path, self.n_iter_ = _lars_gram(X.T @ X, X.T @ y, y.size, self.max_iter, 0.0,
                                                "lasso", self.eps, self.positive, True)
        n = X.shape[0]
        if self.criterion == "aic":
            K = 2
        elif self.criterion == "bic":
            K = log(n)
        else:
            raise ValueError("criterion should be either bic or aic")
        mse = np.mean((y[:, np.newaxis] - X @ path) ** 2, axis=0)
        sigma2 = np.var(y)
        df = np.array([np.sum(np.abs(c) > np.finfo(c.dtype).eps) for c in path.T])
        self.alphas_ = a
        self.criterion_ = n * mse / (sigma2 + _EPS64) + K * df
        best = int(np.argmin(self.criterion_))
        self.alpha_ = a[best]
        self.coef_ = path[:, best]
        self._set_intercept(xm, ym, xs)
        return self


# ====================================================================== OMP
def _omp_gram(G, Xy, n_nonzero, tol, norm_sq, return_path):
    p = G.shape[0]
    min_float = np.finfo(np.float64).eps
    active = []
    gamma = np.zeros(0)
    r = Xy.copy()
    L = np.zeros((p, p))
    tol_curr = norm_sq if tol is not None else None
    delta = 0.0
    max_features = p if tol is not None else n_nonzero
    coefs = []
    while True:
        lam = int(np.argmax(np.abs(r)))
        if lam in active or r[lam] ** 2 < min_float:
            warnings.warn("Orthogonal matching pursuit ended prematurely due to linear "
                          "dependence in the dictionary. The requested precision might not have "
                          "been reached.", RuntimeWarning, stacklevel=3)
            break
        k = len(active)
        if k:
            g = linalg.solve_triangular(L[:k, :k], G[lam, active], lower=True)
            Lkk = G[lam, lam] - g @ g
            if Lkk <= min_float:
                warnings.warn("Orthogonal matching pursuit ended prematurely due to linear "
                              "dependence in the dictionary.", RuntimeWarning, stacklevel=3)
                break
            L[k, :k] = g
            L[k, k] = np.sqrt(Lkk)
        else:
            L[0, 0] = np.sqrt(G[lam, lam])
        active.append(lam)
        k += 1
        gamma = linalg.cho_solve((L[:k, :k], True), Xy[active])
        beta = G[:, active] @ gamma
        r = Xy - beta
        if return_path:
            c = np.zeros(p)
            c[active] = gamma
            coefs.append(c)
        if tol is not None:
            tol_curr += delta
            delta = gamma @ beta[active]
            tol_curr -= delta
            if abs(tol_curr) <= tol:
                break
        elif k == max_features:
            break
    return gamma, active, len(active), (np.array(coefs).T if return_path else None)


def orthogonal_mp_gram(Gram, Xy, *, n_nonzero_coefs=None, tol=None, norms_squared=None,
                       copy_Gram=True, copy_Xy=True, return_path=False, return_n_iter=False):
    Gram = np.asarray(Gram, dtype=np.float64)
    Xy = np.asarray(Xy, dtype=np.float64)
    one = Xy.ndim == 1
    if one:
        Xy = Xy[:, np.newaxis]
        if tol is not None:
            norms_squared = [norms_squared]
    if n_nonzero_coefs is None and tol is None:
        n_nonzero_coefs = int(0.1 * len(Gram))
    if tol is not None and norms_squared is None:
        raise ValueError("Gram OMP needs the precomputed norms in order to evaluate the error "
                         "sum of squares.")
    if tol is not None and tol < 0:
        raise ValueError("Epsilon cannot be negative")
    if tol is None and n_nonzero_coefs <= 0:
        raise ValueError("The number of atoms must be positive")
    if tol is None and n_nonzero_coefs > len(Gram):
        raise ValueError("The number of atoms cannot be more than the number of features")
    p, T = Gram.shape[0], Xy.shape[1]
    coef = np.zeros((p, T, n_nonzero_coefs)) if return_path else np.zeros((p, T))
    n_iters = []
    for k in range(T):
        g, act, it, path = _omp_gram(Gram, Xy[:, k], n_nonzero_coefs,
                                     None if tol is None else tol,
                                     None if tol is None else norms_squared[k], return_path)
        if return_path:
            coef[:, k, :path.shape[1]] = path
        else:
            coef[act, k] = g
        n_iters.append(it)
    if T == 1:
        n_iters = n_iters[0]
    out = np.squeeze(coef)
    return (out, n_iters) if return_n_iter else out


def orthogonal_mp(X, y, *, n_nonzero_coefs=None, tol=None, precompute=False, copy_X=True,
                  return_path=False, return_n_iter=False):
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    if y.ndim == 1:
        y = y[:, np.newaxis]
    if tol is None and n_nonzero_coefs is None:
        n_nonzero_coefs = max(int(0.1 * X.shape[1]), 1)
    if tol is None and n_nonzero_coefs > X.shape[1]:
        raise ValueError("The number of atoms cannot be more than the number of features")
    norms = np.sum(y ** 2, axis=0) if tol is not None else None
    return orthogonal_mp_gram(X.T @ X, X.T @ y, n_nonzero_coefs=n_nonzero_coefs, tol=tol,
                              norms_squared=norms, return_path=return_path,
                              return_n_iter=return_n_iter)


class OrthogonalMatchingPursuit(MultiOutputMixin, RegressorMixin, LinearModel):

    def _more_tags(self):
        return {"poor_score": True}

    def __init__(self, *, n_nonzero_coefs=None, tol=None, fit_intercept=True,
                 normalize="deprecated", precompute="auto"):
        self.n_nonzero_coefs = n_nonzero_coefs
        self.tol = tol
        self.fit_intercept = fit_intercept
        self.normalize = normalize
        self.precompute = precompute

    def fit(self, X, y):
        X = _as_dense64(X).astype(np.float64)
        y = np.asarray(y, dtype=np.float64)
        self.n_features_in_ = X.shape[1]
        X, y, xo, yo, xs = _preprocess_data(X, y, self.fit_intercept,
                                            _norm_flag(self.normalize, True), True)
        if y.ndim == 1:
            y = y[:, np.newaxis]
        if self.n_nonzero_coefs is None and self.tol is None:
            self.n_nonzero_coefs_ = max(int(0.1 * X.shape[1]), 1)
        else:
            self.n_nonzero_coefs_ = self.n_nonzero_coefs
        norms = np.sum(y ** 2, axis=0) if self.tol is not None else None
        coef, self.n_iter_ = orthogonal_mp_gram(X.T @ X, X.T @ y,
                                                n_nonzero_coefs=self.n_nonzero_coefs_,
                                                tol=self.tol, norms_squared=norms,
                                                return_n_iter=True)
        self.coef_ = coef.T
        self._set_intercept(xo, yo, xs)
        return self


class OrthogonalMatchingPursuitCV(RegressorMixin, LinearModel):
    def __init__(self, *, copy=True, fit_intercept=True, normalize="deprecated", max_iter=None,
                 cv=None, n_jobs=None, verbose=False):
        self.copy = copy
        self.fit_intercept = fit_intercept
        self.normalize = normalize
        self.max_iter = max_iter
        self.cv = cv
        self.n_jobs = n_jobs
        self.verbose = verbose

    def fit(self, X, y):
        from ...model_selection import check_cv
        X = _as_dense64(X).astype(np.float64)
        y = np.asarray(y, dtype=np.float64)
        self.n_features_in_ = X.shape[1]
        norm = _norm_flag(self.normalize, True)
        cv = check_cv(self.cv, classifier=False)
        max_iter = min(max(int(0.1 * X.shape[1]), 5), X.shape[1]) if not self.max_iter \
            else self.max_iter
        folds = []
        for tr, te in cv.split(X):
            Xtr, Xte, ytr, yte = X[tr].copy(), X[te].copy(), y[tr].copy(), y[te].copy()
            if self.fit_intercept:
                xm = Xtr.mean(axis=0)
                Xtr -= xm
                Xte -= xm
                ym = ytr.mean(axis=0)
                ytr -= ym
                yte -= ym
            if norm:
                nr = np.sqrt(np.sum(Xtr ** 2, axis=0))
                nz = np.flatnonzero(nr)
                Xtr[:, nz] /= nr[nz]
            c = orthogonal_mp(Xtr, ytr, n_nonzero_coefs=max_iter, return_path=True)
            if c.ndim == 1:
                c = c[:, np.newaxis]
            if norm:
                c[nz] /= nr[nz][:, np.newaxis]
            folds.append(c.T @ Xte.T - yte)
        m = min(f.shape[0] for f in folds)
        mse = np.array([(f[:m] ** 2).mean(axis=1) for f in folds])
        best = int(np.argmin(mse.mean(axis=0)) + 1)
        self.n_nonzero_coefs_ = best
        omp = OrthogonalMatchingPursuit(n_nonzero_coefs=best, fit_intercept=self.fit_intercept,
                                        normalize=self.normalize).fit(X, y)
        self.coef_, self.intercept_, self.n_iter_ = omp.coef_, omp.intercept_, omp.n_iter_
        return self


# ==================================================================== Huber
def _huber_loss_grad(w, X, y, epsilon, alpha, sw):
    d = X.shape[1]
    fit_int = w.shape[0] == d + 2
    sigma = w[-1]
    coef = w[:d]
    r = y - X @ coef - (w[-2] if fit_int else 0.0)
    ar = np.abs(r)
    out = ar > epsilon * sigma
    sw_out = sw[out]
    n_out_w = sw_out.sum()
    out_loss = 2.0 * epsilon * np.sum(sw_out * ar[out]) - sigma * n_out_w * epsilon ** 2
    inl = ~out
    wr = sw[inl] * r[inl]
    sq = (wr @ r[inl]) / sigma
    grad = np.zeros(w.shape[0])
    grad[:d] = -2.0 / sigma * (wr @ X[inl])
    sgn = np.where(r[out] < 0, -1.0, 1.0) * sw_out
    grad[:d] -= 2.0 * epsilon * (sgn @ X[out])
    grad[:d] += 2.0 * alpha * coef
    grad[-1] = sw.sum() - n_out_w * epsilon ** 2 - sq / sigma
    if fit_int:
        grad[-2] = -2.0 * np.sum(wr) / sigma - 2.0 * epsilon * np.sum(sgn)
    loss = sw.sum() * sigma + sq + out_loss + alpha * (coef @ coef)
    return loss, grad


class HuberRegressor(RegressorMixin, LinearModel):
    """Linear regression with the Huber loss and a jointly fitted scale."""

    def __init__(self, *, epsilon=1.35, max_iter=100, alpha=0.0001, warm_start=False,
                 fit_intercept=True, tol=1e-05):
        self.epsilon = epsilon
        self.max_iter = max_iter
        self.alpha = alpha
        self.warm_start = warm_start
        self.fit_intercept = fit_intercept
        self.tol = tol

    def fit(self, X, y, sample_weight=None):
        X = _as_dense64(X).astype(np.float64)
        y = np.asarray(y, dtype=np.float64)
        self.n_features_in_ = X.shape[1]
        sw = _check_sample_weight(sample_weight, X.shape[0])
        sw = np.ones(X.shape[0]) if sw is None else sw
        if self.epsilon < 1.0:
            raise ValueError("epsilon should be greater than or equal to 1.0, got %f"
                             % self.epsilon)
        d = X.shape[1]
        if self.warm_start and hasattr(self, "coef_"):
            w0 = np.concatenate((self.coef_, [self.intercept_, self.scale_]) if self.fit_intercept
                                else (self.coef_, [self.scale_]))
        else:
            w0 = np.zeros(d + (2 if self.fit_intercept else 1))
            w0[-1] = 1.0
        bounds = np.tile([-np.inf, np.inf], (w0.shape[0], 1))
        bounds[-1][0] = _EPS64 * 10
        res = optimize.minimize(_huber_loss_grad, w0, method="L-BFGS-B", jac=True,
                                args=(X, y, self.epsilon, self.alpha, sw),
                                options={"maxiter": self.max_iter, "gtol": self.tol,
                                         "iprint": -1}, bounds=bounds)
        if res.status == 2:
            raise ValueError("HuberRegressor convergence failed: l-BFGS-b solver terminated "
                             "with %s" % res.message)
        w = res.x
        self.n_iter_ = min(res.nit, self.max_iter)
        self.scale_ = w[-1]
        self.intercept_ = w[-2] if self.fit_intercept else 0.0
        self.coef_ = w[:d]
        self.outliers_ = np.abs(y - X @ self.coef_ - self.intercept_) > self.scale_ * self.epsilon
        return self


# =================================================================== RANSAC
_SPACING1 = np.spacing(1)


def _dynamic_max_trials(n_inliers, n_samples, min_samples, probability):
    ratio = n_inliers / float(n_samples)
    nom = max(_SPACING1, 1 - probability)
    den = max(_SPACING1, 1 - ratio ** min_samples)
    if nom == 1:
        return 0
    if den == 1:
        return float("inf")
    return abs(float(np.ceil(np.log(nom) / np.log(den))))


class RANSACRegressor(MetaEstimatorMixin, RegressorMixin, MultiOutputMixin, BaseEstimator):
    """Random sample consensus around any regressor."""

    def __init__(self, base_estimator=None, *, min_samples=None, residual_threshold=None,
                 is_data_valid=None, is_model_valid=None, max_trials=100, max_skips=np.inf,
                 stop_n_inliers=np.inf, stop_score=np.inf, stop_probability=0.99,
                 loss="absolute_error", random_state=None):
        self.base_estimator = base_estimator
        self.min_samples = min_samples
        self.residual_threshold = residual_threshold
        self.is_data_valid = is_data_valid
        self.is_model_valid = is_model_valid
        self.max_trials = max_trials
        self.max_skips = max_skips
        self.stop_n_inliers = stop_n_inliers
        self.stop_score = stop_score
        self.stop_probability = stop_probability
        self.random_state = random_state
        self.loss = loss

    def fit(self, X, y, sample_weight=None):
        from ._base import LinearRegression
        X = _as_dense64(X).astype(np.float64)
        y = np.asarray(y, dtype=np.float64)
        self.n_features_in_ = X.shape[1]
        est = clone(self.base_estimator) if self.base_estimator is not None \
            else LinearRegression()
        if self.min_samples is None:
            min_samples = X.shape[1] + 1
        elif 0 < self.min_samples < 1:
            min_samples = np.ceil(self.min_samples * X.shape[0])
        elif self.min_samples >= 1:
            min_samples = self.min_samples
        else:
            raise ValueError("Value for `min_samples` must be scalar and positive.")
        if min_samples > X.shape[0]:
            raise ValueError("`min_samples` may not be larger than number of samples: "
                             "n_samples = %d." % X.shape[0])
        if not 0 <= self.stop_probability <= 1:
            raise ValueError("`stop_probability` must be in range [0, 1].")
        thr = np.median(np.abs(y - np.median(y))) if self.residual_threshold is None \
            else self.residual_threshold
        if self.loss in ("absolute_error", "absolute_loss"):
            lossf = (lambda a, b: np.abs(a - b)) if y.ndim == 1 else \
                (lambda a, b: np.sum(np.abs(a - b), axis=1))
        elif self.loss in ("squared_error", "squared_loss"):
            lossf = (lambda a, b: (a - b) ** 2) if y.ndim == 1 else \
                (lambda a, b: np.sum((a - b) ** 2, axis=1))
        elif callable(self.loss):
            lossf = self.loss
        else:
            raise ValueError("loss should be 'absolute_error', 'squared_error' or a callable. "
                             "Got %s. " % self.loss)
        rs = check_random_state(self.random_state)
        n = X.shape[0]
        idx_all = np.arange(n)
        best_n, best_score = 1, -np.inf
        best_mask = best_X = best_y = best_idx = None
        self.n_skips_no_inliers_ = self.n_skips_invalid_data_ = self.n_skips_invalid_model_ = 0
        self.n_trials_ = 0
        max_trials = self.max_trials
        while self.n_trials_ < max_trials:
            self.n_trials_ += 1
            if (self.n_skips_no_inliers_ + self.n_skips_invalid_data_
                    + self.n_skips_invalid_model_) > self.max_skips:
                break
            sub = sample_without_replacement(n, int(min_samples), random_state=rs)
            Xs, ys = X[sub], y[sub]
            if self.is_data_valid is not None and not self.is_data_valid(Xs, ys):
                self.n_skips_invalid_data_ += 1
                continue
            if sample_weight is None:
                est.fit(Xs, ys)
            else:
                est.fit(Xs, ys, sample_weight=np.asarray(sample_weight)[sub])
            if self.is_model_valid is not None and not self.is_model_valid(est, Xs, ys):
                self.n_skips_invalid_model_ += 1
                continue
            mask = lossf(y, np.asarray(est.predict(X))) < thr
            n_in = int(np.sum(mask))
            if n_in < best_n:
                self.n_skips_no_inliers_ += 1
                continue
            ii = idx_all[mask]
            score = est.score(X[ii], y[ii])
            if n_in == best_n and score < best_score:
                continue
            best_n, best_score, best_mask = n_in, score, mask
            best_X, best_y, best_idx = X[ii], y[ii], ii
            max_trials = min(max_trials, _dynamic_max_trials(best_n, n, min_samples,
                                                             self.stop_probability))
            if best_n >= self.stop_n_inliers or best_score >= self.stop_score:
                break
        if best_mask is None:
            raise ValueError("RANSAC could not find a valid consensus set. All `max_trials` "
                             "iterations were skipped because each randomly chosen sub-sample "
                             "failed the passing criteria. See estimator attributes for "
                             "diagnostics (n_skips*).")
        if sample_weight is None:
            est.fit(best_X, best_y)
        else:
            est.fit(best_X, best_y, sample_weight=np.asarray(sample_weight)[best_idx])
        self.estimator_ = est
        self.inlier_mask_ = best_mask
        return self

    def predict(self, X):
        check_is_fitted(self, "estimator_")
        return self.estimator_.predict(X)

    def score(self, X, y):
        check_is_fitted(self, "estimator_")
        return self.estimator_.score(X, y)


# ================================================================ TheilSen
def _modified_weiszfeld_step(X, x_old):
    diff = X - x_old
    dn = np.sqrt(np.sum(diff ** 2, axis=1))
    mask = dn >= _SPACING1
    in_x = int(mask.sum() < X.shape[0])
    diff = diff[mask]
    dn = dn[mask][:, np.newaxis]
    qn = linalg.norm(np.sum(diff / dn, axis=0))
    if qn > _SPACING1:
        nd = np.sum(X[mask, :] / dn, axis=0) / np.sum(1 / dn, axis=0)
    else:
        nd, qn = 1.0, 1.0
    return max(0.0, 1.0 - in_x / qn) * nd + min(1.0, in_x / qn) * x_old


def _spatial_median(X, max_iter=300, tol=1.0e-3):
    if X.shape[1] == 1:
        return 1, np.median(X.ravel(), keepdims=True)
    tol **= 2
    old = np.mean(X, axis=0)
    for n_iter in range(max_iter):
        new = _modified_weiszfeld_step(X, old)
        if np.sum((old - new) ** 2) < tol:
            break
        old = new
    else:
        warnings.warn("Maximum number of iterations {max_iter} reached in spatial median for "
                      "TheilSen regressor.".format(max_iter=max_iter), ConvergenceWarning)
    return n_iter, new


def _breakdown_point(n_samples, n_subsamples):
    return 1 - (0.5 ** (1 / n_subsamples) * (n_samples - n_subsamples + 1) + n_subsamples - 1) \
        / n_samples


class TheilSenRegressor(RegressorMixin, LinearModel):
    """Spatial median of least-squares fits on many sample subsets; the
    subset fits are one batched pseudo-inverse on the device."""

    def __init__(self, *, fit_intercept=True, copy_X=True, max_subpopulation=1e4,
                 n_subsamples=None, max_iter=300, tol=1.0e-3, random_state=None, n_jobs=None,
                 verbose=False):
        self.fit_intercept = fit_intercept
        self.copy_X = copy_X
        self.max_subpopulation = int(max_subpopulation)
        self.n_subsamples = n_subsamples
        self.max_iter = max_iter
        self.tol = tol
        self.random_state = random_state
        self.n_jobs = n_jobs
        self.verbose = verbose

    def fit(self, X, y):
        rs = check_random_state(self.random_state)
        X = _as_dense64(X).astype(np.float64)
        y = np.asarray(y, dtype=np.float64)
        n, d = X.shape
        self.n_features_in_ = d
        n_dim = d + 1 if self.fit_intercept else d
        ns = self.n_subsamples
        if ns is not None:
            if ns > n:
                raise ValueError("Invalid parameter since n_subsamples > n_samples ({0} > {1})."
                                 .format(ns, n))
            if n >= d and n_dim > ns:
                raise ValueError("Invalid parameter since n_features{0} > n_subsamples ({1} > "
                                 "{2}).".format(" + 1" if self.fit_intercept else "", n_dim, ns))
        else:
            ns = min(n_dim, n)
        if self.max_subpopulation <= 0:
            raise ValueError("Subpopulation must be strictly positive ({0} <= 0)."
                             .format(self.max_subpopulation))
        allc = max(1, np.rint(binom(n, ns)))
        self.n_subpopulation_ = int(min(self.max_subpopulation, allc))
        self.breakdown_ = _breakdown_point(n, ns)
        if np.rint(binom(n, ns)) <= self.max_subpopulation:
            idx = np.array(list(combinations(range(n), ns)))
        else:
            idx = np.array([rs.choice(n, size=ns, replace=False)
                            for _ in range(self.n_subpopulation_)])
        fi = int(self.fit_intercept)
        dev = resolve_device(None)
        Xt = torch.as_tensor(X, device=dev)
        yt = torch.as_tensor(y, device=dev)
        it = torch.as_tensor(idx, device=dev)
        A = torch.ones((idx.shape[0], ns, d + fi), dtype=torch.float64, device=dev)
        A[:, :, fi:] = Xt[it]
        W = (torch.linalg.pinv(A) @ yt[it].unsqueeze(-1)).squeeze(-1).cpu().numpy()
        self.n_iter_, coefs = _spatial_median(W, max_iter=self.max_iter, tol=self.tol)
        if self.fit_intercept:
            self.intercept_, self.coef_ = coefs[0], coefs[1:]
        else:
            self.intercept_, self.coef_ = 0.0, coefs
        return self


# ===================================================================== GLMs
def _tweedie_unit_deviance(y, mu, p):
    if p == 0:
        return (y - mu) ** 2
    if p == 1:
        return 2 * (xlogy(y, y / mu) - y + mu)
    if p == 2:
        return 2 * (np.log(mu / y) + y / mu - 1)
    return 2 * (np.power(np.maximum(y, 0), 2 - p) / ((1 - p) * (2 - p))
                - y * np.power(mu, 1 - p) / (1 - p) + np.power(mu, 2 - p) / (2 - p))


class TweedieRegressor(RegressorMixin, BaseEstimator):
    """Generalised linear model with a Tweedie distribution (power p) and
    identity / log link, fitted by L-BFGS on 0.5 * mean deviance + L2."""

    def _more_tags(self):
        return {"requires_positive_y": True}


    def __init__(self, *, power=0.0, alpha=1.0, fit_intercept=True, link="auto", max_iter=100,
                 tol=1e-4, warm_start=False, verbose=0):
        self.power = power
        self.alpha = alpha
        self.fit_intercept = fit_intercept
        self.link = link
        self.max_iter = max_iter
        self.tol = tol
        self.warm_start = warm_start
        self.verbose = verbose

    def _link(self):
        link = self.link
        if link == "auto":
            link = "identity" if self.power <= 0 else "log"
        if link not in ("identity", "log"):
            raise ValueError("The link must be an element of ['auto', 'identity', 'log']; got "
                             "(link={0})".format(link))
        return link

    def _check_y(self, y):
        p = self.power
        if 0 < p < 1:
            raise ValueError("Tweedie distribution is only defined for power<=0 and power>=1.")
        if p >= 2 and np.any(y <= 0):
            raise ValueError("Some value(s) of y are out of the valid range for family "
                             "TweedieDistribution")
        if 1 <= p < 2 and np.any(y < 0):
            raise ValueError("Some value(s) of y are out of the valid range for family "
                             "TweedieDistribution")

    def fit(self, X, y, sample_weight=None):
        X = _as_dense64(X).astype(np.float64)
        y = np.asarray(y, dtype=np.float64)
        if not isinstance(self.alpha, (int, float)) or self.alpha < 0:
            raise ValueError("Penalty term must be a non-negative number; got (alpha={0})"
                             .format(self.alpha))
        self._check_y(y)
        self.n_features_in_ = X.shape[1]
        n, d = X.shape
        sw = _check_sample_weight(sample_weight, n)
        sw = np.ones(n) if sw is None else sw
        w = sw / sw.sum()
        link = self._link()
        p = self.power
        inv = (lambda z: z) if link == "identity" else np.exp
        dinv = (lambda z: np.ones_like(z)) if link == "identity" else np.exp
        off = 1 if self.fit_intercept else 0

        def fun(c):
            eta = X @ c[off:] + (c[0] if off else 0.0)
            mu = inv(eta)
            dev = np.sum(w * _tweedie_unit_deviance(y, mu, p))
            t = dinv(eta) * (w * -2 * (y - mu) / np.power(mu, p) if p != 0 else w * -2 * (y - mu))
            g = np.concatenate(([t.sum()], t @ X)) if off else t @ X
            cs = c[off:]
            return 0.5 * dev + 0.5 * self.alpha * (cs @ cs), 0.5 * g + np.r_[
                np.zeros(off), self.alpha * cs]

        if self.warm_start and hasattr(self, "coef_"):
            c0 = np.concatenate(([self.intercept_], self.coef_)) if off else self.coef_.copy()
        else:
            c0 = np.zeros(d + off)
            if off:
                m = np.average(y, weights=w)
                c0[0] = m if link == "identity" else np.log(m)
        res = optimize.minimize(fun, c0, method="L-BFGS-B", jac=True,
                                options={"maxiter": self.max_iter, "iprint": -1, "gtol": self.tol,
                                         "ftol": 1e3 * _EPS64})
        if res.status != 0:
            warnings.warn("lbfgs failed to converge (status=%d): %s" % (res.status, res.message),
                          ConvergenceWarning)
        self.n_iter_ = min(res.nit, self.max_iter)
        c = res.x
        self.intercept_ = c[0] if off else 0.0
        self.coef_ = c[off:]
        return self

    def _linear_predictor(self, X):
        check_is_fitted(self, "coef_")
        return _as_dense64(X) @ self.coef_ + self.intercept_

    def predict(self, X):
        eta = self._linear_predictor(X)
        return eta if self._link() == "identity" else np.exp(eta)

    def score(self, X, y, sample_weight=None):
        y = np.asarray(y, dtype=np.float64)
        sw = _check_sample_weight(sample_weight, len(y))
        sw = np.ones(len(y)) if sw is None else sw
        mu = self.predict(X)
        dev = np.sum(sw * _tweedie_unit_deviance(y, mu, self.power))
        dev0 = np.sum(sw * _tweedie_unit_deviance(y, np.average(y, weights=sw), self.power))
        return 1 - dev / dev0

    @property
    def family(self):
        return "tweedie"


class PoissonRegressor(TweedieRegressor):

    def _more_tags(self):
        return {"requires_positive_y": True}

    def __init__(self, *, alpha=1.0, fit_intercept=True, max_iter=100, tol=1e-4,
                 warm_start=False, verbose=0):
        super().__init__(power=1.0, alpha=alpha, fit_intercept=fit_intercept, link="log",
                         max_iter=max_iter, tol=tol, warm_start=warm_start, verbose=verbose)

    def get_params(self, deep=True):
        return {k: getattr(self, k) for k in ("alpha", "fit_intercept", "max_iter", "tol",
                                               "warm_start", "verbose")}


class GammaRegressor(TweedieRegressor):

    def _more_tags(self):
        return {"requires_positive_y": True}

    def __init__(self, *, alpha=1.0, fit_intercept=True, max_iter=100, tol=1e-4,
                 warm_start=False, verbose=0):
        super().__init__(power=2.0, alpha=alpha, fit_intercept=fit_intercept, link="log",
                         max_iter=max_iter, tol=tol, warm_start=warm_start, verbose=verbose)

    def get_params(self, deep=True):
        return {k: getattr(self, k) for k in ("alpha", "fit_intercept", "max_iter", "tol",
                                               "warm_start", "verbose")}


class GeneralizedLinearRegressor(TweedieRegressor):
    """Generalised linear model of a named exponential-dispersion family
    (reference ``linear_model/_glm/glm.py:GeneralizedLinearRegressor``,
    the base of the Poisson / Gamma / Tweedie regressors): 'normal',
    'poisson', 'gamma' and 'inverse-gaussian' are the Tweedie powers 0, 1,
    2, 3; same L-BFGS solver as TweedieRegressor."""

    _FAMILY_POWER = {"normal": 0.0, "poisson": 1.0, "gamma": 2.0, "inverse-gaussian": 3.0}

    def __init__(self, *, alpha=1.0, fit_intercept=True, family="normal", link="auto",
                 solver="lbfgs", max_iter=100, tol=1e-4, warm_start=False, verbose=0):
        self.family = family
        self.solver = solver
        super().__init__(power=0.0, alpha=alpha, fit_intercept=fit_intercept, link=link,
                         max_iter=max_iter, tol=tol, warm_start=warm_start, verbose=verbose)

    # the family is a constructor parameter here (not TweedieRegressor's
    # read-only property)
    family = None

    def get_params(self, deep=True):
        return {k: getattr(self, k) for k in ("alpha", "fit_intercept", "family", "link",
                                               "solver", "max_iter", "tol", "warm_start",
                                               "verbose")}

    def fit(self, X, y, sample_weight=None):
        from ..._loss.glm_distribution import TweedieDistribution
        if isinstance(self.family, TweedieDistribution):
            if self.solver != "lbfgs":
                raise ValueError("GeneralizedLinearRegressor supports only solvers 'lbfgs'; "
                                 "got {0}".format(self.solver))
            self.power = self.family.power
            return super().fit(X, y, sample_weight=sample_weight)
        if self.family not in self._FAMILY_POWER:
            raise ValueError("The family must be an instance of class ExponentialDispersionModel "
                             "or an element of ['normal', 'poisson', 'gamma', "
                             "'inverse-gaussian']; got (family={0})".format(self.family))
        if self.solver != "lbfgs":
            raise ValueError("GeneralizedLinearRegressor supports only solvers 'lbfgs'; got "
                             "{0}".format(self.solver))
        self.power = self._FAMILY_POWER[self.family]
        return super().fit(X, y, sample_weight=sample_weight)


# ================================================================= Quantile
class QuantileRegressor(RegressorMixin, LinearModel):
    """L1-penalised quantile regression as a linear program (HiGHS)."""

    def _more_tags(self):
        return {"poor_score": True}


    def __init__(self, *, quantile=0.5, alpha=1.0, fit_intercept=True, solver="highs",
                 solver_options=None):
        self.quantile = quantile
        self.alpha = alpha
        self.fit_intercept = fit_intercept
        self.solver = solver
        self.solver_options = solver_options

    def fit(self, X, y, sample_weight=None):
        X = _as_dense64(X).astype(np.float64)
        y = np.asarray(y, dtype=np.float64)
        n, d = X.shape
        self.n_features_in_ = d
        if not 0 < self.quantile < 1:
            raise ValueError("Quantile should be strictly between 0.0 and 1.0, got %r"
                             % self.quantile)
        if self.alpha < 0:
            raise ValueError("Penalty alpha must be a non-negative number, got %r" % self.alpha)
        sw = _check_sample_weight(sample_weight, n)
        sw = np.ones(n) if sw is None else sw
        npar = d + int(self.fit_intercept)
        a = np.sum(sw) * self.alpha
        c = np.concatenate([np.full(2 * npar, a), sw * self.quantile, sw * (1 - self.quantile)])
        if self.fit_intercept:
            c[0] = 0
            c[npar] = 0
        Xa = np.hstack([np.ones((n, 1)), X]) if self.fit_intercept else X
        eye = sp.eye(n, format="csr")
        A = sp.hstack([sp.csr_matrix(Xa), sp.csr_matrix(-Xa), eye, -eye], format="csr")
        method = "highs" if self.solver in ("interior-point", "revised simplex") else self.solver
        res = optimize.linprog(c=c, A_eq=A, b_eq=y, method=method, options=self.solver_options)
        if res.status != 0:
            warnings.warn("Linear programming for QuantileRegressor did not succeed.\nStatus is "
                          "%d: %s" % (res.status, res.message), ConvergenceWarning)
        sol = res.x
        params = sol[:npar] - sol[npar:2 * npar]
        self.n_iter_ = getattr(res, "nit", 0)
        if self.fit_intercept:
            self.coef_, self.intercept_ = params[1:], params[0]
        else:
            self.coef_, self.intercept_ = params, 0.0
        return self


# =============================================================== multitask
def _rand_r(state):
    s = state[0] or 1
    s ^= (s << 13) & 0xFFFFFFFF
    s ^= s >> 17
    s ^= (s << 5) & 0xFFFFFFFF
    state[0] = s & 0xFFFFFFFF
    return state[0] % 0x80000000


def _mt_cd(W, l1, l2, X, Y, max_iter, tol, rs, random):
    """Multi-task (block soft-threshold) coordinate descent; W is (T, p)."""
    n, p = X.shape
    norm_cols = (X ** 2).sum(axis=0)
    R = Y - X @ W.T
    d_w_tol = tol
    tol = tol * np.sum(Y * Y)
    seed = [int(rs.randint(0, 2 ** 31 - 1))]
    gap = tol + 1.0
    n_iter = 0
    for n_iter in range(max_iter):
        w_max = d_w_max = 0.0
        for f in range(p):
            ii = _rand_r(seed) % p if random else f
            if norm_cols[ii] == 0.0:
                continue
            w_old = W[:, ii].copy()
            if np.any(w_old != 0):
                R += np.outer(X[:, ii], w_old)
            tmp = X[:, ii] @ R
            nn = np.sqrt(tmp @ tmp)
            W[:, ii] = tmp * max(1.0 - l1 / nn, 0.0) / (norm_cols[ii] + l2) if nn > 0 else 0.0
            if np.any(W[:, ii] != 0):
                R -= np.outer(X[:, ii], W[:, ii])
            d_w_max = max(d_w_max, np.abs(W[:, ii] - w_old).max())
            w_max = max(w_max, np.abs(W[:, ii]).max())
        if w_max == 0.0 or d_w_max / w_max < d_w_tol or n_iter == max_iter - 1:
            XtA = X.T @ R - l2 * W.T
            dual = np.sqrt((XtA ** 2).sum(axis=1)).max()
            Rn = np.sqrt(np.sum(R * R))
            wn = np.sqrt(np.sum(W * W))
            if dual > l1:
                const = l1 / dual
                gap = 0.5 * (Rn ** 2 + (Rn * const) ** 2)
            else:
                const = 1.0
                gap = Rn ** 2
            gap += l1 * np.sqrt((W ** 2).sum(axis=0)).sum() - const * np.sum(R * Y) \
                + 0.5 * l2 * (1 + const ** 2) * wn ** 2
            if gap < tol:
                break
    else:
        warnings.warn("Objective did not converge. You might want to increase the number of "
                      "iterations. Duality gap: {}, tolerance: {}".format(gap, tol),
                      ConvergenceWarning)
    return W, gap, tol, n_iter + 1


class MultiTaskElasticNet(RegressorMixin, LinearModel):
    """Elastic net with a shared (L2,1) sparsity pattern across targets."""

    def _more_tags(self):
        return {"multioutput_only": True}


    def __init__(self, alpha=1.0, *, l1_ratio=0.5, fit_intercept=True, normalize=False,
                 copy_X=True, max_iter=1000, tol=1e-4, warm_start=False, random_state=None,
                 selection="cyclic"):
        self.l1_ratio = l1_ratio
        self.alpha = alpha
        self.fit_intercept = fit_intercept
        self.normalize = normalize
        self.max_iter = max_iter
        self.copy_X = copy_X
        self.tol = tol
        self.warm_start = warm_start
        self.random_state = random_state
        self.selection = selection

    def fit(self, X, y):
        X = _as_dense64(X).astype(np.float64)
        y = np.asarray(y, dtype=np.float64)
        if y.ndim == 1:
            raise ValueError("For mono-task outputs, use %s" % type(self).__name__[9:])
        n, d = X.shape
        self.n_features_in_ = d
        X, y, xo, yo, xs = _preprocess_data(X, y, self.fit_intercept, _norm_flag(self.normalize,
                                                                                  False), True)
        if self.selection not in ("random", "cyclic"):
            raise ValueError("selection should be either random or cyclic.")
        if not self.warm_start or getattr(self, "coef_", None) is None:
            self.coef_ = np.zeros((y.shape[1], d))
        l1 = self.alpha * self.l1_ratio * n
        l2 = self.alpha * (1.0 - self.l1_ratio) * n
        self.coef_, self.dual_gap_, self.eps_, self.n_iter_ = _mt_cd(
            np.array(self.coef_, dtype=np.float64), l1, l2, X, y, self.max_iter, self.tol,
            check_random_state(self.random_state), self.selection == "random")
        self.dual_gap_ /= n
        self._set_intercept(xo, yo, xs)
        return self


class MultiTaskLasso(MultiTaskElasticNet):

    def _more_tags(self):
        return {"multioutput_only": True}

    def __init__(self, alpha=1.0, *, fit_intercept=True, normalize=False, copy_X=True,
                 max_iter=1000, tol=1e-4, warm_start=False, random_state=None,
                 selection="cyclic"):
        super().__init__(alpha=alpha, l1_ratio=1.0, fit_intercept=fit_intercept,
                         normalize=normalize, copy_X=copy_X, max_iter=max_iter, tol=tol,
                         warm_start=warm_start, random_state=random_state, selection=selection)

    def get_params(self, deep=True):
        p = super().get_params(deep)
        p.pop("l1_ratio", None)
        return p


class _MultiTaskCV(RegressorMixin, LinearModel):
    def _path_fit(self, X, y):
        from ...model_selection import check_cv
        from ._coordinate_descent import _alpha_grid
        X = _as_dense64(X).astype(np.float64)
        y = np.asarray(y, dtype=np.float64)
        self.n_features_in_ = X.shape[1]
        l1s = np.atleast_1d(getattr(self, "l1_ratio", 1.0))
        cv = check_cv(self.cv, classifier=False)
        folds = list(cv.split(X, y))
        best = (np.inf, None, None)
        mse_all, alphas_all = [], []
        for l1r in l1s:
            alphas = self.alphas if self.alphas is not None else _alpha_grid(
                X, y, l1_ratio=l1r, fit_intercept=self.fit_intercept, eps=self.eps,
                n_alphas=self.n_alphas, normalize=_norm_flag(self.normalize, False))
            alphas = np.sort(np.asarray(alphas))[::-1]
            mse = np.zeros((len(alphas), len(folds)))
            for fi, (tr, te) in enumerate(folds):
                m = MultiTaskElasticNet(l1_ratio=l1r, fit_intercept=self.fit_intercept,
                                        normalize=self.normalize, max_iter=self.max_iter,
                                        tol=self.tol, warm_start=True,
                                        random_state=self.random_state, selection=self.selection)
                for ai, a in enumerate(alphas):
                    m.set_params(alpha=a)
                    with warnings.catch_warnings():
                        warnings.simplefilter("ignore", ConvergenceWarning)
                        m.fit(X[tr], y[tr])
                    mse[ai, fi] = np.mean((m.predict(X[te]) - y[te]) ** 2)
            mse_all.append(mse)
            alphas_all.append(alphas)
            i = int(np.argmin(mse.mean(axis=1)))
            if mse[i].mean() < best[0]:
                best = (mse[i].mean(), alphas[i], l1r)
        self.alpha_, self.l1_ratio_ = best[1], best[2]
        self.mse_path_ = np.squeeze(np.array(mse_all))
        self.alphas_ = np.squeeze(np.array(alphas_all))
        m = MultiTaskElasticNet(alpha=self.alpha_, l1_ratio=self.l1_ratio_,
                                fit_intercept=self.fit_intercept, normalize=self.normalize,
                                max_iter=self.max_iter, tol=self.tol,
                                random_state=self.random_state, selection=self.selection).fit(X, y)
        self.coef_, self.intercept_ = m.coef_, m.intercept_
        self.dual_gap_, self.n_iter_ = m.dual_gap_, m.n_iter_
        return self


class MultiTaskElasticNetCV(_MultiTaskCV):

    def _more_tags(self):
        return {"multioutput_only": True}

    def __init__(self, *, l1_ratio=0.5, eps=1e-3, n_alphas=100, alphas=None, fit_intercept=True,
                 normalize=False, max_iter=1000, tol=1e-4, cv=None, copy_X=True, verbose=0,
                 n_jobs=None, random_state=None, selection="cyclic"):
        self.l1_ratio = l1_ratio
        self.eps = eps
        self.n_alphas = n_alphas
        self.alphas = alphas
        self.fit_intercept = fit_intercept
        self.normalize = normalize
        self.max_iter = max_iter
        self.tol = tol
        self.cv = cv
        self.copy_X = copy_X
        self.verbose = verbose
        self.n_jobs = n_jobs
        self.random_state = random_state
        self.selection = selection

    def fit(self, X, y):
        return self._path_fit(X, y)


class MultiTaskLassoCV(_MultiTaskCV):

    def _more_tags(self):
        return {"multioutput_only": True}

    def __init__(self, *, eps=1e-3, n_alphas=100, alphas=None, fit_intercept=True,
                 normalize=False, max_iter=1000, tol=1e-4, copy_X=True, cv=None, verbose=False,
                 n_jobs=None, random_state=None, selection="cyclic"):
        self.eps = eps
        self.n_alphas = n_alphas
        self.alphas = alphas
        self.fit_intercept = fit_intercept
        self.normalize = normalize
        self.max_iter = max_iter
        self.tol = tol
        self.copy_X = copy_X
        self.cv = cv
        self.verbose = verbose
        self.n_jobs = n_jobs
        self.random_state = random_state
        self.selection = selection

    def fit(self, X, y):
        return self._path_fit(X, y)


# ====================================================== LogisticRegressionCV
class LogisticRegressionCV(LinearClassifierMixin, BaseEstimator):
    """Logistic regression with C (and l1_ratio) chosen by cross-validation."""

    def __init__(self, *, Cs=10, fit_intercept=True, cv=None, dual=False, penalty="l2",
                 scoring=None, solver="lbfgs", tol=1e-4, max_iter=100, class_weight=None,
                 n_jobs=None, verbose=0, refit=True, intercept_scaling=1.0, multi_class="auto",
                 random_state=None, l1_ratios=None):
        self.Cs = Cs
        self.fit_intercept = fit_intercept
        self.cv = cv
        self.dual = dual
        self.penalty = penalty
        self.scoring = scoring
        self.tol = tol
        self.max_iter = max_iter
        self.class_weight = class_weight
        self.n_jobs = n_jobs
        self.verbose = verbose
        self.solver = solver
        self.refit = refit
        self.intercept_scaling = intercept_scaling
        self.multi_class = multi_class
        self.random_state = random_state
        self.l1_ratios = l1_ratios

    def _base(self, C, l1r):
        from ._logistic import LogisticRegression
        kw = dict(penalty=self.penalty, C=C, fit_intercept=self.fit_intercept, tol=self.tol,
                  max_iter=self.max_iter, class_weight=self.class_weight, solver=self.solver,
                  multi_class=self.multi_class, random_state=self.random_state,
                  intercept_scaling=self.intercept_scaling)
        if self.penalty == "elasticnet":
            kw["l1_ratio"] = l1r
        return LogisticRegression(**kw)

    def fit(self, X, y, sample_weight=None):
        from ...model_selection import check_cv
        from ...model_selection._validation import get_scorer
        X = _as_dense64(X).astype(np.float64)
        y = np.asarray(y)
        self.n_features_in_ = X.shape[1]
        self.classes_ = np.unique(y)
        Cs = np.logspace(-4, 4, self.Cs) if np.isscalar(self.Cs) else np.asarray(self.Cs)
        self.Cs_ = Cs
        l1rs = [None] if self.penalty != "elasticnet" else list(self.l1_ratios)
        cv = check_cv(self.cv, y, classifier=True)
        folds = list(cv.split(X, y))
        scorer = get_scorer(self.scoring)
        scores = np.zeros((len(folds), len(Cs), len(l1rs)))
        for fi, (tr, te) in enumerate(folds):
            for ci, C in enumerate(Cs):
                for li, l1r in enumerate(l1rs):
                    with warnings.catch_warnings():
                        warnings.simplefilter("ignore", ConvergenceWarning)
                        m = self._base(C, l1r)
                        if sample_weight is None:
                            m.fit(X[tr], y[tr])
                        else:
                            m.fit(X[tr], y[tr], sample_weight=np.asarray(sample_weight)[tr])
                    scores[fi, ci, li] = scorer(m, X[te], y[te])
        mean = scores.mean(axis=0)
        ci, li = np.unravel_index(np.argmax(mean), mean.shape)
        best_C, best_l1 = Cs[ci], l1rs[li]
        n_cls = 1 if len(self.classes_) == 2 else len(self.classes_)
        key = self.classes_[1:] if n_cls == 1 else self.classes_
        sc = scores if self.penalty == "elasticnet" else scores[..., 0]
        self.scores_ = {c: sc for c in key}
        self.C_ = np.full(n_cls, best_C)
        self.l1_ratio_ = np.full(n_cls, best_l1 if best_l1 is not None else None, dtype=object) \
            if self.penalty == "elasticnet" else np.full(n_cls, None)
        if self.refit:
            m = self._base(best_C, best_l1)
            m.fit(X, y) if sample_weight is None else m.fit(X, y, sample_weight=sample_weight)
        else:
            m = self._base(best_C, best_l1).fit(X, y)
        self.coef_, self.intercept_ = m.coef_, m.intercept_
        self.n_iter_ = np.atleast_1d(getattr(m, "n_iter_", 0))
        self._best = m
        return self

    def predict_proba(self, X):
        check_is_fitted(self, "coef_")
        return self._best.predict_proba(X)

    def predict_log_proba(self, X):
        return np.log(self.predict_proba(X))

    def score(self, X, y, sample_weight=None):
        from ...model_selection._validation import get_scorer
        s = get_scorer(self.scoring)
        return s(self, X, y) if sample_weight is None else \
            s(self, X, y, sample_weight=sample_weight)


__all__ = ["lars_path", "lars_path_gram", "Lars", "LassoLars", "LarsCV", "LassoLarsCV",
           "LassoLarsIC", "orthogonal_mp", "orthogonal_mp_gram", "OrthogonalMatchingPursuit",
           "OrthogonalMatchingPursuitCV", "HuberRegressor", "RANSACRegressor",
           "TheilSenRegressor", "TweedieRegressor", "PoissonRegressor", "GammaRegressor",
           "QuantileRegressor", "MultiTaskElasticNet", "MultiTaskLasso", "MultiTaskElasticNetCV",
           "MultiTaskLassoCV", "LogisticRegressionCV"]
