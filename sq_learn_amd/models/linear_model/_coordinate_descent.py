"""Elastic-net / Lasso by coordinate descent (reference
``linear_model/_coordinate_descent.py`` over ``_cd_fast.pyx``).

The per-coordinate loop is the host-native ``sqh_enet_cd_dense`` /
``sqh_enet_cd_gram`` (``csrc/host/cd_host.cpp``, the reference's update,
stopping rule and xorshift coordinate stream); with ``precompute`` the Gram
matrix X^T X and X^T y are formed on the resolved device (fp64 GEMMs) and
only the d x d problem goes to the host loop.  Paths warm-start along a
decreasing alpha grid; the CV estimators score each fold's path by mean
squared error."""

import warnings

import numpy as np
import torch

from ...base import RegressorMixin
from ...exceptions import ConvergenceWarning
from ...ops import _host
from ...runtime.device import resolve_device
from ...utils.validation import check_random_state
from ._base import (LinearModel, _as_dense64, _check_sample_weight, _device_tensor,
                    _preprocess_data, _rescale_data)

_RAND_R_MAX = 0x7FFFFFFF


def _gram(X, y, device):
    Xt = _device_tensor(X, device)
    G = (Xt.T @ Xt).cpu().numpy()
    Xy = (Xt.T @ _device_tensor(y, device)).cpu().numpy()
    return np.ascontiguousarray(G), Xy


def _alpha_grid(X, y, Xy=None, l1_ratio=1.0, fit_intercept=True, eps=1e-3, n_alphas=100,
                normalize=False, copy_X=True):
    if l1_ratio == 0:
        raise ValueError("Automatic alpha grid generation is not supported for l1_ratio=0. "
                         "Please supply a grid by providing your estimator with the appropriate "
                         "`alphas=` argument.")
    n_samples = len(y)
    if Xy is None:
        Xc, yc, _, _, _ = _preprocess_data(X, y, fit_intercept, normalize, copy=copy_X)
        Xy = Xc.T @ yc
    if Xy.ndim == 1:
        Xy = Xy[:, None]
    alpha_max = np.sqrt(np.sum(Xy ** 2, axis=1)).max() / (n_samples * l1_ratio)
    if alpha_max <= np.finfo(float).resolution:
        return np.full(n_alphas, np.finfo(float).resolution)
    return np.logspace(np.log10(alpha_max * eps), np.log10(alpha_max), num=n_alphas)[::-1]


def _cd(w, l1, l2, X_f, y, Gram, Xy, y_norm2, max_iter, tol, seed, random, positive):
    out = np.zeros(4)
    L = _host.lib()
    if Gram is not None:
        L.sqh_enet_cd_gram(_host.ptr(w), l1, l2, _host.ptr(Gram), _host.ptr(Xy), y_norm2,
                           Gram.shape[0], int(max_iter), float(tol), seed, int(random),
                           int(positive), _host.ptr(out))
    else:
        L.sqh_enet_cd_dense(_host.ptr(w), l1, l2, _host.ptr(X_f), _host.ptr(y), y.shape[0],
                            w.shape[0], int(max_iter), float(tol), seed, int(random),
                            int(positive), _host.ptr(out))
    return out


def enet_path(X, y, *, l1_ratio=0.5, eps=1e-3, n_alphas=100, alphas=None, precompute="auto",
              Xy=None, copy_X=True, coef_init=None, verbose=False, return_n_iter=False,
              positive=False, check_input=True, device=None, **params):
    """(alphas, coefs, dual_gaps[, n_iters]) along a warm-started alpha path.

    X, y are used as given (no centring: the estimators centre first)."""
    X = _as_dense64(X)
    y = np.asarray(y, dtype=np.float64)
    n_samples, n_features = X.shape
    multi = y.ndim == 2
    if multi:
        return _enet_path_multi_output(X, y, l1_ratio=l1_ratio, eps=eps, n_alphas=n_alphas,
                                       alphas=alphas, Xy=Xy, coef_init=coef_init,
                                       return_n_iter=return_n_iter, positive=positive, **params)
    y = y.ravel()
    tol = params.get("tol", 1e-4)
    max_iter = params.get("max_iter", 1000)
    rng = check_random_state(params.get("random_state", None))
    selection = params.get("selection", "cyclic")
    if selection not in ("random", "cyclic"):
        raise ValueError("selection should be either random or cyclic.")
    random = selection == "random"
    if isinstance(precompute, str) and precompute == "auto":
        precompute = n_samples > n_features
    Gram = None
    if isinstance(precompute, np.ndarray):
        Gram = np.ascontiguousarray(precompute, dtype=np.float64)
        Xy = X.T @ y if Xy is None else np.asarray(Xy, dtype=np.float64).ravel()
    elif precompute is True:
        Gram, Xy = _gram(X, y, resolve_device(device))
    if alphas is None:
        alphas = _alpha_grid(X, y, Xy=Xy, l1_ratio=l1_ratio, fit_intercept=False, eps=eps,
                             n_alphas=n_alphas)
    else:
        alphas = np.sort(np.asarray(alphas, dtype=np.float64))[::-1]
    n_alphas = len(alphas)
    coefs = np.empty((n_features, n_alphas), dtype=np.float64)
    dual_gaps = np.empty(n_alphas)
    n_iters = []
    w = np.zeros(n_features) if coef_init is None else np.array(coef_init, dtype=np.float64)
    X_f = np.asfortranarray(X) if Gram is None else None
    X_cm = np.ascontiguousarray(X_f.T) if Gram is None else None     # columns contiguous
    y_norm2 = float(y @ y)
    Xy_c = None if Gram is None else np.ascontiguousarray(Xy, dtype=np.float64).ravel()
    for i, alpha in enumerate(alphas):
        l1 = float(alpha * l1_ratio * n_samples)
        l2 = float(alpha * (1.0 - l1_ratio) * n_samples)
        seed = int(rng.randint(0, _RAND_R_MAX))
        if l1 == 0 and l2 == 0:
            warnings.warn("Coordinate descent with no regularization may lead to unexpected "
                          "results and is discouraged.")
        out = _cd(w, l1, l2, X_cm, np.ascontiguousarray(y), Gram, Xy_c, y_norm2, max_iter, tol,
                  seed, random, positive)
        gap, tol_s, n_it, conv = out
        if not conv:
            warnings.warn("Objective did not converge. You might want to increase the number of "
                          "iterations. Duality gap: {:.3e}, tolerance: {:.3e}".format(gap, tol_s),
                          ConvergenceWarning)
        coefs[:, i] = w
        dual_gaps[i] = gap
        n_iters.append(int(n_it))
    if return_n_iter:
        return alphas, coefs, dual_gaps, n_iters
    return alphas, coefs, dual_gaps


def _enet_path_multi_output(X, y, *, l1_ratio, eps, n_alphas, alphas, Xy, coef_init,
                            return_n_iter, positive, **params):
    """Multi-output path (reference ``linear_model/_coordinate_descent.py:
    452-498``): the multi-task (L2,1) coordinate descent of
    MultiTaskElasticNet warm-started along the alphas; coefs [n_targets,
    n_features, n_alphas], dual gaps rescaled by 1 / n_samples."""
    from ._lm_extra import _mt_cd
    if positive:
        raise ValueError("positive=True is not allowed for multi-output (y.ndim != 1)")
    n_samples, n_features = X.shape
    n_outputs = y.shape[1]
    tol = params.get("tol", 1e-4)
    max_iter = params.get("max_iter", 1000)
    rng = check_random_state(params.get("random_state", None))
    selection = params.get("selection", "cyclic")
    if selection not in ("random", "cyclic"):
        raise ValueError("selection should be either random or cyclic.")
    if alphas is None:
        alphas = _alpha_grid(X, y, Xy=Xy, l1_ratio=l1_ratio, fit_intercept=False, eps=eps,
                             n_alphas=n_alphas)
    else:
        alphas = np.sort(np.asarray(alphas, dtype=np.float64))[::-1]
    coefs = np.empty((n_outputs, n_features, len(alphas)), dtype=np.float64)
    dual_gaps = np.empty(len(alphas))
    n_iters = []
    W = (np.zeros((n_outputs, n_features)) if coef_init is None
         else np.array(coef_init, dtype=np.float64).reshape(n_outputs, n_features))
    for i, alpha in enumerate(alphas):
        l1 = float(alpha * l1_ratio * n_samples)
        l2 = float(alpha * (1.0 - l1_ratio) * n_samples)
        W, gap, _, n_it = _mt_cd(W, l1, l2, X, y, max_iter, tol, rng, selection == "random")
        coefs[..., i] = W
        dual_gaps[i] = gap / n_samples
        n_iters.append(int(n_it))
    if return_n_iter:
        return alphas, coefs, dual_gaps, n_iters
    return alphas, coefs, dual_gaps


def lasso_path(X, y, *, eps=1e-3, n_alphas=100, alphas=None, precompute="auto", Xy=None,
               copy_X=True, coef_init=None, verbose=False, return_n_iter=False, positive=False,
               **params):
    return enet_path(X, y, l1_ratio=1.0, eps=eps, n_alphas=n_alphas, alphas=alphas,
                     precompute=precompute, Xy=Xy, copy_X=copy_X, coef_init=coef_init,
                     verbose=verbose, positive=positive, return_n_iter=return_n_iter, **params)


class ElasticNet(RegressorMixin, LinearModel):
    """Linear regression with combined l1 / l2 priors."""

    path = staticmethod(enet_path)

    def __init__(self, alpha=1.0, *, l1_ratio=0.5, fit_intercept=True, normalize=False,
                 precompute=False, max_iter=1000, copy_X=True, tol=1e-4, warm_start=False,
                 positive=False, random_state=None, selection="cyclic", device=None):
        self.alpha = alpha
        self.l1_ratio = l1_ratio
        self.fit_intercept = fit_intercept
        self.normalize = normalize
        self.precompute = precompute
        self.max_iter = max_iter
        self.copy_X = copy_X
        self.tol = tol
        self.warm_start = warm_start
        self.positive = positive
        self.random_state = random_state
        self.selection = selection
        self.device = device

    def fit(self, X, y, sample_weight=None, check_input=True):
        if self.alpha == 0:
            warnings.warn("With alpha=0, this algorithm does not converge well. You are advised "
                          "to use the LinearRegression estimator", stacklevel=2)
        if self.selection not in ("cyclic", "random"):
            raise ValueError("selection should be either random or cyclic.")
        X = _as_dense64(X)
        y = np.asarray(y, dtype=X.dtype)
        n_samples, n_features = X.shape
        self.n_features_in_ = n_features
        sw = _check_sample_weight(sample_weight, n_samples, X.dtype)
        if sw is not None:
            sw = sw * (n_samples / np.sum(sw))
        X, y, X_offset, y_offset, X_scale = _preprocess_data(
            X, y, self.fit_intercept, self.normalize, copy=True, sample_weight=sw)
        if sw is not None:
            X, y = _rescale_data(X, y, sw)
        precompute = self.precompute
        if isinstance(precompute, str) and precompute == "auto":
            precompute = n_samples > n_features
        if precompute is True:
            Gram = _gram(X, np.zeros(n_samples), resolve_device(self.device))[0]
        elif isinstance(precompute, np.ndarray):
            Gram = precompute
        else:
            Gram = False
        Y = y[:, None] if y.ndim == 1 else y
        n_targets = Y.shape[1]
        if not self.warm_start or not hasattr(self, "coef_"):
            coef_ = np.zeros((n_targets, n_features), dtype=np.float64)
        else:
            coef_ = np.atleast_2d(self.coef_).astype(np.float64)
        gaps = np.zeros(n_targets)
        self.n_iter_ = []
        rs = self.random_state
        for k in range(n_targets):
            _, c, g, it = enet_path(X, Y[:, k], l1_ratio=self.l1_ratio, alphas=[self.alpha],
                                    precompute=Gram, coef_init=coef_[k], return_n_iter=True,
                                    positive=self.positive, tol=self.tol, max_iter=self.max_iter,
                                    random_state=rs, selection=self.selection,
                                    device=self.device)
            coef_[k] = c[:, 0]
            gaps[k] = g[0]
            self.n_iter_.append(it[0])
        if n_targets == 1:
            self.n_iter_ = self.n_iter_[0]
            self.coef_ = coef_[0]
            self.dual_gap_ = gaps[0]
        else:
            self.coef_ = coef_
            self.dual_gap_ = gaps
        self._set_intercept(X_offset, y_offset, X_scale)
        return self

    @property
    def sparse_coef_(self):
        import scipy.sparse as sp
        return sp.csr_matrix(self.coef_)


class Lasso(ElasticNet):
    """Linear model trained with an l1 prior (ElasticNet with l1_ratio=1)."""

    path = staticmethod(enet_path)

    def __init__(self, alpha=1.0, *, fit_intercept=True, normalize=False, precompute=False,
                 copy_X=True, max_iter=1000, tol=1e-4, warm_start=False, positive=False,
                 random_state=None, selection="cyclic", device=None):
        super().__init__(alpha=alpha, l1_ratio=1.0, fit_intercept=fit_intercept,
                         normalize=normalize, precompute=precompute, copy_X=copy_X,
                         max_iter=max_iter, tol=tol, warm_start=warm_start, positive=positive,
                         random_state=random_state, selection=selection, device=device)


class _LinearModelCV(RegressorMixin, LinearModel):
    def _cv_fit(self, X, y, l1_ratios):
        from ...model_selection import KFold
        X = _as_dense64(X)
        y = np.asarray(y, dtype=np.float64).ravel()
        self.n_features_in_ = X.shape[1]
        cv = self.cv if self.cv is not None else 5
        splitter = KFold(cv) if isinstance(cv, int) else cv
        folds = list(splitter.split(X, y))
        Xc, yc, _, _, _ = _preprocess_data(X, y, self.fit_intercept, self.normalize, copy=True)
        alphas_all = []
        for r in l1_ratios:
            if self.alphas is None:
                alphas_all.append(_alpha_grid(Xc, yc, l1_ratio=r, fit_intercept=False,
                                              eps=self.eps, n_alphas=self.n_alphas))
            else:
                alphas_all.append(np.sort(np.asarray(self.alphas, dtype=np.float64))[::-1])
        mse = np.zeros((len(l1_ratios), len(alphas_all[0]), len(folds)))
        for li, r in enumerate(l1_ratios):
            for fi, (tr, te) in enumerate(folds):
                Xt, yt, xo, yo, xs = _preprocess_data(X[tr], y[tr], self.fit_intercept,
                                                      self.normalize, copy=True)
                _, coefs, _ = enet_path(Xt, yt, l1_ratio=r, alphas=alphas_all[li],
                                        precompute=self.precompute, tol=self.tol,
                                        max_iter=self.max_iter, positive=self.positive,
                                        random_state=self.random_state,
                                        selection=self.selection, device=self.device)
                coefs = coefs / xs[:, None]
                icpt = yo - xo @ coefs
                pred = X[te] @ coefs + icpt
                mse[li, :, fi] = ((pred - y[te][:, None]) ** 2).mean(0)
        mean = mse.mean(2)
        li, ai = np.unravel_index(np.argmin(mean), mean.shape)
        self.l1_ratio_ = l1_ratios[li]
        self.alpha_ = float(alphas_all[li][ai])
        self.alphas_ = alphas_all[li] if len(l1_ratios) == 1 else np.asarray(alphas_all)
        self.mse_path_ = mse[0] if len(l1_ratios) == 1 else mse
        model = ElasticNet(alpha=self.alpha_, l1_ratio=self.l1_ratio_,
                           fit_intercept=self.fit_intercept, normalize=self.normalize,
                           precompute=self.precompute, max_iter=self.max_iter, tol=self.tol,
                           positive=self.positive, random_state=self.random_state,
                           selection=self.selection, device=self.device).fit(X, y)
        self.coef_, self.intercept_ = model.coef_, model.intercept_
        self.dual_gap_, self.n_iter_ = model.dual_gap_, model.n_iter_
        return self


class LassoCV(_LinearModelCV):
    def __init__(self, *, eps=1e-3, n_alphas=100, alphas=None, fit_intercept=True,
                 normalize=False, precompute="auto", max_iter=1000, tol=1e-4, copy_X=True,
                 cv=None, verbose=False, n_jobs=None, positive=False, random_state=None,
                 selection="cyclic", device=None):
        self.eps, self.n_alphas, self.alphas = eps, n_alphas, alphas
        self.fit_intercept, self.normalize, self.precompute = fit_intercept, normalize, precompute
        self.max_iter, self.tol, self.copy_X, self.cv = max_iter, tol, copy_X, cv
        self.verbose, self.n_jobs, self.positive = verbose, n_jobs, positive
        self.random_state, self.selection, self.device = random_state, selection, device

    def fit(self, X, y):
        return self._cv_fit(X, y, [1.0])


class ElasticNetCV(_LinearModelCV):
    def __init__(self, *, l1_ratio=0.5, eps=1e-3, n_alphas=100, alphas=None, fit_intercept=True,
                 normalize=False, precompute="auto", max_iter=1000, tol=1e-4, cv=None,
                 copy_X=True, verbose=0, n_jobs=None, positive=False, random_state=None,
                 selection="cyclic", device=None):
        self.l1_ratio = l1_ratio
        self.eps, self.n_alphas, self.alphas = eps, n_alphas, alphas
        self.fit_intercept, self.normalize, self.precompute = fit_intercept, normalize, precompute
        self.max_iter, self.tol, self.cv, self.copy_X = max_iter, tol, cv, copy_X
        self.verbose, self.n_jobs, self.positive = verbose, n_jobs, positive
        self.random_state, self.selection, self.device = random_state, selection, device

    def fit(self, X, y):
        return self._cv_fit(X, y, list(np.atleast_1d(self.l1_ratio)))
