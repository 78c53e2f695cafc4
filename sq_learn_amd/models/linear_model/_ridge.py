"""Ridge regression / classification (reference ``linear_model/_ridge.py``).

Dense solves on the resolved device in fp64: the primal normal equations
(X^T X + alpha I) w = X^T y when n_samples >= n_features, the dual (kernel)
form otherwise, and ``solver='svd'`` / ``RidgeCV`` from one thin SVD of
the centred design (every alpha re-uses it; leave-one-out errors come from
the closed-form hat-matrix diagonal with an unpenalised intercept).
``solver`` values of the reference ('auto', 'cholesky', 'svd', 'lsqr',
'sparse_cg', 'sag', 'saga') are accepted: 'sag' / 'saga' run the reference's
stochastic average gradient epochs (:mod:`._sag`, sample weights passed to
the solver, ``n_iter_`` per target); the other iterative ones solve the same
strongly convex problem exactly (normal equations)."""

import numpy as np
import torch

from ...base import ClassifierMixin, RegressorMixin
from ...utils.validation import check_is_fitted
from ._base import (LinearClassifierMixin, LinearModel, _as_dense64, _check_sample_weight,
                    _device_tensor, _preprocess_data, _rescale_data, label_binarize_pm1)

_SOLVERS = ("auto", "svd", "cholesky", "lsqr", "sparse_cg", "sag", "saga")


def _solve(X, y, alpha, solver, device):
    """coef (n_targets, n_features) for per-target alphas."""
    Xt, Y = _device_tensor(X, device), _device_tensor(y, device)
    if Y.ndim == 1:
        Y = Y[:, None]
    n, d = Xt.shape
    alphas = torch.as_tensor(np.broadcast_to(np.asarray(alpha, dtype=np.float64), (Y.shape[1],))
                             .copy(), device=device)
    if solver == "svd":
        U, S, Vh = torch.linalg.svd(Xt, full_matrices=False)
        UtY = U.T @ Y
        d_ = S[:, None] / (S[:, None] ** 2 + alphas[None, :])
        return (Vh.T @ (d_ * UtY)).T
    coefs = []
    if n >= d:
        A = Xt.T @ Xt
        B = Xt.T @ Y
        for t in range(Y.shape[1]):
            M = A + alphas[t] * torch.eye(d, dtype=A.dtype, device=device)
            coefs.append(torch.linalg.solve(M, B[:, t]))
    else:
        K = Xt @ Xt.T
        for t in range(Y.shape[1]):
            M = K + alphas[t] * torch.eye(n, dtype=K.dtype, device=device)
            coefs.append(Xt.T @ torch.linalg.solve(M, Y[:, t]))
    return torch.stack(coefs)


def _solve_sag(X, y, alpha, sw, solver, max_iter, tol, random_state, fit_intercept=False):
    """Per-target SAG / SAGA on the squared loss (reference ``_ridge.py:
    477-501``): (coef [n_targets, d], n_iter [n_targets], intercept)."""
    from ._sag import sag_solver
    Y = y[:, None] if y.ndim == 1 else y
    n, d = X.shape
    alphas = np.broadcast_to(np.asarray(alpha, dtype=np.float64).ravel(), (Y.shape[1],))
    max_sq = float(np.einsum("ij,ij->i", X, X).max()) if n else 0.0
    coef = np.empty((Y.shape[1], d))
    n_iter = np.empty(Y.shape[1], dtype=np.int32)
    intercept = np.zeros(Y.shape[1])
    for t in range(Y.shape[1]):
        init = {"coef": np.zeros((d + int(fit_intercept), 1))}
        c, it, _ = sag_solver(X, Y[:, t], sw, "squared", alphas[t], 0.0, max_iter, tol, 0,
                              random_state, False, max_sq, init, is_saga=solver == "saga")
        coef[t] = c[:d]
        if fit_intercept:
            intercept[t] = c[d]
        n_iter[t] = it
    return coef, n_iter, intercept


def ridge_regression(X, y, alpha, *, sample_weight=None, solver="auto", max_iter=None, tol=1e-3,
                     verbose=0, random_state=None, return_n_iter=False, return_intercept=False,
                     check_input=True, device=None):
    from ...runtime.device import resolve_device
    X = _as_dense64(X)
    y = np.asarray(y, dtype=np.float64)
    intercept = 0.0
    if solver in ("sag", "saga"):
        if return_intercept and solver != "sag":
            raise ValueError("In Ridge, only 'sag' solver can directly fit the intercept. Please "
                             "change solver to 'sag' or set return_intercept=False.")
        sw = _check_sample_weight(sample_weight, X.shape[0])
        coef, n_iter, icpt = _solve_sag(X, y, alpha, sw, solver, max_iter, tol, random_state,
                                        fit_intercept=return_intercept)
        if y.ndim == 1:
            coef, icpt = coef.ravel(), icpt[0]
        out = (coef,)
        if return_n_iter:
            out += (n_iter,)
        if return_intercept:
            out += (icpt,)
        return out[0] if len(out) == 1 else out
    if return_intercept:
        X, y, X_offset, y_offset, _ = _preprocess_data(X, y, True, sample_weight=sample_weight)
    sw = _check_sample_weight(sample_weight, X.shape[0])
    if sw is not None:
        X, y = _rescale_data(X, y, sw)
    coef = _solve(X, y, alpha, solver, resolve_device(device)).cpu().numpy()
    if y.ndim == 1:
        coef = coef.ravel()
    if return_intercept:
        intercept = y_offset - X_offset @ coef.T
    out = (coef,)
    if return_n_iter:
        out += (None,)
    if return_intercept:
        out += (intercept,)
    return out[0] if len(out) == 1 else out


class _BaseRidge(LinearModel):
    def __init__(self, alpha=1.0, *, fit_intercept=True, normalize=False, copy_X=True,
                 max_iter=None, tol=1e-3, solver="auto", random_state=None, device=None):
        self.alpha = alpha
        self.fit_intercept = fit_intercept
        self.normalize = normalize
        self.copy_X = copy_X
        self.max_iter = max_iter
        self.tol = tol
        self.solver = solver
        self.random_state = random_state
        self.device = device

    def fit(self, X, y, sample_weight=None):
        if self.solver not in _SOLVERS:
            raise ValueError("Known solvers are 'sparse_cg', 'cholesky', 'svd' 'lsqr', 'sag' or "
                             "'saga'. Got %s." % self.solver)
        if np.any(np.asarray(self.alpha) < 0):
            raise ValueError("alpha must be non-negative")
        X = _as_dense64(X)
        y = np.asarray(y, dtype=X.dtype)
        self.n_features_in_ = X.shape[1]
        sw = _check_sample_weight(sample_weight, X.shape[0], X.dtype)
        X, y, X_offset, y_offset, X_scale = _preprocess_data(
            X, y, self.fit_intercept, self.normalize, copy=self.copy_X, sample_weight=sw)
        if self.solver in ("sag", "saga"):
            # the solver takes the weights itself (reference _ridge.py:430-434)
            coef, n_iter, _ = _solve_sag(X, y, self.alpha, sw, self.solver, self.max_iter,
                                         self.tol, self.random_state)
            self.coef_ = coef.ravel() if y.ndim == 1 else coef
            self.n_iter_ = n_iter
            self._set_intercept(X_offset, y_offset, X_scale)
            return self
        if sw is not None:
            X, y = _rescale_data(X, y, sw)
        coef = _solve(X, y, self.alpha, "svd" if self.solver == "svd" else "cholesky",
                      self._device()).cpu().numpy()
        self.coef_ = coef.ravel() if y.ndim == 1 else coef
        self.n_iter_ = None
        self._set_intercept(X_offset, y_offset, X_scale)
        return self


class Ridge(RegressorMixin, _BaseRidge):
    """Linear least squares with l2 regularisation."""


class RidgeClassifier(LinearClassifierMixin, _BaseRidge):
    """Ridge regression on {-1, 1} targets (one column per class)."""

    def __init__(self, alpha=1.0, *, fit_intercept=True, normalize=False, copy_X=True,
                 max_iter=None, tol=1e-3, class_weight=None, solver="auto", random_state=None,
                 device=None):
        super().__init__(alpha=alpha, fit_intercept=fit_intercept, normalize=normalize,
                         copy_X=copy_X, max_iter=max_iter, tol=tol, solver=solver,
                         random_state=random_state, device=device)
        self.class_weight = class_weight

    def fit(self, X, y, sample_weight=None):
        y = np.asarray(y)
        self.classes_ = np.unique(y)
        Y = label_binarize_pm1(y, self.classes_)
        if self.class_weight is not None:
            cw = self.class_weight
            if cw == "balanced":
                counts = np.array([(y == c).sum() for c in self.classes_])
                cw = {c: len(y) / (len(self.classes_) * k) for c, k in zip(self.classes_, counts)}
            w = np.array([cw.get(c, 1.0) for c in y], dtype=np.float64)
            sample_weight = w if sample_weight is None else w * np.asarray(sample_weight)
        super().fit(X, Y, sample_weight=sample_weight)
        self.coef_ = np.atleast_2d(self.coef_)
        self.intercept_ = np.atleast_1d(self.intercept_)
        return self


class _RidgeGCV:
    """Efficient leave-one-out over an alpha grid from one SVD."""

    @staticmethod
    def loo(X, y, alphas, fit_intercept, device):
        Xt, Y = _device_tensor(X, device), _device_tensor(y, device)
        if Y.ndim == 1:
            Y = Y[:, None]
        n = Xt.shape[0]
        U, S, _ = torch.linalg.svd(Xt, full_matrices=False)
        UtY = U.T @ Y
        results = []
        for a in alphas:
            w = S ** 2 / (S ** 2 + a)                      # shrinkage of each direction
            Yhat = U @ (w[:, None] * UtY)
            h = (U ** 2) @ w                               # hat diagonal (centred part)
            if fit_intercept:
                h = h + 1.0 / n
            err = (Y - Yhat) / (1.0 - h)[:, None]
            results.append(err)
        return results


class RidgeCV(RegressorMixin, LinearModel):
    """Ridge with built-in efficient leave-one-out cross-validation (or a
    generic ``cv`` splitter) over ``alphas``."""

    def __init__(self, alphas=(0.1, 1.0, 10.0), *, fit_intercept=True, normalize=False,
                 scoring=None, cv=None, gcv_mode=None, store_cv_values=False,
                 alpha_per_target=False, device=None):
        self.alphas = alphas
        self.fit_intercept = fit_intercept
        self.normalize = normalize
        self.scoring = scoring
        self.cv = cv
        self.gcv_mode = gcv_mode
        self.store_cv_values = store_cv_values
        self.alpha_per_target = alpha_per_target
        self.device = device

    def fit(self, X, y, sample_weight=None):
        alphas = np.asarray(self.alphas, dtype=np.float64).ravel()
        if np.any(alphas <= 0):
            raise ValueError("alphas must be strictly positive. Got {} containing some negative "
                             "or null value instead.".format(self.alphas))
        X = _as_dense64(X)
        y = np.asarray(y, dtype=np.float64)
        self.n_features_in_ = X.shape[1]
        if self.cv is not None:
            from ...model_selection import GridSearchCV
            gs = GridSearchCV(Ridge(fit_intercept=self.fit_intercept, device=self.device),
                              {"alpha": list(alphas)}, cv=self.cv, scoring=self.scoring)
            gs.fit(X, y, sample_weight=sample_weight) if sample_weight is not None else gs.fit(X, y)
            est = gs.best_estimator_
            self.alpha_ = gs.best_params_["alpha"]
            self.best_score_ = gs.best_score_
            self.coef_, self.intercept_ = est.coef_, est.intercept_
            return self
        sw = _check_sample_weight(sample_weight, X.shape[0])
        Xc, yc, X_offset, y_offset, X_scale = _preprocess_data(
            X, y, self.fit_intercept, self.normalize, copy=True, sample_weight=sw)
        if sw is not None:
            Xc, yc = _rescale_data(Xc, yc, sw)
        errs = _RidgeGCV.loo(Xc, yc, alphas, self.fit_intercept and sw is None, self._device())
        if self.scoring is None:
            scores = [-(e ** 2).mean(0).cpu().numpy() for e in errs]     # per target
        else:
            # a user scorer on the leave-one-out predictions (reference
            # _ridge.py:1518-1535): predictions = y - LOO residual, scored
            # through an identity "estimator" whose predict returns its input,
            # per target when alpha_per_target, else on the raveled arrays
            from ...model_selection._validation import get_scorer
            scorer = get_scorer(self.scoring)
            Y = np.asarray(yc, dtype=np.float64).reshape(yc.shape[0], -1)
            preds = [Y - e.cpu().numpy().reshape(Y.shape) for e in errs]
            ident = _IdentityRegressor()
            if isinstance(self, LinearClassifierMixin):
                # RidgeClassifierCV: the class of the largest LOO score
                # against the true class (reference _ridge.py:1546-1551)
                ic = _IdentityClassifier(np.arange(Y.shape[1]))
                scores = [np.full(Y.shape[1], scorer(ic, P, Y.argmax(axis=1))) for P in preds]
            elif self.alpha_per_target and Y.shape[1] > 1:
                scores = [np.array([scorer(ident, P[:, j], Y[:, j]) for j in range(Y.shape[1])])
                          for P in preds]
            else:
                scores = [np.full(Y.shape[1], scorer(ident, P.ravel(), Y.ravel()))
                          for P in preds]
        scores = np.stack(scores)                                    # (n_alphas, n_targets)
        if self.alpha_per_target and scores.shape[1] > 1:
            best = scores.argmax(0)
            self.alpha_ = alphas[best]
            self.best_score_ = scores[best, np.arange(scores.shape[1])]
        else:
            tot = scores.mean(1)
            best = int(np.argmax(tot))
            self.alpha_ = float(alphas[best])
            self.best_score_ = float(tot[best])
        if self.store_cv_values:
            if self.scoring is None:
                cvv = np.stack([(e ** 2).cpu().numpy() for e in errs], axis=-1)
            else:   # the reference stores the LOO predictions with a scorer
                Y = np.asarray(yc, dtype=np.float64).reshape(yc.shape[0], -1)
                cvv = np.stack([Y - e.cpu().numpy().reshape(Y.shape) for e in errs], axis=-1)
            self.cv_values_ = cvv[:, 0, :] if y.ndim == 1 else cvv
        coef = _solve(Xc, yc, self.alpha_, "svd", self._device()).cpu().numpy()
        self.coef_ = coef.ravel() if y.ndim == 1 else coef
        self._set_intercept(X_offset, y_offset, X_scale)
        return self


class _IdentityRegressor:
    """Scorer adapter: ``predict`` / ``decision_function`` return their input
    (the LOO predictions themselves; reference ``_ridge.py:1433``)."""

    def decision_function(self, y_predict):
        return y_predict

    def predict(self, y_predict):
        return y_predict


class _IdentityClassifier(LinearClassifierMixin):
    """Scorer adapter of RidgeClassifierCV: ``decision_function`` returns its
    input, ``predict`` the class of its largest column."""

    def __init__(self, classes):
        self.classes_ = classes

    def decision_function(self, y_predict):
        return y_predict

    def predict(self, y_predict):
        return self.classes_[np.asarray(y_predict).argmax(axis=1)]


class RidgeClassifierCV(LinearClassifierMixin, RidgeCV):
    def __init__(self, alphas=(0.1, 1.0, 10.0), *, fit_intercept=True, normalize=False,
                 scoring=None, cv=None, class_weight=None, store_cv_values=False, device=None):
        super().__init__(alphas=alphas, fit_intercept=fit_intercept, normalize=normalize,
                         scoring=scoring, cv=cv, store_cv_values=store_cv_values, device=device)
        self.class_weight = class_weight

    def fit(self, X, y, sample_weight=None):
        y = np.asarray(y)
        self.classes_ = np.unique(y)
        Y = label_binarize_pm1(y, self.classes_)
        RidgeCV.fit(self, X, Y, sample_weight=sample_weight)
        self.coef_ = np.atleast_2d(self.coef_)
        self.intercept_ = np.atleast_1d(self.intercept_)
        return self
