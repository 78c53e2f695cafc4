"""Logistic regression (reference ``linear_model/_logistic.py``; SURVEY.md
N20-N22 for the stochastic solvers it replaces).

Loss and gradient are evaluated on the resolved device in fp64 (two GEMMs
per evaluation: X W^T forward, residual^T X backward, a fused
log-sum-exp); the quasi-Newton driver is scipy's L-BFGS-B on the host with
the reference's options (gtol = tol, maxiter = max_iter), so the iterates
follow the reference's lbfgs solver.  'sag' / 'saga' run the reference's
stochastic average gradient epochs (host-native, :mod:`._sag`; l1 and
elastic-net through SAGA's proximal step).  'liblinear' with the l2
penalty is liblinear's trust-region Newton method (host-native TRON,
``csrc/host/tron.cpp``; penalised bias column of intercept_scaling) -
coefficients and n_iter_ as the reference's; 'newton-cg' solves the same
strictly convex problem with the L-BFGS driver; liblinear's l1 penalty
uses an accelerated proximal gradient
(FISTA with backtracking) on the device, minimising
sum_i w_i loss_i + (1 - r) / (2C) ||W||^2 + r / C ||W||_1."""

import numbers
import warnings

import numpy as np
import torch
from scipy import optimize

from ...base import ClassifierMixin
from ...exceptions import ConvergenceWarning
from ...runtime.device import resolve_device
from ._base import LinearClassifierMixin, SparseCoefMixin, _as_dense64, _check_sample_weight
from ...base import BaseEstimator


def _check_multi_class(multi_class, solver, n_classes):
    if multi_class == "auto":
        if solver == "liblinear":
            multi_class = "ovr"
        elif n_classes > 2:
            multi_class = "multinomial"
        else:
            multi_class = "ovr"
    if multi_class not in ("multinomial", "ovr"):
        raise ValueError("multi_class should be 'multinomial', 'ovr' or 'auto'. Got %s."
                         % multi_class)
    if multi_class == "multinomial" and solver == "liblinear":
        raise ValueError("Solver %s does not support a multinomial backend." % solver)
    return multi_class


def _class_weights(class_weight, classes, y):
    if class_weight is None:
        return np.ones(len(classes))
    if class_weight == "balanced":
        counts = np.array([(y == c).sum() for c in classes], dtype=np.float64)
        return len(y) / (len(classes) * counts)
    return np.array([class_weight.get(c, 1.0) for c in classes], dtype=np.float64)


class _Objective:
    """fp64 loss / gradient on the device for a flattened weight vector."""

    def __init__(self, X, target, sw, alpha, fit_intercept, multinomial, device):
        self.dev = device
        self.X = torch.as_tensor(X, dtype=torch.float64, device=device)
        self.T = torch.as_tensor(target, dtype=torch.float64, device=device)
        self.sw = torch.as_tensor(sw, dtype=torch.float64, device=device)
        self.alpha = alpha
        self.fi = fit_intercept
        self.multi = multinomial
        self.nf = X.shape[1]

    def _split(self, w):
        W = torch.as_tensor(w, dtype=torch.float64, device=self.dev)
        if self.multi:
            W = W.reshape(self.T.shape[1], -1)
            return (W[:, :-1], W[:, -1]) if self.fi else (W, torch.zeros(W.shape[0], dtype=W.dtype,
                                                                         device=self.dev))
        return (W[:-1], W[-1]) if self.fi else (W, torch.zeros((), dtype=W.dtype, device=self.dev))

    def smooth(self, w, alpha=None):
        """(loss, grad) of sum sw * logloss + alpha/2 ||W||^2 (intercept free)."""
        alpha = self.alpha if alpha is None else alpha
        W, b = self._split(w)
        if self.multi:
            z = self.X @ W.T + b
            lse = torch.logsumexp(z, dim=1, keepdim=True)
            logp = z - lse
            loss = -(self.sw[:, None] * self.T * logp).sum() + 0.5 * alpha * (W * W).sum()
            diff = self.sw[:, None] * (torch.exp(logp) - self.T)
            gW = diff.T @ self.X + alpha * W
            g = torch.cat([gW, diff.sum(0)[:, None]], 1) if self.fi else gW
        else:
            z = self.X @ W + b
            yz = self.T * z
            loss = -(self.sw * torch.nn.functional.logsigmoid(yz)).sum() + 0.5 * alpha * (W @ W)
            z0 = self.sw * (torch.sigmoid(yz) - 1) * self.T
            gW = self.X.T @ z0 + alpha * W
            g = torch.cat([gW, z0.sum().reshape(1)]) if self.fi else gW
        return float(loss), g.reshape(-1).cpu().numpy()


def _lbfgs(obj, w0, tol, max_iter, verbose=0):
    res = optimize.minimize(obj.smooth, w0, method="L-BFGS-B", jac=True,
                            options={"iprint": -1, "gtol": tol, "maxiter": max_iter})
    if not res.success:
        warnings.warn("lbfgs failed to converge (status=%d):\n%s.\n\nIncrease the number of "
                      "iterations (max_iter) or scale the data." % (res.status, res.message),
                      ConvergenceWarning, stacklevel=3)
    return res.x, min(int(res.nit), max_iter)


def _fista(obj, w0, l1, tol, max_iter):
    """Proximal gradient with backtracking for smooth + l1 * ||W||_1."""
    nf, fi, multi = obj.nf, obj.fi, obj.multi

    def pen_mask(size):
        m = np.ones(size)
        if fi:
            if multi:
                m.reshape(obj.T.shape[1], -1)[:, -1] = 0
            else:
                m[-1] = 0
        return m

    mask = pen_mask(w0.size)
    w, z, t, L = w0.copy(), w0.copy(), 1.0, 1.0
    f_old = None
    it = 0
    for it in range(1, max_iter + 1):
        fz, gz = obj.smooth(z)
        while True:
            v = z - gz / L
            w_new = np.sign(v) * np.maximum(np.abs(v) - mask * l1 / L, 0.0)
            fw, _ = obj.smooth(w_new)
            dlt = w_new - z
            if fw <= fz + gz @ dlt + 0.5 * L * (dlt @ dlt) + 1e-12 * abs(fz):
                break
            L *= 2.0
        t_new = 0.5 * (1 + np.sqrt(1 + 4 * t * t))
        z = w_new + ((t - 1) / t_new) * (w_new - w)
        f_tot = fw + l1 * np.abs(mask * w_new).sum()
        change = np.max(np.abs(w_new - w)) / max(np.max(np.abs(w_new)), 1e-12)
        w, t = w_new, t_new
        if f_old is not None and change < tol:
            break
        f_old = f_tot
        L = max(L / 1.5, 1e-12)
    else:
        warnings.warn("FISTA did not converge; increase max_iter", ConvergenceWarning)
    return w, it


class LogisticRegression(LinearClassifierMixin, SparseCoefMixin, BaseEstimator):
    """Logistic regression classifier (ovr or multinomial)."""

    def __init__(self, penalty="l2", *, dual=False, tol=1e-4, C=1.0, fit_intercept=True,
                 intercept_scaling=1, class_weight=None, random_state=None, solver="lbfgs",
                 max_iter=100, multi_class="auto", verbose=0, warm_start=False, n_jobs=None,
                 l1_ratio=None, device=None):
        self.penalty = penalty
        self.dual = dual
        self.tol = tol
        self.C = C
        self.fit_intercept = fit_intercept
        self.intercept_scaling = intercept_scaling
        self.class_weight = class_weight
        self.random_state = random_state
        self.solver = solver
        self.max_iter = max_iter
        self.multi_class = multi_class
        self.verbose = verbose
        self.warm_start = warm_start
        self.n_jobs = n_jobs
        self.l1_ratio = l1_ratio
        self.device = device

    def fit(self, X, y, sample_weight=None):
        if not isinstance(self.C, numbers.Number) or self.C < 0:
            raise ValueError("Penalty term must be positive; got (C=%r)" % self.C)
        penalty = "none" if self.penalty is None else self.penalty
        if penalty not in ("l1", "l2", "elasticnet", "none"):
            raise ValueError("Logistic Regression supports only penalties in ['l1', 'l2', "
                             "'elasticnet', 'none'], got %s." % self.penalty)
        if self.solver not in ("lbfgs", "newton-cg", "liblinear", "sag", "saga"):
            raise ValueError("Logistic Regression supports only solvers in ['liblinear', "
                             "'newton-cg', 'lbfgs', 'sag', 'saga'], got %s." % self.solver)
        if penalty in ("l1", "elasticnet") and self.solver not in ("liblinear", "saga"):
            raise ValueError("Solver %s supports only 'l2' or 'none' penalties, got %s penalty."
                             % (self.solver, penalty))
        if penalty == "elasticnet" and (self.l1_ratio is None or
                                              not 0 <= self.l1_ratio <= 1):
            raise ValueError("l1_ratio must be between 0 and 1; got (l1_ratio=%r)"
                             % self.l1_ratio)
        if not isinstance(self.max_iter, numbers.Number) or self.max_iter < 0:
            raise ValueError("Maximum number of iteration must be positive; got (max_iter=%r)"
                             % self.max_iter)
        import scipy.sparse as _sp
        self._sparse_fit = _sp.issparse(X)
        X = _as_dense64(X).astype(np.float64)
        y = np.asarray(y)
        if y.ndim != 1:
            y = y.ravel()
        self.n_features_in_ = X.shape[1]
        self.classes_ = np.unique(y)
        n_classes = len(self.classes_)
        if n_classes < 2:
            raise ValueError("This solver needs samples of at least 2 classes in the data, but "
                             "the data contains only one class: %r" % self.classes_[0])
        multi = _check_multi_class(self.multi_class, self.solver, n_classes)
        C = np.inf if penalty == "none" else self.C
        r = 1.0 if penalty == "l1" else (self.l1_ratio if penalty == "elasticnet" else 0.0)
        alpha = 0.0 if C == np.inf else (1.0 - r) / C
        l1 = 0.0 if C == np.inf else r / C
        sw = _check_sample_weight(sample_weight, X.shape[0])
        sw = np.ones(X.shape[0]) if sw is None else sw.copy()
        cw = _class_weights(self.class_weight, self.classes_, y)
        sw_raw = sw
        sw = sw * cw[np.searchsorted(self.classes_, y)]
        dev = resolve_device(self.device)
        nf1 = X.shape[1] + int(self.fit_intercept)
        warm = getattr(self, "coef_", None) if self.warm_start else None

        def solve(obj, w0):
            if l1 > 0:
                return _fista(obj, w0, l1, self.tol, self.max_iter)
            return _lbfgs(obj, w0, self.tol, self.max_iter)

        if self.solver in ("sag", "saga"):
            W = self._fit_sag(X, y, sw, alpha, l1, multi, warm)
        elif multi == "multinomial":
            Y = (y[:, None] == self.classes_[None, :]).astype(np.float64)
            w0 = np.zeros((n_classes, nf1))
            if warm is not None:
                w0[-warm.shape[0]:, :warm.shape[1]] = warm
                if self.fit_intercept:
                    w0[-warm.shape[0]:, -1] = self.intercept_
            obj = _Objective(X, Y, sw, alpha, self.fit_intercept, True, dev)
            w, it = solve(obj, w0.ravel())
            W = w.reshape(n_classes, nf1)
            if n_classes == 2:
                W = W[1][None, :]
            self.n_iter_ = np.array([it], dtype=np.int32)
        else:
            pos = self.classes_[1:] if n_classes == 2 else self.classes_
            rows, its = [], []
            for k, c in enumerate(pos):
                t = np.where(y == c, 1.0, -1.0)
                w0 = np.zeros(nf1)
                if warm is not None:
                    w0[:warm.shape[1]] = warm[k]
                    if self.fit_intercept:
                        w0[-1] = self.intercept_[k]
                if self.solver == "liblinear" and l1 == 0 and np.isfinite(C):
                    # L2R_LR (liblinear type 0): TRON on the augmented rows,
                    # the bias column scaled by intercept_scaling and
                    # penalised like the weights (reference _base.py
                    # _fit_liblinear, linear.cpp:2320)
                    # liblinear's one-vs-rest weighs only the positive
                    # class (weighted_C[k]); the rest keep C (linear.cpp
                    # train(), nr_class > 2); binary: both classes weighted
                    Cv = sw * C if n_classes == 2 else \
                        sw_raw * C * np.where(y == c, cw[k], 1.0)
                    w, it = self._liblinear_l2(X, t, Cv, w0)
                else:
                    obj = _Objective(X, t, sw, alpha, self.fit_intercept, False, dev)
                    w, it = solve(obj, w0)
                rows.append(w)
                its.append(it)
            W = np.vstack(rows)
            self.n_iter_ = np.asarray(its, dtype=np.int32)
        if self.fit_intercept:
            self.intercept_ = W[:, -1].copy()
            if self.solver == "liblinear" and l1 == 0 and np.isfinite(C):
                self.intercept_ *= self.intercept_scaling
            self.coef_ = W[:, :-1].copy()
        else:
            self.coef_ = W
            self.intercept_ = np.zeros(W.shape[0])
        self._multi = multi
        return self

    def _liblinear_l2(self, X, t, Cvec, w0):
        from ..svm._liblinear import primal_tol, tron
        Xa = np.hstack([X, np.full((X.shape[0], 1), float(self.intercept_scaling))]) \
            if self.fit_intercept else X
        if self.fit_intercept and w0 is not None and np.any(w0):
            w0 = w0.copy()
            w0[-1] /= self.intercept_scaling
        w, it = tron(0, Xa, t, Cvec, primal_tol(self.tol, t), self.max_iter, w0=w0)
        if it >= self.max_iter:
            warnings.warn("Liblinear failed to converge, increase the number of iterations.",
                          ConvergenceWarning)
        return w, it

    def _fit_sag(self, X, y, sw, alpha, beta, multi, warm):
        """The reference's stochastic average gradient path (``_logistic.py:
        784-805``, :mod:`._sag`): one 'log' problem per class on {-1, +1}
        targets (OvR) or one 'multinomial' problem on label-encoded targets;
        returns the coefficient rows [n_rows, n_features (+1)]."""
        from ._sag import sag_solver
        n_classes = len(self.classes_)
        nf1 = X.shape[1] + int(self.fit_intercept)
        max_sq = float(np.einsum("ij,ij->i", X, X).max())
        saga = self.solver == "saga"
        if multi == "multinomial":
            w0 = np.zeros((n_classes, nf1))
            if warm is not None:
                w0[-warm.shape[0]:, :warm.shape[1]] = warm
                if self.fit_intercept:
                    w0[-warm.shape[0]:, -1] = self.intercept_
            target = np.searchsorted(self.classes_, y).astype(np.float64)
            coef, it, _ = sag_solver(X, target, sw, "multinomial", alpha, beta, self.max_iter,
                                     self.tol, self.verbose, self.random_state, False, max_sq,
                                     {"coef": w0.T}, is_saga=saga,
                                     sparse_input=getattr(self, "_sparse_fit", False))
            self.n_iter_ = np.array([it], dtype=np.int32)
            return coef[1][None, :] if n_classes == 2 else coef
        pos = self.classes_[1:] if n_classes == 2 else self.classes_
        rows, its = [], []
        for k, c in enumerate(pos):
            w0 = np.zeros(nf1)
            if warm is not None:
                w0[:warm.shape[1]] = warm[k]
                if self.fit_intercept:
                    w0[-1] = self.intercept_[k]
            t = np.where(y == c, 1.0, -1.0)
            coef, it, _ = sag_solver(X, t, sw, "log", alpha, beta, self.max_iter, self.tol,
                                     self.verbose, self.random_state, False, max_sq,
                                     {"coef": w0[:, None]}, is_saga=saga,
                                     sparse_input=getattr(self, "_sparse_fit", False))
            rows.append(coef)
            its.append(it)
        self.n_iter_ = np.asarray(its, dtype=np.int32)
        return np.vstack(rows)

    def predict_proba(self, X):
        ovr = (self.multi_class == "ovr" or
               (self.multi_class == "auto" and (len(self.classes_) <= 2 or
                                                self.solver == "liblinear")))
        if ovr:
            return self._predict_proba_lr(X)
        d = self.decision_function(X)
        d2 = np.c_[-d, d] if d.ndim == 1 else d
        d2 = d2 - d2.max(1, keepdims=True)
        e = np.exp(d2)
        return e / e.sum(1, keepdims=True)

    def predict_log_proba(self, X):
        return np.log(self.predict_proba(X))
