"""Linear SVMs with liblinear semantics (reference ``svm/_classes.py``:
LinearSVC :15-258, LinearSVR :259-444; ``svm/_base.py: _fit_liblinear``;
solvers of ``svm/src/liblinear/linear.cpp``).

Dual problems (the default ``dual=True``) run the host-native dual
coordinate descent (``csrc/host/liblinear_cd.cpp``) with the reference's
class-grouped sample order, per-instance C, shrinking and mt19937 visiting
order - the fitted coefficients are the reference's.  Primal problems
(``dual=False``) minimise the same objective with L-BFGS (squared losses)
or proximal gradient (L1 penalty); the optimum is the same, the iterates are
not.  The regularised bias column of liblinear (``intercept_scaling``) is
kept.
"""

import warnings

import numpy as np
import scipy.sparse as sp

from ...base import BaseEstimator, ClassifierMixin, RegressorMixin
from ...exceptions import ConvergenceWarning
from ...ops import _host
from ...utils.class_weight import compute_class_weight
from ...utils.validation import check_is_fitted, check_random_state


def _dense(X):
    if hasattr(X, "detach"):
        X = X.detach().cpu().numpy()
    if sp.issparse(X):
        X = X.toarray()
    return np.ascontiguousarray(X, dtype=np.float64)


def _augment(X, fit_intercept, intercept_scaling):
    if not fit_intercept:
        return X
    if intercept_scaling <= 0:
        raise ValueError("Intercept scaling is %r but needs to be greater than 0. To disable "
                         "fitting an intercept, set fit_intercept=False." % intercept_scaling)
    return np.hstack([X, np.full((X.shape[0], 1), float(intercept_scaling))])


class _MTStream:
    """One mt19937 stream per fit, shared by its sub-problems (reference)."""

    def __init__(self, seed):
        self.h = _host.lib().sqh_mt_new(int(seed) & 0xFFFFFFFF)

    def __del__(self):
        if getattr(self, "h", None):
            _host.lib().sqh_mt_free(self.h)
            self.h = None


def _svc_dual(X, y, C, l1loss, tol, max_iter, stream):
    w = np.zeros(X.shape[1])
    X = np.ascontiguousarray(X)
    y = np.ascontiguousarray(y, dtype=np.float64)
    C = np.ascontiguousarray(C, dtype=np.float64)
    it = _host.lib().sqh_linear_svc_dual(X.ctypes.data, X.shape[0], X.shape[1], y.ctypes.data,
                                         C.ctypes.data, int(l1loss), float(tol), int(max_iter),
                                         stream.h, w.ctypes.data, None)
    return w, it


def tron(kind, X, y, C, eps, max_iter, p=0.0, w0=None):
    """liblinear's trust-region Newton method on the primal (host native,
    ``csrc/host/tron.cpp``): kind 0 L2R_LR, 1 L2R_L2LOSS_SVC, 2
    L2R_L2LOSS_SVR.  Returns (w, iterations)."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    C = np.ascontiguousarray(np.broadcast_to(C, (X.shape[0],)), dtype=np.float64)
    w = np.zeros(X.shape[1]) if w0 is None else np.array(w0, dtype=np.float64)
    it = _host.lib().sqh_tron(X.ctypes.data, X.shape[0], X.shape[1], y.ctypes.data, C.ctypes.data,
                              int(kind), float(p), float(eps), int(max_iter), w.ctypes.data)
    return w, int(it)


def primal_tol(tol, y):
    """liblinear's primal stopping tolerance for the classification types:
    eps * max(min(#pos, #neg), 1) / l (reference ``linear.cpp:2315``)."""
    pos = int(np.sum(y > 0))
    return tol * max(min(pos, len(y) - pos), 1) / len(y)


def _svc_primal_l2(X, y, C, tol, max_iter):
    """min 0.5 |w|^2 + sum C_i max(0, 1 - y_i w.x_i)^2 (liblinear type 2) by
    TRON."""
    return tron(1, X, y, C, primal_tol(tol, y), max_iter)


def _svc_primal_l1(X, y, C, tol, max_iter):
    """min |w|_1 + sum C_i max(0, 1 - y_i w.x_i)^2 by FISTA (liblinear type 5)."""
    L = 2 * np.max(C) * np.linalg.norm(X, 2) ** 2 + 1e-12
    w = np.zeros(X.shape[1])
    z, t = w.copy(), 1.0
    it = 0
    for it in range(1, max_iter * 10 + 1):
        a = np.maximum(1 - y * (X @ z), 0)
        g = -2 * X.T @ (C * a * y)
        w_new = z - g / L
        w_new = np.sign(w_new) * np.maximum(np.abs(w_new) - 1.0 / L, 0.0)
        t_new = (1 + np.sqrt(1 + 4 * t * t)) / 2
        z = w_new + (t - 1) / t_new * (w_new - w)
        if np.max(np.abs(w_new - w)) <= tol * max(1.0, np.max(np.abs(w_new))):
            w = w_new
            break
        w, t = w_new, t_new
    return w, it


def _svc_crammer_singer(X, y, Cvec, K, tol, stream, max_iter=100000):
    """Crammer-Singer multi-class dual (host native, ``sqh_linear_mcsvm_cs``):
    returns (coef rows [K, d], iterations)."""
    X = np.ascontiguousarray(X)
    yi = np.ascontiguousarray(y, dtype=np.int32)
    C = np.ascontiguousarray(Cvec, dtype=np.float64)
    w = np.zeros(X.shape[1] * K)
    it = _host.lib().sqh_linear_mcsvm_cs(X.ctypes.data, X.shape[0], X.shape[1], yi.ctypes.data,
                                         int(K), C.ctypes.data, float(tol), int(max_iter),
                                         stream.h, w.ctypes.data)
    return w.reshape(X.shape[1], K).T.copy(), it


class LinearSVC(ClassifierMixin, BaseEstimator):
    """Linear support vector classification (one-vs-rest or Crammer-Singer,
    liblinear)."""

    def __init__(self, penalty="l2", loss="squared_hinge", *, dual=True, tol=1e-4, C=1.0,
                 multi_class="ovr", fit_intercept=True, intercept_scaling=1, class_weight=None,
                 verbose=0, random_state=None, max_iter=1000):
        self.dual = dual
        self.tol = tol
        self.C = C
        self.multi_class = multi_class
        self.fit_intercept = fit_intercept
        self.intercept_scaling = intercept_scaling
        self.class_weight = class_weight
        self.verbose = verbose
        self.random_state = random_state
        self.max_iter = max_iter
        self.penalty = penalty
        self.loss = loss

    def _solver(self):
        if self.multi_class == "crammer_singer":
            return "cs"
        key = (self.penalty, self.loss, bool(self.dual))
        table = {("l2", "squared_hinge", True): "l2l2_dual", ("l2", "hinge", True): "l2l1_dual",
                 ("l2", "squared_hinge", False): "l2l2_primal",
                 ("l1", "squared_hinge", False): "l1l2_primal"}
        if key not in table:
            raise ValueError("Unsupported set of arguments: The combination of penalty='%s' and "
                             "loss='%s' are not supported when dual=%s" % key)
        return table[key]

    def fit(self, X, y, sample_weight=None):
        if self.C < 0:
            raise ValueError("Penalty term must be positive; got (C=%r)" % self.C)
        X = _dense(X)
        y = np.asarray(y).reshape(-1)
        self.n_features_in_ = X.shape[1]
        self.classes_, y_ind = np.unique(y, return_inverse=True)
        if len(self.classes_) < 2:
            raise ValueError("This solver needs samples of at least 2 classes in the data, but "
                             "the data contains only one class: %r" % self.classes_[0])
        cw = compute_class_weight(self.class_weight, classes=self.classes_, y=y)
        sw = np.ones(X.shape[0]) if sample_weight is None else \
            np.asarray(sample_weight, dtype=np.float64)
        rnd = check_random_state(self.random_state)
        seed = rnd.randint(np.iinfo("i").max)
        Xa = _augment(X, self.fit_intercept, self.intercept_scaling)
        solver = self._solver()
        # liblinear groups samples by (sorted) class, original order within a class
        perm = np.argsort(y_ind, kind="stable")
        Xp, yp, swp = Xa[perm], y_ind[perm], sw[perm]
        weighted_C = self.C * cw
        K = len(self.classes_)
        models = []
        n_iter = 0
        stream = _MTStream(seed)
        tasks = []
        if solver == "cs":
            # one joint problem over all classes; the reference runs it with
            # the solver's own iteration cap (linear.cpp:496, :2530)
            raw, n_iter = _svc_crammer_singer(Xp, yp, swp * weighted_C[yp], K, self.tol, stream)
        elif K == 2:
            tasks = [(np.where(yp == 1, 1.0, -1.0), weighted_C[1], weighted_C[0])]
        else:
            tasks = [(np.where(yp == k, 1.0, -1.0), weighted_C[k], self.C) for k in range(K)]
        for ysub, Cp, Cn in tasks:
            Cvec = swp * np.where(ysub > 0, Cp, Cn)
            if solver in ("l2l2_dual", "l2l1_dual"):
                w, it = _svc_dual(Xp, ysub, Cvec, solver == "l2l1_dual", self.tol, self.max_iter,
                                  stream)
            elif solver == "l2l2_primal":
                w, it = _svc_primal_l2(Xp, ysub, Cvec, self.tol, self.max_iter)
            else:
                w, it = _svc_primal_l1(Xp, ysub, Cvec, self.tol, self.max_iter)
            models.append(w)
            n_iter = max(n_iter, it)
        if solver != "cs":
            raw = np.asarray(models)
        if self.fit_intercept:
            self.coef_ = raw[:, :-1]
            self.intercept_ = self.intercept_scaling * raw[:, -1]
        else:
            self.coef_ = raw
            self.intercept_ = np.zeros(raw.shape[0])
        if solver == "cs" and K == 2:
            # binary Crammer-Singer: the score difference (reference
            # svm/_classes.py:242-246)
            self.coef_ = (self.coef_[1] - self.coef_[0]).reshape(1, -1)
            self.intercept_ = np.array([self.intercept_[1] - self.intercept_[0]])
        self.n_iter_ = n_iter
        if n_iter >= self.max_iter:
            warnings.warn("Liblinear failed to converge, increase the number of iterations.",
                          ConvergenceWarning)
        return self

    def decision_function(self, X):
        check_is_fitted(self)
        X = _dense(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError(f"X has {X.shape[1]} features, but LinearSVC is expecting "
                             f"{self.n_features_in_} features as input.")
        s = X @ self.coef_.T + self.intercept_
        return s.ravel() if s.shape[1] == 1 else s

    def predict(self, X):
        s = self.decision_function(X)
        idx = (s > 0).astype(int) if s.ndim == 1 else s.argmax(axis=1)
        return self.classes_[idx]

    def densify(self):
        return self

    def sparsify(self):
        self.coef_ = sp.csr_matrix(self.coef_)
        return self


class LinearSVR(RegressorMixin, BaseEstimator):
    """Linear support vector regression (liblinear)."""

    def __init__(self, *, epsilon=0.0, tol=1e-4, C=1.0, loss="epsilon_insensitive",
                 fit_intercept=True, intercept_scaling=1.0, dual=True, verbose=0,
                 random_state=None, max_iter=1000):
        self.tol = tol
        self.C = C
        self.epsilon = epsilon
        self.fit_intercept = fit_intercept
        self.intercept_scaling = intercept_scaling
        self.verbose = verbose
        self.random_state = random_state
        self.max_iter = max_iter
        self.dual = dual
        self.loss = loss

    def fit(self, X, y, sample_weight=None):
        if self.C < 0:
            raise ValueError("Penalty term must be positive; got (C=%r)" % self.C)
        X = _dense(X)
        y = np.asarray(y, dtype=np.float64).reshape(-1)
        self.n_features_in_ = X.shape[1]
        sw = np.ones(X.shape[0]) if sample_weight is None else \
            np.asarray(sample_weight, dtype=np.float64)
        rnd = check_random_state(self.random_state)
        seed = rnd.randint(np.iinfo("i").max)
        Xa = np.ascontiguousarray(_augment(X, self.fit_intercept, self.intercept_scaling))
        Cvec = np.ascontiguousarray(sw * self.C)
        if self.loss == "epsilon_insensitive" and not self.dual:
            raise ValueError("Unsupported set of arguments: loss='epsilon_insensitive' is not "
                             "supported when dual=False")
        if self.loss not in ("epsilon_insensitive", "squared_epsilon_insensitive"):
            raise ValueError("loss='%s' is not supported" % self.loss)
        if self.dual:
            w = np.zeros(Xa.shape[1])
            stream = _MTStream(seed)     # must outlive the native call
            it = _host.lib().sqh_linear_svr_dual(
                Xa.ctypes.data, Xa.shape[0], Xa.shape[1], y.ctypes.data, Cvec.ctypes.data,
                int(self.loss == "epsilon_insensitive"), float(self.epsilon), float(self.tol),
                int(self.max_iter), stream.h, w.ctypes.data)
        else:
            # L2R_L2LOSS_SVR primal: TRON with eps = tol (reference linear.cpp:2397)
            w, it = tron(2, Xa, y, Cvec, self.tol, self.max_iter, p=self.epsilon)
        if self.fit_intercept:
            self.coef_ = w[:-1]
            self.intercept_ = np.array([self.intercept_scaling * w[-1]])
        else:
            self.coef_ = w
            self.intercept_ = np.array([0.0])
        self.n_iter_ = it
        if it >= self.max_iter:
            warnings.warn("Liblinear failed to converge, increase the number of iterations.",
                          ConvergenceWarning)
        return self

    def predict(self, X):
        check_is_fitted(self)
        X = _dense(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError(f"X has {X.shape[1]} features, but LinearSVR is expecting "
                             f"{self.n_features_in_} features as input.")
        return X @ self.coef_ + self.intercept_[0]


__all__ = ["LinearSVC", "LinearSVR"]
