"""Covariance estimators (reference ``sklearn/covariance``:
``_empirical_covariance.py`` EmpiricalCovariance / log_likelihood,
``_shrunk_covariance.py`` ShrunkCovariance / LedoitWolf / OAS,
``_robust_covariance.py`` MinCovDet (FastMCD), ``_elliptic_envelope.py``,
``_graph_lasso.py`` GraphicalLasso / GraphicalLassoCV).

The O(n d^2) Gram products run on the resolved device in fp64
(``X.T @ X`` is one GEMM); the d x d algebra (inverse, shrinkage, the
graphical-lasso coordinate descent) is host numpy."""

import warnings

import numpy as np
import scipy.linalg
import torch

from .base import BaseEstimator
from .exceptions import ConvergenceWarning
from .runtime.device import resolve_device
from .utils.validation import check_is_fitted, check_random_state


def _dense(X):
    if hasattr(X, "detach"):
        X = X.detach().cpu().numpy()
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X.reshape(1, -1)
    return X


def _gram(X, device=None):
    dev = resolve_device(device)
    if dev.type == "cpu":
        return X.T @ X
    t = torch.as_tensor(X, device=dev)
    return (t.T @ t).cpu().numpy()


def empirical_covariance(X, *, assume_centered=False):
    X = _dense(X)
    if X.shape[0] == 1:
        warnings.warn("Only one sample available. You may want to reshape your data array")
    if assume_centered:
        return _gram(X) / X.shape[0]
    cov = np.cov(X.T, bias=1)
    return np.atleast_2d(cov)


def log_likelihood(emp_cov, precision):
    p = precision.shape[0]
    log_lik = -np.sum(emp_cov * precision) + np.linalg.slogdet(precision)[1]
    log_lik -= p * np.log(2 * np.pi)
    return log_lik / 2.0


def shrunk_covariance(emp_cov, shrinkage=0.1):
    emp_cov = np.asarray(emp_cov, dtype=np.float64)
    n = emp_cov.shape[0]
    mu = np.trace(emp_cov) / n
    out = (1.0 - shrinkage) * emp_cov
    out.flat[::n + 1] += shrinkage * mu
    return out


def ledoit_wolf_shrinkage(X, assume_centered=False, block_size=1000):
    X = _dense(X)
    if X.shape[0] == 1:
        return 0.0
    if not assume_centered:
        X = X - X.mean(0)
    n_samples, n_features = X.shape
    X2 = X ** 2
    emp_cov_trace = np.sum(X2, axis=0) / n_samples
    mu = np.sum(emp_cov_trace) / n_features
    beta_ = np.sum(X2.T @ X2)
    delta_ = np.sum((X.T @ X) ** 2) / n_samples ** 2
    beta = 1.0 / (n_features * n_samples) * (beta_ / n_samples - delta_)
    delta = delta_ - 2.0 * mu * emp_cov_trace.sum() + n_features * mu ** 2
    delta /= n_features
    beta = min(beta, delta)
    return 0 if beta == 0 else beta / delta


def ledoit_wolf(X, *, assume_centered=False, block_size=1000):
    X = _dense(X)
    if X.shape[1] == 1:
        if not assume_centered:
            X = X - X.mean()
        return np.atleast_2d((X ** 2).mean()), 0.0
    s = ledoit_wolf_shrinkage(X, assume_centered=assume_centered)
    emp = empirical_covariance(X, assume_centered=assume_centered)
    mu = np.sum(np.trace(emp)) / X.shape[1]
    out = (1.0 - s) * emp
    out.flat[::X.shape[1] + 1] += s * mu
    return out, s


def oas(X, *, assume_centered=False):
    X = _dense(X)
    if X.shape[1] == 1:
        if not assume_centered:
            X = X - X.mean()
        return np.atleast_2d((X ** 2).mean()), 0.0
    n_samples, n_features = X.shape
    emp = empirical_covariance(X, assume_centered=assume_centered)
    mu = np.trace(emp) / n_features
    alpha = np.mean(emp ** 2)
    num = alpha + mu ** 2
    den = (n_samples + 1.0) * (alpha - (mu ** 2) / n_features)
    s = 1.0 if den == 0 else min(num / den, 1.0)
    out = (1.0 - s) * emp
    out.flat[::n_features + 1] += s * mu
    return out, s


class EmpiricalCovariance(BaseEstimator):
    def __init__(self, *, store_precision=True, assume_centered=False):
        self.store_precision = store_precision
        self.assume_centered = assume_centered

    def _set_covariance(self, covariance):
        self.covariance_ = np.atleast_2d(covariance)
        self.precision_ = scipy.linalg.pinvh(self.covariance_, check_finite=False) \
            if self.store_precision else None

    def get_precision(self):
        if self.store_precision:
            return self.precision_
        return scipy.linalg.pinvh(self.covariance_, check_finite=False)

    def _center(self, X):
        X = _dense(X)
        self.n_features_in_ = X.shape[1]
        self.location_ = np.zeros(X.shape[1]) if self.assume_centered else X.mean(0)
        return X

    def fit(self, X, y=None):
        X = self._center(X)
        self._set_covariance(empirical_covariance(X, assume_centered=self.assume_centered))
        return self

    def score(self, X_test, y=None):
        X_test = _dense(X_test)
        test_cov = empirical_covariance(X_test - self.location_, assume_centered=True)
        return log_likelihood(test_cov, self.get_precision())

    def error_norm(self, comp_cov, norm="frobenius", scaling=True, squared=True):
        err = comp_cov - self.covariance_
        if norm == "frobenius":
            e = np.sum(err ** 2)
        elif norm == "spectral":
            e = np.amax(np.linalg.svd(err.T @ err, compute_uv=False))
        else:
            raise NotImplementedError("Only spectral and frobenius norms are implemented")
        if scaling:
            e = e / err.shape[0]
        return e if squared else np.sqrt(e)

    def mahalanobis(self, X):
        X = _dense(X)
        Xc = X - self.location_
        return np.einsum("ij,jk,ik->i", Xc, self.get_precision(), Xc)


class ShrunkCovariance(EmpiricalCovariance):
    def __init__(self, *, store_precision=True, assume_centered=False, shrinkage=0.1):
        super().__init__(store_precision=store_precision, assume_centered=assume_centered)
        self.shrinkage = shrinkage

    def fit(self, X, y=None):
        X = self._center(X)
        cov = shrunk_covariance(empirical_covariance(X, assume_centered=self.assume_centered),
                                self.shrinkage)
        self._set_covariance(cov)
        return self


class LedoitWolf(EmpiricalCovariance):
    def __init__(self, *, store_precision=True, assume_centered=False, block_size=1000):
        super().__init__(store_precision=store_precision, assume_centered=assume_centered)
        self.block_size = block_size

    def fit(self, X, y=None):
        X = self._center(X)
        cov, s = ledoit_wolf(X - self.location_, assume_centered=True)
        self.shrinkage_ = s
        self._set_covariance(cov)
        return self


class OAS(EmpiricalCovariance):
    def fit(self, X, y=None):
        X = self._center(X)
        cov, s = oas(X - self.location_, assume_centered=True)
        self.shrinkage_ = s
        self._set_covariance(cov)
        return self


# ------------------------------------------------------------- robust (MCD)
def _c_step(X, n_support, random_state, remaining_iterations=30, initial_estimates=None):
    n_samples, n_features = X.shape
    dist = np.inf
    if initial_estimates is None:
        support = np.zeros(n_samples, dtype=bool)
        support[random_state.permutation(n_samples)[:n_support]] = True
    else:
        location, covariance = initial_estimates
        precision = scipy.linalg.pinvh(covariance)
        Xc = X - location
        dist = (Xc @ precision * Xc).sum(1)
        support = np.zeros(n_samples, dtype=bool)
        support[np.argsort(dist)[:n_support]] = True
    Xs = X[support]
    location = Xs.mean(0)
    covariance = empirical_covariance(Xs)
    det = np.linalg.slogdet(covariance)[1]
    if np.isinf(det):
        precision = scipy.linalg.pinvh(covariance)
    previous_det = np.inf
    while det < previous_det and remaining_iterations > 0 and not np.isinf(det):
        previous = (location, covariance, det, support, dist)
        previous_det = det
        precision = scipy.linalg.pinvh(covariance)
        Xc = X - location
        dist = (Xc @ precision * Xc).sum(1)
        support = np.zeros(n_samples, dtype=bool)
        support[np.argsort(dist)[:n_support]] = True
        Xs = X[support]
        location = Xs.mean(axis=0)
        covariance = empirical_covariance(Xs)
        det = np.linalg.slogdet(covariance)[1]
        remaining_iterations -= 1
    if np.allclose(det, previous_det):
        pass
    if det > previous_det:
        location, covariance, det, support, dist = previous
    return location, covariance, det, support, dist


def fast_mcd(X, support_fraction=None, random_state=None):
    random_state = check_random_state(random_state)
    X = _dense(X)
    n_samples, n_features = X.shape
    n_support = int(np.ceil(0.5 * (n_samples + n_features + 1))) if support_fraction is None \
        else int(support_fraction * n_samples)
    if n_features == 1:
        if n_support < n_samples:
            Xs = np.sort(X[:, 0])
            diff = Xs[n_support:] - Xs[:(n_samples - n_support)]
            half = np.where(diff == diff.min())[0]
            loc = 0.5 * (Xs[n_support + half] + Xs[half]).mean()
            support = np.zeros(n_samples, dtype=bool)
            support[np.argsort(np.abs(X[:, 0] - loc))[:n_support]] = True
            cov = np.atleast_2d(np.var(X[support]))
            loc = np.array([np.mean(X[support])])
        else:
            support = np.ones(n_samples, dtype=bool)
            cov = np.atleast_2d(np.var(X))
            loc = np.array([np.mean(X)])
        Xc = X - loc
        dist = (Xc @ scipy.linalg.pinvh(cov) * Xc).sum(1)
        return loc, cov, support, dist
    n_trials = 30
    results = [_c_step(X, n_support, random_state, remaining_iterations=2) for _ in range(n_trials)]
    best = sorted(results, key=lambda r: r[2])[:10]
    refined = [_c_step(X, n_support, random_state, remaining_iterations=100,
                       initial_estimates=(r[0], r[1])) for r in best]
    loc, cov, det, support, dist = min(refined, key=lambda r: r[2])
    return loc, cov, support, dist


class MinCovDet(EmpiricalCovariance):
    def __init__(self, *, store_precision=True, assume_centered=False, support_fraction=None,
                 random_state=None):
        super().__init__(store_precision=store_precision, assume_centered=assume_centered)
        self.support_fraction = support_fraction
        self.random_state = random_state

    def fit(self, X, y=None):
        X = _dense(X)
        self.n_features_in_ = X.shape[1]
        rs = check_random_state(self.random_state)
        loc, cov, support, dist = fast_mcd(X, self.support_fraction, rs)
        if self.assume_centered:
            loc = np.zeros(X.shape[1])
            cov = empirical_covariance(X[support], assume_centered=True)
            dist = (X @ scipy.linalg.pinvh(cov) * X).sum(1)
        self.raw_location_, self.raw_covariance_, self.raw_support_ = loc, cov, support
        self.location_ = loc
        self.support_ = support
        self.dist_ = dist
        self.correct_covariance(X)
        self.reweight_covariance(X)
        return self

    def correct_covariance(self, data):
        n_samples = len(self.dist_)
        n_support = np.sum(self.support_)
        if n_support < n_samples and np.allclose(self.raw_covariance_, 0):
            raise ValueError("The covariance matrix of the support data is equal to 0, try to "
                             "increase support_fraction")
        from scipy.stats import chi2
        correction = np.median(self.dist_) / chi2(data.shape[1]).isf(0.5)
        covariance_corrected = self.raw_covariance_ * correction
        self.dist_ /= correction
        return covariance_corrected

    def reweight_covariance(self, data):
        from scipy.stats import chi2
        n_samples, n_features = data.shape
        mask = self.dist_ < chi2(n_features).isf(0.025)
        location = np.zeros(n_features) if self.assume_centered else data[mask].mean(0)
        cov = empirical_covariance(data[mask], assume_centered=self.assume_centered)
        self._set_covariance(cov)
        self.location_ = location
        self.support_ = mask
        Xc = data - self.location_
        self.dist_ = (Xc @ self.get_precision() * Xc).sum(1)
        return location, cov, mask


class EllipticEnvelope(MinCovDet):
    _estimator_type = "outlier_detector"

    def __init__(self, *, store_precision=True, assume_centered=False, support_fraction=None,
                 contamination=0.1, random_state=None):
        super().__init__(store_precision=store_precision, assume_centered=assume_centered,
                         support_fraction=support_fraction, random_state=random_state)
        self.contamination = contamination

    def fit(self, X, y=None):
        if not 0.0 < self.contamination <= 0.5:
            raise ValueError("contamination must be in (0, 0.5]")
        super().fit(X)
        self.offset_ = np.percentile(-self.dist_, 100.0 * self.contamination)
        return self

    def decision_function(self, X):
        return -self.mahalanobis(X) - self.offset_

    def score_samples(self, X):
        return -self.mahalanobis(X)

    def predict(self, X):
        return np.where(self.decision_function(X) < 0, -1, 1)

    def fit_predict(self, X, y=None):
        return self.fit(X).predict(X)

    def score(self, X, y, sample_weight=None):
        from .utils.metrics import accuracy_score
        return accuracy_score(y, self.predict(X), sample_weight=sample_weight)


# ----------------------------------------------------------- graphical lasso
def _lasso_cd(Q, b, alpha, w, max_iter=100, tol=1e-4):
    """min 0.5 w'Qw - b'w + alpha |w|_1 by cyclic coordinate descent."""
    for _ in range(max_iter):
        w_max = 0.0
        d_max = 0.0
        for j in range(len(b)):
            old = w[j]
            r = b[j] - Q[j] @ w + Q[j, j] * w[j]
            w[j] = np.sign(r) * max(abs(r) - alpha, 0.0) / Q[j, j]
            d_max = max(d_max, abs(w[j] - old))
            w_max = max(w_max, abs(w[j]))
        if w_max == 0 or d_max / w_max < tol:
            break
    return w


def graphical_lasso(emp_cov, alpha, *, cov_init=None, mode="cd", tol=1e-4, enet_tol=1e-4,
                    max_iter=100, verbose=False, return_costs=False, eps=np.finfo(np.float64).eps,
                    return_n_iter=False):
    _, n_features = emp_cov.shape
    if alpha == 0:
        precision = scipy.linalg.inv(emp_cov)
        out = (emp_cov, precision)
        if return_costs:
            out = out + ([],)
        if return_n_iter:
            out = out + (0,)
        return out
    covariance_ = emp_cov.copy() if cov_init is None else cov_init.copy()
    covariance_ *= 0.95
    diagonal = emp_cov.flat[::n_features + 1]
    covariance_.flat[::n_features + 1] = diagonal
    precision_ = scipy.linalg.pinvh(covariance_)
    indices = np.arange(n_features)
    costs = []
    for i in range(max_iter):
        for idx in range(n_features):
            sub_cov = np.ascontiguousarray(covariance_[indices != idx].T[indices != idx])
            row = emp_cov[idx, indices != idx]
            coefs = -(precision_[indices != idx, idx] / (precision_[idx, idx] + 1000 * eps))
            coefs = _lasso_cd(sub_cov, row, alpha, coefs, max_iter=int(max_iter),
                              tol=enet_tol)
            precision_[idx, idx] = 1.0 / (covariance_[idx, idx]
                                          - covariance_[indices != idx, idx] @ coefs)
            precision_[indices != idx, idx] = -precision_[idx, idx] * coefs
            precision_[idx, indices != idx] = -precision_[idx, idx] * coefs
            coefs = sub_cov @ coefs
            covariance_[idx, indices != idx] = coefs
            covariance_[indices != idx, idx] = coefs
        d_gap = (np.sum(emp_cov * precision_) - n_features
                 + alpha * (np.abs(precision_).sum() - np.abs(np.diag(precision_)).sum()))
        cost = (-log_likelihood(emp_cov, precision_) * 2 / 1.0)
        costs.append((cost, d_gap))
        if np.abs(d_gap) < tol:
            break
    else:
        warnings.warn("graphical_lasso: did not converge after %i iteration: dual gap: %.3e"
                      % (max_iter, d_gap), ConvergenceWarning)
    out = (covariance_, precision_)
    if return_costs:
        out = out + (costs,)
    if return_n_iter:
        out = out + (i + 1,)
    return out


class GraphicalLasso(EmpiricalCovariance):
    def __init__(self, alpha=0.01, *, mode="cd", tol=1e-4, enet_tol=1e-4, max_iter=100,
                 verbose=False, assume_centered=False):
        super().__init__(assume_centered=assume_centered)
        self.alpha = alpha
        self.mode = mode
        self.tol = tol
        self.enet_tol = enet_tol
        self.max_iter = max_iter
        self.verbose = verbose

    def fit(self, X, y=None):
        X = self._center(X)
        emp = empirical_covariance(X, assume_centered=self.assume_centered)
        self.covariance_, self.precision_, self.n_iter_ = graphical_lasso(
            emp, alpha=self.alpha, tol=self.tol, enet_tol=self.enet_tol,
            max_iter=self.max_iter, return_n_iter=True)
        return self


class GraphicalLassoCV(GraphicalLasso):
    def __init__(self, *, alphas=4, n_refinements=4, cv=None, tol=1e-4, enet_tol=1e-4,
                 max_iter=100, mode="cd", n_jobs=None, verbose=False, assume_centered=False):
        super().__init__(mode=mode, tol=tol, enet_tol=enet_tol, max_iter=max_iter,
                         verbose=verbose, assume_centered=assume_centered)
        self.alphas = alphas
        self.n_refinements = n_refinements
        self.cv = cv
        self.n_jobs = n_jobs

    def fit(self, X, y=None):
        from .model_selection import check_cv
        X = self._center(X)
        emp = empirical_covariance(X, assume_centered=self.assume_centered)
        if np.isscalar(self.alphas):
            a_max = np.max(np.abs(emp - np.diag(np.diag(emp))))
            alphas = np.logspace(np.log10(a_max), np.log10(a_max * 1e-2), int(self.alphas))
        else:
            alphas = np.asarray(self.alphas)
        cv = check_cv(self.cv)
        scores = np.zeros(len(alphas))
        for tr, te in cv.split(X):
            e_tr = empirical_covariance(X[tr], assume_centered=self.assume_centered)
            e_te = empirical_covariance(X[te], assume_centered=self.assume_centered)
            for i, a in enumerate(alphas):
                with warnings.catch_warnings():
                    warnings.simplefilter("ignore", ConvergenceWarning)
                    _, prec = graphical_lasso(e_tr, a, tol=self.tol, max_iter=self.max_iter)
                scores[i] += log_likelihood(e_te, prec)
        best = int(np.argmax(scores))
        self.alpha_ = alphas[best]
        self.cv_alphas_ = list(alphas)
        self.grid_scores_ = scores
        self.covariance_, self.precision_, self.n_iter_ = graphical_lasso(
            emp, alpha=self.alpha_, tol=self.tol, enet_tol=self.enet_tol,
            max_iter=self.max_iter, return_n_iter=True)
        return self


__all__ = ["EmpiricalCovariance", "ShrunkCovariance", "LedoitWolf", "OAS", "MinCovDet",
           "EllipticEnvelope", "GraphicalLasso", "GraphicalLassoCV", "empirical_covariance",
           "shrunk_covariance", "ledoit_wolf", "ledoit_wolf_shrinkage", "oas", "log_likelihood",
           "graphical_lasso", "fast_mcd"]

from .utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
