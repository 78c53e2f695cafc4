"""Gaussian mixture models (reference ``sklearn/mixture/_base.py`` EM
driver :155-260 and ``_gaussian_mixture.py``: parameter estimation for
full / tied / diag / spherical covariances, Cholesky precisions, E-step log
probabilities, BIC / AIC, sampling).

The EM iterations run in torch fp64 on the resolved device: the E-step is
one batched triangular GEMM per component and a logsumexp over k, the
M-step a (k x n) @ (n x d) GEMM plus per-component scatter matrices -
exactly the shapes the MI355X is built for; only the k x d x d Cholesky
factorisations are small."""

import warnings

import numpy as np
import torch

from .base import BaseEstimator, DensityMixin
from .exceptions import ConvergenceWarning
from .runtime.device import resolve_device
from .utils.validation import check_is_fitted, check_random_state


def _dense(X):
    if hasattr(X, "detach"):
        X = X.detach().cpu().numpy()
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X.reshape(-1, 1)
    return X


def _split_k(n, target=512):
    """Number of row chunks for a split-K reduction over n rows."""
    return max(1, n // target)


def _atb(A, B):
    """A^T B for tall (n, p) / (n, q) operands with small p, q.  A library
    GEMM maps such a product onto a single output tile, i.e. one CU walking
    all n rows; splitting the rows into chunks turns it into a batched GEMM
    over many CUs followed by a tiny reduction."""
    n = A.shape[0]
    C = _split_k(n)
    if C == 1 or A.device.type == "cpu":
        return A.T @ B
    m = (n // C) * C
    out = torch.bmm(A[:m].reshape(C, n // C, -1).transpose(1, 2),
                    B[:m].reshape(C, n // C, -1)).sum(0)
    if m < n:
        out += A[m:].T @ B[m:]
    return out


def _weighted_scatter(X, means, resp):
    """Per-component sum_i r_ik (x_i - m_k)(x_i - m_k)^T, batched over the
    components and split over the rows (see ``_atb``)."""
    n, d = X.shape
    K = means.shape[0]
    if X.device.type == "cpu":
        out = torch.empty((K, d, d), dtype=X.dtype)
        for k in range(K):
            diff = X - means[k]
            out[k] = (resp[:, k, None] * diff).T @ diff
        return out
    # bound the temporaries to ~1 GiB: per (component group, row chunk) the
    # loop holds three (g, rows, d) tensors - D, Dw and the split-K reshape
    budget = 1 << 30
    per_row = 3 * X.element_size() * d
    rows = max(1, min(n, budget // max(1, per_row)))
    kg = max(1, min(K, budget // max(1, per_row * rows)))
    out = torch.zeros((K, d, d), dtype=X.dtype, device=X.device)
    for r0 in range(0, n, rows):
        Xr = X[r0:r0 + rows]
        rr = resp[r0:r0 + rows]
        nr = Xr.shape[0]
        C = _split_k(nr)
        m = (nr // C) * C
        for k0 in range(0, K, kg):
            k1 = min(K, k0 + kg)
            D = Xr[None] - means[k0:k1, None, :]                     # (g, rows, d)
            Dw = D * rr[:, k0:k1].T[:, :, None]
            g = k1 - k0
            acc = torch.bmm(Dw[:, :m].reshape(g * C, nr // C, d).transpose(1, 2),
                            D[:, :m].reshape(g * C, nr // C, d)).reshape(g, C, d, d).sum(1)
            if m < nr:
                acc += torch.bmm(Dw[:, m:].transpose(1, 2), D[:, m:])
            out[k0:k1] += acc
    return out


def _estimate_gaussian_parameters(X, resp, reg_covar, covariance_type):
    nk = resp.sum(0) + 10 * torch.finfo(resp.dtype).eps
    means = _atb(resp, X) / nk[:, None]
    d = X.shape[1]
    if covariance_type == "full":
        cov = _weighted_scatter(X, means, resp) / nk[:, None, None]
        cov.diagonal(dim1=-2, dim2=-1).add_(reg_covar)
    elif covariance_type == "tied":
        avg_X2 = _atb(X, X)
        avg_means2 = (nk * means.T) @ means
        cov = (avg_X2 - avg_means2) / nk.sum()
        cov.diagonal().add_(reg_covar)
    elif covariance_type == "diag":
        avg_X2 = _atb(resp, X * X) / nk[:, None]
        avg_means2 = means ** 2
        avg_X_means = means * _atb(resp, X) / nk[:, None]
        cov = avg_X2 - 2 * avg_X_means + avg_means2 + reg_covar
    else:
        avg_X2 = _atb(resp, X * X) / nk[:, None]
        avg_means2 = means ** 2
        avg_X_means = means * _atb(resp, X) / nk[:, None]
        cov = (avg_X2 - 2 * avg_X_means + avg_means2 + reg_covar).mean(1)
    return nk, means, cov


_CHOL_ERR = ("Fitting the mixture model failed because some components have ill-defined "
             "empirical covariance (for instance caused by singleton or collapsed samples). "
             "Try to decrease the number of components, or increase reg_covar.")


def _compute_precision_cholesky(cov, covariance_type):
    if covariance_type == "full":
        d = cov.shape[-1]
        L, info = torch.linalg.cholesky_ex(cov)
        if bool((info != 0).any()):
            raise ValueError(_CHOL_ERR)
        eye = torch.eye(d, dtype=cov.dtype, device=cov.device).expand_as(cov)
        return torch.linalg.solve_triangular(L, eye, upper=False).transpose(-1, -2)
    if covariance_type == "tied":
        L, info = torch.linalg.cholesky_ex(cov)
        if int(info) != 0:
            raise ValueError(_CHOL_ERR)
        eye = torch.eye(cov.shape[0], dtype=cov.dtype, device=cov.device)
        return torch.linalg.solve_triangular(L, eye, upper=False).T
    if bool((cov <= 0.0).any()):
        raise ValueError(_CHOL_ERR)
    return 1.0 / torch.sqrt(cov)


def _log_det_cholesky(pc, covariance_type, n_features):
    if covariance_type == "full":
        return torch.log(torch.diagonal(pc, dim1=-2, dim2=-1)).sum(-1)
    if covariance_type == "tied":
        return torch.log(torch.diagonal(pc)).sum()
    if covariance_type == "diag":
        return torch.log(pc).sum(1)
    return n_features * torch.log(pc)


def _estimate_log_gaussian_prob(X, means, pc, covariance_type):
    n, d = X.shape
    log_det = _log_det_cholesky(pc, covariance_type, d)
    if covariance_type == "full":
        y = torch.einsum("nd,kde->kne", X, pc) - torch.einsum("kd,kde->ke", means, pc)[:, None, :]
        log_prob = (y * y).sum(-1).T
    elif covariance_type == "tied":
        Xp = X @ pc
        log_prob = torch.stack([((Xp - m) ** 2).sum(1) for m in (means @ pc)], dim=1)
    elif covariance_type == "diag":
        prec = pc ** 2
        log_prob = ((means ** 2 * prec).sum(1) - 2.0 * X @ (means * prec).T
                    + (X ** 2) @ prec.T)
    else:
        prec = pc ** 2
        log_prob = ((means ** 2).sum(1) * prec - 2 * X @ means.T * prec
                    + torch.outer((X ** 2).sum(1), prec))
    return -0.5 * (d * np.log(2 * np.pi) + log_prob) + log_det


class BaseMixture(DensityMixin, BaseEstimator):
    """Base of the mixture models (reference ``mixture/_base.py``): EM
    estimators exposing fit / predict / predict_proba / score_samples /
    sample."""


class GaussianMixture(BaseMixture):
    def __init__(self, n_components=1, *, covariance_type="full", tol=1e-3, reg_covar=1e-6,
                 max_iter=100, n_init=1, init_params="kmeans", weights_init=None,
                 means_init=None, precisions_init=None, random_state=None, warm_start=False,
                 verbose=0, verbose_interval=10, device=None):
        self.n_components = n_components
        self.covariance_type = covariance_type
        self.tol = tol
        self.reg_covar = reg_covar
        self.max_iter = max_iter
        self.n_init = n_init
        self.init_params = init_params
        self.weights_init = weights_init
        self.means_init = means_init
        self.precisions_init = precisions_init
        self.random_state = random_state
        self.warm_start = warm_start
        self.verbose = verbose
        self.verbose_interval = verbose_interval
        self.device = device

    # ----------------------------------------------------------- internals
    def _t(self, a):
        return torch.as_tensor(np.asarray(a, dtype=np.float64), device=self._dev)

    def _check_parameters(self, X):
        if self.covariance_type not in ("spherical", "tied", "diag", "full"):
            raise ValueError("Invalid value for 'covariance_type': %s 'covariance_type' should "
                             "be in ['spherical', 'tied', 'diag', 'full']" % self.covariance_type)
        if self.n_components < 1:
            raise ValueError("Invalid value for 'n_components': %d Estimation requires at least "
                             "one component" % self.n_components)
        if X.shape[0] < self.n_components:
            raise ValueError("Expected n_samples >= n_components but got n_components = %d, "
                             "n_samples = %d" % (self.n_components, X.shape[0]))

    def _initialize_parameters(self, X, random_state):
        n = X.shape[0]
        if self.init_params == "kmeans":
            from .models.cluster import KMeans
            labels = KMeans(n_clusters=self.n_components, n_init=1,
                            random_state=random_state, device="cpu").fit(X).labels_
            resp = np.zeros((n, self.n_components))
            resp[np.arange(n), labels] = 1
        elif self.init_params == "random":
            resp = random_state.rand(n, self.n_components)
            resp /= resp.sum(axis=1)[:, None]
        elif self.init_params == "random_from_data":
            resp = np.zeros((n, self.n_components))
            idx = random_state.choice(n, size=self.n_components, replace=False)
            resp[idx, np.arange(self.n_components)] = 1
        elif self.init_params == "k-means++":
            from .models.cluster._init import kmeans_plusplus
            _, idx = kmeans_plusplus(X, self.n_components, random_state=random_state)
            resp = np.zeros((n, self.n_components))
            resp[np.asarray(idx), np.arange(self.n_components)] = 1
        else:
            raise ValueError("Unimplemented initialization method '%s'" % self.init_params)
        self._initialize(self._t(X), self._t(resp))

    def _initialize(self, X, resp):
        n = X.shape[0]
        w, m, c = _estimate_gaussian_parameters(X, resp, self.reg_covar, self.covariance_type)
        w = w / n
        self._w = w if self.weights_init is None else self._t(self.weights_init)
        self._m = m if self.means_init is None else self._t(self.means_init)
        if self.precisions_init is None:
            self._c = c
            self._pc = _compute_precision_cholesky(c, self.covariance_type)
        else:
            P = self._t(self.precisions_init)
            if self.covariance_type == "full":
                self._pc = torch.linalg.cholesky(P)
            elif self.covariance_type == "tied":
                self._pc = torch.linalg.cholesky(P)
            else:
                self._pc = torch.sqrt(P)

    def _estimate_weighted_log_prob(self, X):
        return _estimate_log_gaussian_prob(X, self._m, self._pc, self.covariance_type) + \
            torch.log(self._w)

    def _e_step(self, X):
        wlp = self._estimate_weighted_log_prob(X)
        lpn = torch.logsumexp(wlp, dim=1)
        return lpn.mean(), wlp - lpn[:, None]

    def _m_step(self, X, log_resp):
        n = X.shape[0]
        w, m, c = _estimate_gaussian_parameters(X, torch.exp(log_resp), self.reg_covar,
                                                self.covariance_type)
        self._w = w / n
        self._m = m
        self._c = c
        self._pc = _compute_precision_cholesky(c, self.covariance_type)

    def _compute_lower_bound(self, log_resp, log_prob_norm):
        return float(log_prob_norm)

    def _get_params(self):
        return (self._w.clone(), self._m.clone(), self._c.clone() if hasattr(self, "_c") else None,
                self._pc.clone())

    def _set_params(self, p):
        self._w, self._m, c, self._pc = p
        if c is not None:
            self._c = c
        self._export()

    def _export(self):
        self.weights_ = self._w.cpu().numpy()
        self.means_ = self._m.cpu().numpy()
        pc = self._pc.cpu().numpy()
        self.precisions_cholesky_ = pc
        ct = self.covariance_type
        if ct == "full":
            self.precisions_ = np.einsum("kij,klj->kil", pc, pc)
        elif ct == "tied":
            self.precisions_ = pc @ pc.T
        else:
            self.precisions_ = pc ** 2
        if hasattr(self, "_c"):
            self.covariances_ = self._c.cpu().numpy()
        else:
            self.covariances_ = (np.linalg.inv(self.precisions_) if ct in ("full", "tied")
                                 else 1.0 / self.precisions_)

    # -------------------------------------------------------------- public
    def fit(self, X, y=None):
        self.fit_predict(X, y)
        return self

    def fit_predict(self, X, y=None):
        X = _dense(X)
        self._check_parameters(X)
        self.n_features_in_ = X.shape[1]
        self._dev = resolve_device(self.device)
        Xt = self._t(X)
        do_init = not (self.warm_start and hasattr(self, "converged_"))
        n_init = self.n_init if do_init else 1
        max_lower_bound = -np.inf
        self.converged_ = False
        random_state = check_random_state(self.random_state)
        best_params, best_n_iter = None, 0
        for init in range(n_init):
            if do_init:
                self._initialize_parameters(X, random_state)
            lower_bound = -np.inf if do_init else self.lower_bound_
            converged = False
            n_iter = 0
            for n_iter in range(1, self.max_iter + 1):
                prev = lower_bound
                lpn, log_resp = self._e_step(Xt)
                self._m_step(Xt, log_resp)
                lower_bound = self._compute_lower_bound(log_resp, lpn)
                if abs(lower_bound - prev) < self.tol:
                    converged = True
                    break
            if lower_bound > max_lower_bound or max_lower_bound == -np.inf:
                max_lower_bound = lower_bound
                best_params = self._get_params()
                best_n_iter = n_iter
                self.converged_ = converged
        if not self.converged_ and self.max_iter > 0:
            warnings.warn("Initialization %d did not converge. Try different init parameters, "
                          "or increase max_iter, tol or check for degenerate data." % (init + 1),
                          ConvergenceWarning)
        self._set_params(best_params)
        self.n_iter_ = best_n_iter
        self.lower_bound_ = max_lower_bound
        _, log_resp = self._e_step(Xt)
        return log_resp.argmax(dim=1).cpu().numpy()

    def _X(self, X):
        check_is_fitted(self, "weights_")
        X = _dense(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError(f"X has {X.shape[1]} features, but GaussianMixture is expecting "
                             f"{self.n_features_in_} features as input.")
        if not hasattr(self, "_w"):
            self._dev = resolve_device(self.device)
            self._w, self._m = self._t(self.weights_), self._t(self.means_)
            self._pc = self._t(self.precisions_cholesky_)
        return self._t(X)

    def score_samples(self, X):
        return torch.logsumexp(self._estimate_weighted_log_prob(self._X(X)), dim=1).cpu().numpy()

    def score(self, X, y=None):
        return float(self.score_samples(X).mean())

    def predict(self, X):
        return self._estimate_weighted_log_prob(self._X(X)).argmax(dim=1).cpu().numpy()

    def predict_proba(self, X):
        _, log_resp = self._e_step(self._X(X))
        return torch.exp(log_resp).cpu().numpy()

    def _n_parameters(self):
        _, d = self.means_.shape
        k = self.n_components
        cov_params = {"full": k * d * (d + 1) / 2.0, "diag": k * d, "tied": d * (d + 1) / 2.0,
                      "spherical": k}[self.covariance_type]
        return int(cov_params + k * d + k - 1)

    def bic(self, X):
        X = _dense(X)
        return -2 * self.score(X) * X.shape[0] + self._n_parameters() * np.log(X.shape[0])

    def aic(self, X):
        return -2 * self.score(X) * _dense(X).shape[0] + 2 * self._n_parameters()

    def sample(self, n_samples=1):
        check_is_fitted(self, "weights_")
        if n_samples < 1:
            raise ValueError("Invalid value for 'n_samples': %d . The sampling requires at least "
                             "one sample." % n_samples)
        rng = check_random_state(self.random_state)
        n_per = rng.multinomial(n_samples, self.weights_)
        if self.covariance_type == "full":
            X = np.vstack([rng.multivariate_normal(m, c, int(s))
                           for m, c, s in zip(self.means_, self.covariances_, n_per)])
        elif self.covariance_type == "tied":
            X = np.vstack([rng.multivariate_normal(m, self.covariances_, int(s))
                           for m, s in zip(self.means_, n_per)])
        else:
            X = np.vstack([m + rng.standard_normal(size=(s, self.means_.shape[1])) * np.sqrt(c)
                           for m, c, s in zip(self.means_, self.covariances_, n_per)])
        y = np.concatenate([np.full(s, j, dtype=int) for j, s in enumerate(n_per)])
        return X, y

    def __getstate__(self):
        st = super().__getstate__()
        for k in ("_w", "_m", "_c", "_pc", "_dev"):
            st.pop(k, None)
        return st


__all__ = ["GaussianMixture", "BayesianGaussianMixture"]


from ._bayesian_mixture import BayesianGaussianMixture  # noqa: E402,F401

from .utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
