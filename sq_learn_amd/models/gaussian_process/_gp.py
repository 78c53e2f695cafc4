"""Gaussian-process regression and classification (reference
``gaussian_process/_gpr.py`` and ``_gpc.py``).

* ``GaussianProcessRegressor``: exact GP with Cholesky of K + alpha I,
  hyperparameters by L-BFGS-B on the log marginal likelihood (analytic
  gradient), optional random restarts drawn from the bounds.
* ``GaussianProcessClassifier``: binary Laplace approximation (Rasmussen &
  Williams algorithms 3.1/3.2/5.1) with the reference's 5-term erf
  approximation of the predictive integral; multi-class by one-vs-rest or
  one-vs-one.

The factorisations run in fp64 with host LAPACK: the hyperparameter search
issues many small dependent Cholesky solves, where per-call device launch
latency would dominate for the training-set sizes GPs are used at.
"""

import warnings
from operator import itemgetter

import numpy as np
import scipy.optimize
from scipy.linalg import cho_solve, cholesky, solve, solve_triangular
from scipy.special import erf, expit

from ...base import BaseEstimator, ClassifierMixin, MultiOutputMixin, RegressorMixin
from ...exceptions import ConvergenceWarning
from ...utils.validation import check_is_fitted, check_random_state
from .kernels import RBF, CompoundKernel
from .kernels import ConstantKernel as C

LAMBDAS = np.array([0.41, 0.4, 0.37, 0.44, 0.39])[:, np.newaxis]
COEFS = np.array([-1854.8214151, 3516.89893646, 221.29346712, 128.12323805,
                  -2010.49422654])[:, np.newaxis]


def _arr(X):
    if hasattr(X, "detach"):
        X = X.detach().cpu().numpy()
    return np.asarray(X, dtype=np.float64)


def _default_kernel():
    return C(1.0, constant_value_bounds="fixed") * RBF(1.0, length_scale_bounds="fixed")


def _optimize(est, obj, theta0, bounds):
    if est.optimizer == "fmin_l_bfgs_b":
        res = scipy.optimize.minimize(obj, theta0, method="L-BFGS-B", jac=True, bounds=bounds)
        if res.status != 0:
            warnings.warn("lbfgs failed to converge (status=%d): %s" % (res.status, res.message),
                          ConvergenceWarning)
        return res.x, res.fun
    if callable(est.optimizer):
        return est.optimizer(obj, theta0, bounds=bounds)
    raise ValueError("Unknown optimizer %s." % est.optimizer)


def _fit_hyper(est, kernel, lml):
    def obj(theta, eval_gradient=True):
        if eval_gradient:
            v, g = lml(theta, eval_gradient=True, clone_kernel=False)
            return -v, -g
        return -lml(theta, clone_kernel=False)
    optima = [_optimize(est, obj, kernel.theta, kernel.bounds)]
    if est.n_restarts_optimizer > 0:
        if not np.isfinite(kernel.bounds).all():
            raise ValueError("Multiple optimizer restarts (n_restarts_optimizer>0) requires that "
                             "all bounds are finite.")
        b = kernel.bounds
        for _ in range(est.n_restarts_optimizer):
            optima.append(_optimize(est, obj, est._rng.uniform(b[:, 0], b[:, 1]), b))
    vals = list(map(itemgetter(1), optima))
    kernel.theta = optima[int(np.argmin(vals))][0]
    kernel._check_bounds_params()
    return -np.min(vals)


class GaussianProcessRegressor(MultiOutputMixin, RegressorMixin, BaseEstimator):

    def _more_tags(self):
        return {"requires_fit": False}

    def __init__(self, kernel=None, *, alpha=1e-10, optimizer="fmin_l_bfgs_b",
                 n_restarts_optimizer=0, normalize_y=False, copy_X_train=True,
                 random_state=None):
        self.kernel = kernel
        self.alpha = alpha
        self.optimizer = optimizer
        self.n_restarts_optimizer = n_restarts_optimizer
        self.normalize_y = normalize_y
        self.copy_X_train = copy_X_train
        self.random_state = random_state

    def fit(self, X, y):
        self.kernel_ = _default_kernel() if self.kernel is None else clone_kernel(self.kernel)
        self._rng = check_random_state(self.random_state)
        X = _arr(X) if self.kernel_.requires_vector_input else X
        y = _arr(y)
        if self.kernel_.requires_vector_input:
            self.n_features_in_ = X.shape[1]
        if self.normalize_y:
            self._y_train_mean = np.mean(y, axis=0)
            std = np.std(y, axis=0)
            self._y_train_std = np.where(std == 0.0, 1.0, std) if np.ndim(std) else \
                (1.0 if std == 0.0 else std)
            y = (y - self._y_train_mean) / self._y_train_std
        else:
            self._y_train_mean = np.zeros(1)
            self._y_train_std = 1
        if np.iterable(self.alpha) and np.asarray(self.alpha).shape[0] != y.shape[0]:
            if np.asarray(self.alpha).shape[0] == 1:
                self.alpha = self.alpha[0]
            else:
                raise ValueError("alpha must be a scalar or an array with same number of entries "
                                 "as y. (%d != %d)" % (np.asarray(self.alpha).shape[0],
                                                        y.shape[0]))
        self.X_train_ = np.copy(X) if self.copy_X_train else X
        self.y_train_ = np.copy(y) if self.copy_X_train else y
        if self.optimizer is not None and self.kernel_.n_dims > 0:
            self.log_marginal_likelihood_value_ = _fit_hyper(self, self.kernel_,
                                                             self.log_marginal_likelihood)
        else:
            self.log_marginal_likelihood_value_ = self.log_marginal_likelihood(
                self.kernel_.theta, clone_kernel=False)
        K = self.kernel_(self.X_train_)
        K[np.diag_indices_from(K)] += self.alpha
        try:
            self.L_ = cholesky(K, lower=True, check_finite=False)
        except np.linalg.LinAlgError as exc:
            exc.args = ("The kernel, %s, is not returning a positive definite matrix. Try "
                        "gradually increasing the 'alpha' parameter of your "
                        "GaussianProcessRegressor estimator." % self.kernel_,) + exc.args
            raise
        self.alpha_ = cho_solve((self.L_, True), self.y_train_, check_finite=False)
        return self

    def predict(self, X, return_std=False, return_cov=False):
        if return_std and return_cov:
            raise RuntimeError("At most one of return_std or return_cov can be requested.")
        if self.kernel is None or self.kernel.requires_vector_input:
            X = _arr(X)
        if not hasattr(self, "X_train_"):
            kernel = _default_kernel() if self.kernel is None else self.kernel
            mean = np.zeros(X.shape[0])
            if return_cov:
                return mean, kernel(X)
            if return_std:
                return mean, np.sqrt(kernel.diag(X))
            return mean
        Kt = self.kernel_(X, self.X_train_)
        mean = Kt @ self.alpha_
        mean = self._y_train_std * mean + self._y_train_mean
        if return_cov:
            v = cho_solve((self.L_, True), Kt.T)
            cov = self.kernel_(X) - Kt @ v
            return mean, cov * np.asarray(self._y_train_std) ** 2
        if return_std:
            Linv = solve_triangular(self.L_.T, np.eye(self.L_.shape[0]))
            self._K_inv = Linv @ Linv.T
            var = self.kernel_.diag(X).astype(np.float64)
            var -= np.einsum("ij,ij->i", Kt @ self._K_inv, Kt)
            neg = var < 0
            if np.any(neg):
                warnings.warn("Predicted variances smaller than 0. Setting those variances to "
                              "0.")
                var[neg] = 0.0
            var = var * np.asarray(self._y_train_std) ** 2 if np.ndim(self._y_train_std) == 0 \
                else var[:, None] * self._y_train_std ** 2
            return mean, np.sqrt(var)
        return mean

    def sample_y(self, X, n_samples=1, random_state=0):
        rng = check_random_state(random_state)
        mean, cov = self.predict(X, return_cov=True)
        if mean.ndim == 1:
            return rng.multivariate_normal(mean, cov, n_samples).T
        return np.hstack([rng.multivariate_normal(mean[:, i], cov, n_samples).T[:, np.newaxis]
                          for i in range(mean.shape[1])])

    def log_marginal_likelihood(self, theta=None, eval_gradient=False, clone_kernel=True):
        if theta is None:
            if eval_gradient:
                raise ValueError("Gradient can only be evaluated for theta!=None")
            return self.log_marginal_likelihood_value_
        if clone_kernel:
            kernel = self.kernel_.clone_with_theta(theta)
        else:
            kernel = self.kernel_
            kernel.theta = theta
        if eval_gradient:
            K, Kg = kernel(self.X_train_, eval_gradient=True)
        else:
            K = kernel(self.X_train_)
        K[np.diag_indices_from(K)] += self.alpha
        try:
            L = cholesky(K, lower=True, check_finite=False)
        except np.linalg.LinAlgError:
            return (-np.inf, np.zeros_like(theta)) if eval_gradient else -np.inf
        y = self.y_train_
        if y.ndim == 1:
            y = y[:, np.newaxis]
        a = cho_solve((L, True), y, check_finite=False)
        lld = -0.5 * np.einsum("ik,ik->k", y, a)
        lld -= np.log(np.diag(L)).sum()
        lld -= K.shape[0] / 2 * np.log(2 * np.pi)
        ll = lld.sum(axis=-1)
        if not eval_gradient:
            return ll
        inner = np.einsum("ik,jk->ijk", a, a)
        Kinv = cho_solve((L, True), np.eye(K.shape[0]), check_finite=False)
        inner -= Kinv[..., np.newaxis]
        g = 0.5 * np.einsum("ijl,jik->kl", inner, Kg)
        return ll, g.sum(axis=-1)


def clone_kernel(k):
    from copy import deepcopy
    return deepcopy(k)


class _BinaryGPCLaplace(BaseEstimator):
    def __init__(self, kernel=None, *, optimizer="fmin_l_bfgs_b", n_restarts_optimizer=0,
                 max_iter_predict=100, warm_start=False, copy_X_train=True, random_state=None):
        self.kernel = kernel
        self.optimizer = optimizer
        self.n_restarts_optimizer = n_restarts_optimizer
        self.max_iter_predict = max_iter_predict
        self.warm_start = warm_start
        self.copy_X_train = copy_X_train
        self.random_state = random_state

    def fit(self, X, y):
        from ...preprocessing import LabelEncoder
        self.kernel_ = _default_kernel() if self.kernel is None else clone_kernel(self.kernel)
        self._rng = check_random_state(self.random_state)
        self.X_train_ = np.copy(X) if self.copy_X_train else X
        le = LabelEncoder()
        self.y_train_ = le.fit_transform(y)
        self.classes_ = le.classes_
        if self.classes_.size > 2:
            raise ValueError("%s supports only binary classification. y contains classes %s"
                             % (self.__class__.__name__, self.classes_))
        if self.classes_.size == 1:
            raise ValueError("{0:s} requires 2 classes; got {1:d} class"
                             .format(self.__class__.__name__, self.classes_.size))
        if self.optimizer is not None and self.kernel_.n_dims > 0:
            self.log_marginal_likelihood_value_ = _fit_hyper(self, self.kernel_,
                                                             self.log_marginal_likelihood)
        else:
            self.log_marginal_likelihood_value_ = self.log_marginal_likelihood(self.kernel_.theta)
        K = self.kernel_(self.X_train_)
        _, (self.pi_, self.W_sr_, self.L_, _, _) = self._posterior_mode(K, True)
        return self

    def predict(self, X):
        check_is_fitted(self)
        f = self.kernel_(self.X_train_, X).T @ (self.y_train_ - self.pi_)
        return np.where(f > 0, self.classes_[1], self.classes_[0])

    def predict_proba(self, X):
        check_is_fitted(self)
        Ks = self.kernel_(self.X_train_, X)
        f = Ks.T @ (self.y_train_ - self.pi_)
        v = solve(self.L_, self.W_sr_[:, np.newaxis] * Ks)
        var = self.kernel_.diag(X) - np.einsum("ij,ij->j", v, v)
        alpha = 1 / (2 * var)
        g = LAMBDAS * f
        integ = np.sqrt(np.pi / alpha) * erf(g * np.sqrt(alpha / (alpha + LAMBDAS ** 2))) \
            / (2 * np.sqrt(var * 2 * np.pi))
        pi = (COEFS * integ).sum(axis=0) + 0.5 * COEFS.sum()
        return np.vstack((1 - pi, pi)).T

    def log_marginal_likelihood(self, theta=None, eval_gradient=False, clone_kernel=True):
        if theta is None:
            if eval_gradient:
                raise ValueError("Gradient can only be evaluated for theta!=None")
            return self.log_marginal_likelihood_value_
        if clone_kernel:
            kernel = self.kernel_.clone_with_theta(theta)
        else:
            kernel = self.kernel_
            kernel.theta = theta
        if eval_gradient:
            K, Kg = kernel(self.X_train_, eval_gradient=True)
        else:
            K = kernel(self.X_train_)
        Z, (pi, W_sr, L, b, a) = self._posterior_mode(K, True)
        if not eval_gradient:
            return Z
        dZ = np.empty(theta.shape[0])
        R = W_sr[:, np.newaxis] * cho_solve((L, True), np.diag(W_sr))
        Cm = solve(L, W_sr[:, np.newaxis] * K)
        s2 = -0.5 * (np.diag(K) - np.einsum("ij, ij -> j", Cm, Cm)) * (pi * (1 - pi) * (1 - 2 * pi))
        for j in range(dZ.shape[0]):
            Cj = Kg[:, :, j]
            s1 = 0.5 * a.T @ Cj @ a - 0.5 * R.T.ravel() @ Cj.ravel()
            bj = Cj @ (self.y_train_ - pi)
            s3 = bj - K @ (R @ bj)
            dZ[j] = s1 + s2.T @ s3
        return Z, dZ

    def _posterior_mode(self, K, return_temporaries=False):
        if self.warm_start and hasattr(self, "f_cached") and \
                self.f_cached.shape == self.y_train_.shape:
            f = self.f_cached
        else:
            f = np.zeros_like(self.y_train_, dtype=np.float64)
        lml = -np.inf
        for _ in range(self.max_iter_predict):
            pi = expit(f)
            W = pi * (1 - pi)
            W_sr = np.sqrt(W)
            W_sr_K = W_sr[:, np.newaxis] * K
            B = np.eye(W.shape[0]) + W_sr_K * W_sr
            L = cholesky(B, lower=True)
            b = W * f + (self.y_train_ - pi)
            a = b - W_sr * cho_solve((L, True), W_sr_K @ b)
            f = K @ a
            new = -0.5 * a.T @ f - np.log1p(np.exp(-(self.y_train_ * 2 - 1) * f)).sum() \
                - np.log(np.diag(L)).sum()
            if new - lml < 1e-10:
                break
            lml = new
        self.f_cached = f
        return (lml, (pi, W_sr, L, b, a)) if return_temporaries else lml


class GaussianProcessClassifier(ClassifierMixin, BaseEstimator):
    def __init__(self, kernel=None, *, optimizer="fmin_l_bfgs_b", n_restarts_optimizer=0,
                 max_iter_predict=100, warm_start=False, copy_X_train=True, random_state=None,
                 multi_class="one_vs_rest", n_jobs=None):
        self.kernel = kernel
        self.optimizer = optimizer
        self.n_restarts_optimizer = n_restarts_optimizer
        self.max_iter_predict = max_iter_predict
        self.warm_start = warm_start
        self.copy_X_train = copy_X_train
        self.random_state = random_state
        self.multi_class = multi_class
        self.n_jobs = n_jobs

    def fit(self, X, y):
        from ...multiclass import OneVsOneClassifier, OneVsRestClassifier
        if self.kernel is None or self.kernel.requires_vector_input:
            X = _arr(X)
            self.n_features_in_ = X.shape[1]
        y = np.asarray(y)
        base = _BinaryGPCLaplace(kernel=self.kernel, optimizer=self.optimizer,
                                 n_restarts_optimizer=self.n_restarts_optimizer,
                                 max_iter_predict=self.max_iter_predict,
                                 warm_start=self.warm_start, copy_X_train=self.copy_X_train,
                                 random_state=self.random_state)
        self.classes_ = np.unique(y)
        self.n_classes_ = self.classes_.size
        if self.n_classes_ == 1:
            raise ValueError("GaussianProcessClassifier requires 2 or more distinct classes; got "
                             "%d class (only class %s is present)"
                             % (self.n_classes_, self.classes_[0]))
        if self.n_classes_ > 2:
            if self.multi_class == "one_vs_rest":
                base = OneVsRestClassifier(base, n_jobs=self.n_jobs)
            elif self.multi_class == "one_vs_one":
                base = OneVsOneClassifier(base, n_jobs=self.n_jobs)
            else:
                raise ValueError("Unknown multi-class mode %s" % self.multi_class)
        self.base_estimator_ = base.fit(X, y)
        if self.n_classes_ > 2:
            self.log_marginal_likelihood_value_ = np.mean(
                [e.log_marginal_likelihood() for e in self.base_estimator_.estimators_])
        else:
            self.log_marginal_likelihood_value_ = self.base_estimator_.log_marginal_likelihood()
        return self

    def predict(self, X):
        check_is_fitted(self)
        if self.kernel is None or self.kernel.requires_vector_input:
            X = _arr(X)
        return self.base_estimator_.predict(X)

    def predict_proba(self, X):
        check_is_fitted(self)
        if self.n_classes_ > 2 and self.multi_class == "one_vs_one":
            raise ValueError("one_vs_one multi-class mode does not support predicting probability "
                             "estimates. Use one_vs_rest mode instead.")
        if self.kernel is None or self.kernel.requires_vector_input:
            X = _arr(X)
        return self.base_estimator_.predict_proba(X)

    @property
    def kernel_(self):
        if self.n_classes_ == 2:
            return self.base_estimator_.kernel_
        return CompoundKernel([e.kernel_ for e in self.base_estimator_.estimators_])

    def log_marginal_likelihood(self, theta=None, eval_gradient=False, clone_kernel=True):
        check_is_fitted(self)
        if theta is None:
            if eval_gradient:
                raise ValueError("Gradient can only be evaluated for theta!=None")
            return self.log_marginal_likelihood_value_
        theta = np.asarray(theta)
        if self.n_classes_ == 2:
            return self.base_estimator_.log_marginal_likelihood(theta, eval_gradient,
                                                                clone_kernel=clone_kernel)
        if eval_gradient:
            raise NotImplementedError("Gradient of log-marginal-likelihood not implemented for "
                                      "multi-class GPC.")
        ests = self.base_estimator_.estimators_
        nk = ests[0].kernel_.n_dims
        if theta.shape[0] == nk:
            return np.mean([e.log_marginal_likelihood(theta, clone_kernel=clone_kernel)
                            for e in ests])
        if theta.shape[0] == nk * self.classes_.shape[0]:
            return np.mean([e.log_marginal_likelihood(theta[nk * i:nk * (i + 1)],
                                                      clone_kernel=clone_kernel)
                            for i, e in enumerate(ests)])
        raise ValueError("Shape of theta must be either %d or %d. Obtained theta with shape %d."
                         % (nk, nk * self.classes_.shape[0], theta.shape[0]))


__all__ = ["GaussianProcessRegressor", "GaussianProcessClassifier"]
