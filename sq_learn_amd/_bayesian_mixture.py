"""Variational Bayesian Gaussian mixture (reference
``mixture/_bayesian_mixture.py``).

Shares the EM driver and the device E-step of ``GaussianMixture``: the
responsibilities and the sufficient statistics (n_k, x_k, S_k) are device
GEMMs over the samples; the variational updates of the Dirichlet(-process)
weights, Gaussian-Wishart means / precisions and the evidence lower bound act
on k x d(x d) parameters and run on the host in fp64."""

import math

import numpy as np
import torch
from scipy.special import betaln, digamma, gammaln

from .mixture import (GaussianMixture, _compute_precision_cholesky,
                      _estimate_gaussian_parameters, _estimate_log_gaussian_prob,
                      _log_det_cholesky)


def _log_dirichlet_norm(c):
    return gammaln(np.sum(c)) - np.sum(gammaln(c))


def _log_wishart_norm(dof, log_det_chol, d):
    return -(dof * log_det_chol + dof * d * 0.5 * math.log(2.0)
             + np.sum(gammaln(0.5 * (dof - np.arange(d)[:, None])), 0))


class BayesianGaussianMixture(GaussianMixture):
    """Gaussian mixture fitted by variational inference with a Dirichlet
    process (stick-breaking) or Dirichlet distribution prior on the
    weights."""

    def __init__(self, *, n_components=1, covariance_type="full", tol=1e-3, reg_covar=1e-6,
                 max_iter=100, n_init=1, init_params="kmeans",
                 weight_concentration_prior_type="dirichlet_process",
                 weight_concentration_prior=None, mean_precision_prior=None, mean_prior=None,
                 degrees_of_freedom_prior=None, covariance_prior=None, random_state=None,
                 warm_start=False, verbose=0, verbose_interval=10, device=None):
        self.n_components = n_components
        self.covariance_type = covariance_type
        self.tol = tol
        self.reg_covar = reg_covar
        self.max_iter = max_iter
        self.n_init = n_init
        self.init_params = init_params
        self.weight_concentration_prior_type = weight_concentration_prior_type
        self.weight_concentration_prior = weight_concentration_prior
        self.mean_precision_prior = mean_precision_prior
        self.mean_prior = mean_prior
        self.degrees_of_freedom_prior = degrees_of_freedom_prior
        self.covariance_prior = covariance_prior
        self.random_state = random_state
        self.warm_start = warm_start
        self.verbose = verbose
        self.verbose_interval = verbose_interval
        self.device = device

    # the GaussianMixture initialiser reads these
    weights_init = means_init = precisions_init = None

    def _check_parameters(self, X):
        super()._check_parameters(X)
        d = X.shape[1]
        if self.weight_concentration_prior_type not in ("dirichlet_process",
                                                        "dirichlet_distribution"):
            raise ValueError("Invalid value for 'weight_concentration_prior_type': %s "
                             "'weight_concentration_prior_type' should be in "
                             "['dirichlet_process', 'dirichlet_distribution']"
                             % self.weight_concentration_prior_type)
        if self.weight_concentration_prior is None:
            self.weight_concentration_prior_ = 1.0 / self.n_components
        elif self.weight_concentration_prior > 0.0:
            self.weight_concentration_prior_ = self.weight_concentration_prior
        else:
            raise ValueError("The parameter 'weight_concentration_prior' should be greater than "
                             "0., but got %.3f." % self.weight_concentration_prior)
        if self.mean_precision_prior is None:
            self.mean_precision_prior_ = 1.0
        elif self.mean_precision_prior > 0.0:
            self.mean_precision_prior_ = self.mean_precision_prior
        else:
            raise ValueError("The parameter 'mean_precision_prior' should be greater than 0., "
                             "but got %.3f." % self.mean_precision_prior)
        self.mean_prior_ = X.mean(axis=0) if self.mean_prior is None else \
            np.asarray(self.mean_prior, dtype=np.float64).reshape(d)
        if self.degrees_of_freedom_prior is None:
            self.degrees_of_freedom_prior_ = d
        elif self.degrees_of_freedom_prior > d - 1.0:
            self.degrees_of_freedom_prior_ = self.degrees_of_freedom_prior
        else:
            raise ValueError("The parameter 'degrees_of_freedom_prior' should be greater than "
                             "%d, but got %.3f." % (d - 1, self.degrees_of_freedom_prior))
        ct = self.covariance_type
        if self.covariance_prior is None:
            self.covariance_prior_ = {
                "full": np.atleast_2d(np.cov(X.T)), "tied": np.atleast_2d(np.cov(X.T)),
                "diag": np.var(X, axis=0, ddof=1),
                "spherical": np.var(X, axis=0, ddof=1).mean()}[ct]
        elif ct in ("full", "tied"):
            self.covariance_prior_ = np.asarray(self.covariance_prior, dtype=np.float64)
        elif ct == "diag":
            self.covariance_prior_ = np.asarray(self.covariance_prior, dtype=np.float64)
            if np.any(self.covariance_prior_ <= 0):
                raise ValueError("'covariance_prior' should be positive")
        else:
            if self.covariance_prior <= 0.0:
                raise ValueError("The parameter 'spherical covariance_prior' should be greater "
                                 "than 0., but got %.3f." % self.covariance_prior)
            self.covariance_prior_ = float(self.covariance_prior)

    # ----------------------------------------------------------- updates
    def _update(self, nk, xk, sk):
        nk, xk, sk = (t.cpu().numpy() for t in (nk, xk, sk))
        K = self.n_components
        if self.weight_concentration_prior_type == "dirichlet_process":
            self.weight_concentration_ = (
                1.0 + nk, self.weight_concentration_prior_ + np.hstack(
                    (np.cumsum(nk[::-1])[-2::-1], 0)))
        else:
            self.weight_concentration_ = self.weight_concentration_prior_ + nk
        self.mean_precision_ = self.mean_precision_prior_ + nk
        self.means_ = (self.mean_precision_prior_ * self.mean_prior_ + nk[:, None] * xk) / \
            self.mean_precision_[:, None]
        diff = xk - self.mean_prior_
        ct = self.covariance_type
        if ct == "full":
            self.degrees_of_freedom_ = self.degrees_of_freedom_prior_ + nk
            cov = (self.covariance_prior_[None] + nk[:, None, None] * sk
                   + (nk * self.mean_precision_prior_ / self.mean_precision_)[:, None, None]
                   * np.einsum("ki,kj->kij", diff, diff))
            cov /= self.degrees_of_freedom_[:, None, None]
        elif ct == "tied":
            self.degrees_of_freedom_ = self.degrees_of_freedom_prior_ + nk.sum() / K
            cov = (self.covariance_prior_ + sk * nk.sum() / K + self.mean_precision_prior_ / K
                   * np.dot((nk / self.mean_precision_) * diff.T, diff))
            cov /= self.degrees_of_freedom_
        elif ct == "diag":
            self.degrees_of_freedom_ = self.degrees_of_freedom_prior_ + nk
            cov = self.covariance_prior_ + nk[:, None] * (
                sk + (self.mean_precision_prior_ / self.mean_precision_)[:, None] * diff ** 2)
            cov /= self.degrees_of_freedom_[:, None]
        else:
            self.degrees_of_freedom_ = self.degrees_of_freedom_prior_ + nk
            cov = self.covariance_prior_ + nk * (
                sk + self.mean_precision_prior_ / self.mean_precision_ * np.mean(diff ** 2, 1))
            cov /= self.degrees_of_freedom_
        self.covariances_ = cov
        self._c = self._t(cov)
        self._pc = _compute_precision_cholesky(self._c, ct)
        self._m = self._t(self.means_)

    def _initialize(self, X, resp):
        self._update(*_estimate_gaussian_parameters(X, resp, self.reg_covar,
                                                    self.covariance_type))

    def _m_step(self, X, log_resp):
        self._update(*_estimate_gaussian_parameters(X, torch.exp(log_resp), self.reg_covar,
                                                    self.covariance_type))

    def _log_weights(self):
        if self.weight_concentration_prior_type == "dirichlet_process":
            a, b = self.weight_concentration_
            ds = digamma(a + b)
            return digamma(a) - ds + np.hstack((0, np.cumsum(digamma(b) - ds)[:-1]))
        c = self.weight_concentration_
        return digamma(c) - digamma(np.sum(c))

    def _estimate_weighted_log_prob(self, X):
        d = X.shape[1]
        dof = np.asarray(self.degrees_of_freedom_, dtype=np.float64)
        log_lambda = d * np.log(2.0) + np.sum(digamma(0.5 * (dof - np.arange(d)[:, None])), 0)
        extra = -0.5 * d * np.log(dof) + 0.5 * (log_lambda - d / self.mean_precision_)
        return (_estimate_log_gaussian_prob(X, self._m, self._pc, self.covariance_type)
                + self._t(np.asarray(extra + self._log_weights())))

    def _compute_lower_bound(self, log_resp, log_prob_norm):
        d = self.mean_prior_.shape[0]
        pc = self._pc
        ldc = _log_det_cholesky(pc, self.covariance_type, d).cpu().numpy() - \
            0.5 * d * np.log(self.degrees_of_freedom_)
        if self.covariance_type == "tied":
            log_wishart = self.n_components * np.float64(
                _log_wishart_norm(self.degrees_of_freedom_, ldc, d))
        else:
            log_wishart = np.sum(_log_wishart_norm(self.degrees_of_freedom_, ldc, d))
        if self.weight_concentration_prior_type == "dirichlet_process":
            log_norm_w = -np.sum(betaln(*self.weight_concentration_))
        else:
            log_norm_w = _log_dirichlet_norm(self.weight_concentration_)
        ent = float((torch.exp(log_resp) * log_resp).sum())
        return (-ent - float(log_wishart) - float(log_norm_w)
                - 0.5 * d * float(np.sum(np.log(self.mean_precision_))))

    # --------------------------------------------------------- parameters
    def _get_params(self):
        wc = self.weight_concentration_
        wc = tuple(np.copy(w) for w in wc) if isinstance(wc, tuple) else np.copy(wc)
        return (wc, np.copy(self.mean_precision_), np.copy(self.means_),
                np.copy(self.degrees_of_freedom_), np.copy(self.covariances_), self._pc.clone())

    def _set_params(self, p):
        (self.weight_concentration_, self.mean_precision_, self.means_,
         self.degrees_of_freedom_, self.covariances_, self._pc) = p
        if self.weight_concentration_prior_type == "dirichlet_process":
            a, b = self.weight_concentration_
            s = a + b
            w = a / s * np.hstack((1, np.cumprod((b / s)[:-1])))
            self.weights_ = w / np.sum(w)
        else:
            self.weights_ = self.weight_concentration_ / np.sum(self.weight_concentration_)
        self._m = self._t(self.means_)
        self._c = self._t(self.covariances_)
        pc = self._pc.cpu().numpy()
        self.precisions_cholesky_ = pc
        if self.covariance_type == "full":
            self.precisions_ = np.einsum("kij,klj->kil", pc, pc)
        elif self.covariance_type == "tied":
            self.precisions_ = pc @ pc.T
        else:
            self.precisions_ = pc ** 2

    def _X(self, X):
        Xt = super()._X(X)
        if not hasattr(self, "_pc") or self._pc is None:
            self._pc = self._t(self.precisions_cholesky_)
        self._m = self._t(self.means_)
        return Xt

    def _n_parameters(self):
        raise AttributeError("BayesianGaussianMixture has no information criteria")

    def bic(self, X):
        raise AttributeError("'BayesianGaussianMixture' object has no attribute 'bic'")

    def aic(self, X):
        raise AttributeError("'BayesianGaussianMixture' object has no attribute 'aic'")
