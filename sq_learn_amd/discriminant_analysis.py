"""Linear / quadratic discriminant analysis (reference
``sklearn/discriminant_analysis.py``: LDA solvers 'svd' (:437-513),
'lsqr' and 'eigen' with Ledoit-Wolf / fixed shrinkage, transform; QDA with
regularisation).  Dense fp64; the SVDs / eigendecompositions are small
(d x d or n_classes x d)."""

import warnings

import numpy as np
import scipy.linalg
from scipy.special import expit, softmax

from .base import BaseEstimator, ClassifierMixin, TransformerMixin
from .covariance import empirical_covariance, ledoit_wolf, shrunk_covariance
from .utils.validation import check_is_fitted


def _dense(X):
    if hasattr(X, "detach"):
        X = X.detach().cpu().numpy()
    return np.asarray(X, dtype=np.float64)


def _cov(X, shrinkage=None, covariance_estimator=None):
    if covariance_estimator is not None:
        covariance_estimator.fit(X)
        return covariance_estimator.covariance_
    if shrinkage is None:
        return empirical_covariance(X)
    if isinstance(shrinkage, str):
        if shrinkage != "auto":
            raise ValueError("unknown shrinkage parameter")
        sc = X.std(axis=0)
        sc[sc == 0] = 1.0
        Xs = (X - X.mean(axis=0)) / sc
        s = ledoit_wolf(Xs)[0]
        return sc[:, None] * s * sc[None, :]
    if not 0 <= shrinkage <= 1:
        raise ValueError("shrinkage parameter must be between 0 and 1")
    return shrunk_covariance(empirical_covariance(X), shrinkage)


def _class_means(X, y):
    classes, yi = np.unique(y, return_inverse=True)
    means = np.zeros((len(classes), X.shape[1]))
    np.add.at(means, yi, X)
    means /= np.bincount(yi)[:, None]
    return means


def _class_cov(X, y, priors, shrinkage=None, covariance_estimator=None):
    classes = np.unique(y)
    cov = np.zeros((X.shape[1], X.shape[1]))
    for idx, g in enumerate(classes):
        cov += priors[idx] * np.atleast_2d(_cov(X[y == g], shrinkage, covariance_estimator))
    return cov


class LinearDiscriminantAnalysis(ClassifierMixin, TransformerMixin, BaseEstimator):
    def __init__(self, solver="svd", shrinkage=None, priors=None, n_components=None,
                 store_covariance=False, tol=1e-4, covariance_estimator=None):
        self.solver = solver
        self.shrinkage = shrinkage
        self.priors = priors
        self.n_components = n_components
        self.store_covariance = store_covariance
        self.tol = tol
        self.covariance_estimator = covariance_estimator

    def _solve_lsqr(self, X, y, shrinkage, covariance_estimator):
        self.means_ = _class_means(X, y)
        self.covariance_ = _class_cov(X, y, self.priors_, shrinkage, covariance_estimator)
        self.coef_ = np.linalg.lstsq(self.covariance_, self.means_.T, rcond=None)[0].T
        self.intercept_ = -0.5 * np.diag(self.means_ @ self.coef_.T) + np.log(self.priors_)

    def _solve_eigen(self, X, y, shrinkage, covariance_estimator):
        self.means_ = _class_means(X, y)
        self.covariance_ = _class_cov(X, y, self.priors_, shrinkage, covariance_estimator)
        Sw = self.covariance_
        St = _cov(X, shrinkage, covariance_estimator)
        Sb = St - Sw
        evals, evecs = scipy.linalg.eigh(Sb, Sw)
        self.explained_variance_ratio_ = np.sort(evals / np.sum(evals))[::-1][:self._max_components]
        evecs = evecs[:, np.argsort(evals)[::-1]]
        self.scalings_ = evecs
        self.coef_ = self.means_ @ evecs @ evecs.T
        self.intercept_ = -0.5 * np.diag(self.means_ @ self.coef_.T) + np.log(self.priors_)

    def _solve_svd(self, X, y):
        n_samples, n_features = X.shape
        n_classes = len(self.classes_)
        self.means_ = _class_means(X, y)
        if self.store_covariance:
            self.covariance_ = _class_cov(X, y, self.priors_)
        Xc = []
        for idx, group in enumerate(self.classes_):
            Xg = X[y == group]
            Xc.append(Xg - self.means_[idx])
        self.xbar_ = self.priors_ @ self.means_
        Xc = np.concatenate(Xc, axis=0)
        std = Xc.std(axis=0)
        std[std == 0] = 1.0
        fac = 1.0 / (n_samples - n_classes)
        Xs = np.sqrt(fac) * (Xc / std)
        U, S, Vt = scipy.linalg.svd(Xs, full_matrices=False)
        rank = np.sum(S > self.tol)
        scalings = (Vt[:rank] / std).T / S[:rank]
        fac = 1.0 if n_classes == 1 else 1.0 / (n_classes - 1)
        Xm = np.sqrt((n_samples * self.priors_) * fac) * (self.means_ - self.xbar_).T
        Xm = Xm.T @ scalings
        _, S, Vt = scipy.linalg.svd(Xm, full_matrices=False)
        if self._max_components == 0:
            self.explained_variance_ratio_ = np.empty((0,), dtype=S.dtype)
        else:
            self.explained_variance_ratio_ = (S ** 2 / np.sum(S ** 2))[:self._max_components]
        rank = np.sum(S > self.tol * S[0])
        self.scalings_ = scalings @ Vt.T[:, :rank]
        coef = (self.means_ - self.xbar_) @ self.scalings_
        self.intercept_ = -0.5 * np.sum(coef ** 2, axis=1) + np.log(self.priors_)
        self.coef_ = coef @ self.scalings_.T
        self.intercept_ -= self.xbar_ @ self.coef_.T

    def fit(self, X, y):
        X = _dense(X)
        y = np.asarray(y).reshape(-1)
        self.n_features_in_ = X.shape[1]
        self.classes_ = np.unique(y)
        n_samples, _ = X.shape
        n_classes = len(self.classes_)
        if n_samples == n_classes:
            raise ValueError("The number of samples must be more than the number of classes.")
        if self.priors is None:
            _, y_t = np.unique(y, return_inverse=True)
            self.priors_ = np.bincount(y_t) / float(len(y))
        else:
            self.priors_ = np.asarray(self.priors, dtype=np.float64)
        if (self.priors_ < 0).any():
            raise ValueError("priors must be non-negative")
        if not np.isclose(self.priors_.sum(), 1.0):
            warnings.warn("The priors do not sum to 1. Renormalizing", UserWarning)
            self.priors_ = self.priors_ / self.priors_.sum()
        max_components = min(len(self.classes_) - 1, X.shape[1])
        if self.n_components is None:
            self._max_components = max_components
        else:
            if self.n_components > max_components:
                raise ValueError("n_components cannot be larger than min(n_features, "
                                 "n_classes - 1).")
            self._max_components = self.n_components
        if self.solver == "svd":
            if self.shrinkage is not None:
                raise NotImplementedError("shrinkage not supported with 'svd' solver.")
            if self.covariance_estimator is not None:
                raise ValueError("covariance estimator is not supported with svd solver.")
            self._solve_svd(X, y)
        elif self.solver == "lsqr":
            self._solve_lsqr(X, y, self.shrinkage, self.covariance_estimator)
        elif self.solver == "eigen":
            self._solve_eigen(X, y, self.shrinkage, self.covariance_estimator)
        else:
            raise ValueError("unknown solver {} (valid solvers are 'svd', 'lsqr', and 'eigen')."
                             .format(self.solver))
        if self.classes_.size == 2:
            self.coef_ = np.array(self.coef_[1, :] - self.coef_[0, :], ndmin=2)
            self.intercept_ = np.array(self.intercept_[1] - self.intercept_[0], ndmin=1)
        return self

    def transform(self, X):
        if self.solver == "lsqr":
            raise NotImplementedError("transform not implemented for 'lsqr' solver (use 'svd' "
                                      "or 'eigen').")
        check_is_fitted(self)
        X = _dense(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError(f"X has {X.shape[1]} features, but LinearDiscriminantAnalysis is "
                             f"expecting {self.n_features_in_} features as input.")
        if self.solver == "svd":
            Xn = (X - self.xbar_) @ self.scalings_
        else:
            Xn = X @ self.scalings_
        return Xn[:, :self._max_components]

    def decision_function(self, X):
        check_is_fitted(self)
        X = _dense(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError(f"X has {X.shape[1]} features, but LinearDiscriminantAnalysis is "
                             f"expecting {self.n_features_in_} features as input.")
        s = X @ self.coef_.T + self.intercept_
        return s.ravel() if s.shape[1] == 1 else s

    def predict(self, X):
        s = self.decision_function(X)
        idx = (s > 0).astype(int) if s.ndim == 1 else s.argmax(axis=1)
        return self.classes_[idx]

    def predict_proba(self, X):
        d = self.decision_function(X)
        if self.classes_.size == 2:
            p = expit(d)
            return np.vstack([1 - p, p]).T
        return softmax(d, axis=1)

    def predict_log_proba(self, X):
        p = self.predict_proba(X)
        p[p == 0.0] += np.finfo(p.dtype).tiny
        return np.log(p)


class QuadraticDiscriminantAnalysis(ClassifierMixin, BaseEstimator):
    def __init__(self, *, priors=None, reg_param=0.0, store_covariance=False, tol=1.0e-4):
        self.priors = priors
        self.reg_param = reg_param
        self.store_covariance = store_covariance
        self.tol = tol

    def fit(self, X, y):
        X = _dense(X)
        y = np.asarray(y).reshape(-1)
        self.n_features_in_ = X.shape[1]
        self.classes_, y = np.unique(y, return_inverse=True)
        n_samples, n_features = X.shape
        n_classes = len(self.classes_)
        if n_classes < 2:
            raise ValueError("The number of classes has to be greater than one; got %d class"
                             % n_classes)
        self.priors_ = np.bincount(y) / float(n_samples) if self.priors is None else \
            np.asarray(self.priors)
        geo = [self._class_geometry(X[y == c], self.classes_[c]) for c in range(n_classes)]
        self.means_ = np.stack([g[0] for g in geo])
        self.scalings_ = [g[1] for g in geo]
        self.rotations_ = [g[2] for g in geo]
        if self.store_covariance:
            # Sigma_c = R diag(s) R^T of the regularised class covariance
            self.covariance_ = [(R * s) @ R.T for _, s, R in geo]
        return self

    def _class_geometry(self, Xk, label):
        """(mean, eigenvalues, eigenvectors as columns) of one class's
        regularised covariance (1 - reg) Sigma + reg I, from the SVD of the
        centred class rows (eigenvalues in decreasing order)."""
        m = Xk.shape[0]
        if m < 2:
            raise ValueError("y has only 1 sample in class %s, covariance is ill defined."
                             % str(label))
        mu = Xk.mean(axis=0)
        _, sv, Vt = np.linalg.svd(Xk - mu, full_matrices=False)
        if np.count_nonzero(sv > self.tol) < Xk.shape[1]:
            warnings.warn("Variables are collinear")
        ev = sv * sv / (m - 1)
        return mu, ev + self.reg_param * (1.0 - ev), Vt.T

    def _decision_function(self, X):
        check_is_fitted(self)
        X = _dense(X)
        norm2 = []
        for i in range(len(self.classes_)):
            R, S = self.rotations_[i], self.scalings_[i]
            Xm = X - self.means_[i]
            X2 = Xm @ (R * (S ** (-0.5)))
            norm2.append(np.sum(X2 ** 2, axis=1))
        norm2 = np.array(norm2).T
        u = np.asarray([np.sum(np.log(s)) for s in self.scalings_])
        return -0.5 * (norm2 + u) + np.log(self.priors_)

    def decision_function(self, X):
        d = self._decision_function(X)
        if len(self.classes_) == 2:
            return d[:, 1] - d[:, 0]
        return d

    def predict(self, X):
        return self.classes_.take(self._decision_function(X).argmax(1))

    def predict_proba(self, X):
        values = self._decision_function(X)
        likelihood = np.exp(values - values.max(axis=1)[:, None])
        return likelihood / likelihood.sum(axis=1)[:, None]

    def predict_log_proba(self, X):
        return np.log(self.predict_proba(X))


__all__ = ["LinearDiscriminantAnalysis", "QuadraticDiscriminantAnalysis"]
