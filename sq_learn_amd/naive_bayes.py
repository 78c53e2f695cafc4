"""Naive Bayes (reference ``sklearn/naive_bayes.py``: GaussianNB with
incremental Chan variance updates, MultinomialNB, ComplementNB, BernoulliNB,
CategoricalNB; partial_fit for all)."""

import warnings

import numpy as np
from scipy.special import logsumexp

from .base import BaseEstimator, ClassifierMixin
from .preprocessing import LabelBinarizer
from .utils.validation import check_is_fitted


def _dense(X):
    if hasattr(X, "detach"):
        X = X.detach().cpu().numpy()
    if hasattr(X, "toarray"):
        X = X.toarray()
    return np.asarray(X, dtype=np.float64)


class _BaseNB(ClassifierMixin, BaseEstimator):
    def predict_joint_log_proba(self, X):
        check_is_fitted(self)
        return self._joint_log_likelihood(self._check_X(X))

    def _check_X(self, X):
        X = _dense(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError(f"X has {X.shape[1]} features, but {type(self).__name__} is "
                             f"expecting {self.n_features_in_} features as input.")
        return X

    def predict(self, X):
        jll = self.predict_joint_log_proba(X)
        return self.classes_[np.argmax(jll, axis=1)]

    def predict_log_proba(self, X):
        jll = self.predict_joint_log_proba(X)
        return jll - logsumexp(jll, axis=1)[:, None]

    def predict_proba(self, X):
        return np.exp(self.predict_log_proba(X))


class GaussianNB(_BaseNB):
    def __init__(self, *, priors=None, var_smoothing=1e-9):
        self.priors = priors
        self.var_smoothing = var_smoothing

    def fit(self, X, y, sample_weight=None):
        X = _dense(X)
        self.n_features_in_ = X.shape[1]
        return self._partial_fit(X, y, np.unique(y), _refit=True, sample_weight=sample_weight)

    def partial_fit(self, X, y, classes=None, sample_weight=None):
        return self._partial_fit(_dense(X), y, classes, _refit=False,
                                 sample_weight=sample_weight)

    @staticmethod
    def _update_mean_variance(n_past, mu, var, X, sample_weight=None):
        if X.shape[0] == 0:
            return mu, var
        if sample_weight is not None:
            n_new = float(sample_weight.sum())
            new_mu = np.average(X, axis=0, weights=sample_weight)
            new_var = np.average((X - new_mu) ** 2, axis=0, weights=sample_weight)
        else:
            n_new = X.shape[0]
            new_var = np.var(X, axis=0)
            new_mu = np.mean(X, axis=0)
        if n_past == 0:
            return new_mu, new_var
        n_total = float(n_past + n_new)
        total_mu = (n_new * new_mu + n_past * mu) / n_total
        old_ssd = n_past * var
        new_ssd = n_new * new_var
        total_ssd = old_ssd + new_ssd + (n_new * n_past / n_total) * (mu - new_mu) ** 2
        return total_mu, total_ssd / n_total

    def _partial_fit(self, X, y, classes=None, _refit=False, sample_weight=None):
        y = np.asarray(y).reshape(-1)
        if sample_weight is not None:
            sample_weight = np.asarray(sample_weight, dtype=np.float64)
        self.epsilon_ = self.var_smoothing * np.var(X, axis=0).max()
        first = _refit or not hasattr(self, "classes_")
        if first:
            self.classes_ = np.asarray(classes) if classes is not None else np.unique(y)
            self.n_features_in_ = X.shape[1]
            n_cls = len(self.classes_)
            self.theta_ = np.zeros((n_cls, X.shape[1]))
            self.var_ = np.zeros((n_cls, X.shape[1]))
            self.class_count_ = np.zeros(n_cls)
            if self.priors is not None:
                priors = np.asarray(self.priors)
                if len(priors) != n_cls:
                    raise ValueError("Number of priors must match number of classes.")
                if not np.isclose(priors.sum(), 1.0):
                    raise ValueError("The sum of the priors should be 1.")
                if (priors < 0).any():
                    raise ValueError("Priors must be non-negative.")
                self.class_prior_ = priors
            else:
                self.class_prior_ = np.zeros(n_cls)
        else:
            if X.shape[1] != self.theta_.shape[1]:
                raise ValueError("Number of features %d does not match previous data %d."
                                 % (X.shape[1], self.theta_.shape[1]))
            self.var_[:, :] -= self.epsilon_
        unique_y = np.unique(y)
        if not np.all(np.isin(unique_y, self.classes_)):
            raise ValueError("The target label(s) %s in y do not exist in the initial classes %s"
                             % (unique_y[~np.isin(unique_y, self.classes_)], self.classes_))
        for yi in unique_y:
            i = int(np.searchsorted(self.classes_, yi))
            m = y == yi
            Xi = X[m]
            sw = sample_weight[m] if sample_weight is not None else None
            N_i = sw.sum() if sw is not None else Xi.shape[0]
            self.theta_[i], self.var_[i] = self._update_mean_variance(
                self.class_count_[i], self.theta_[i], self.var_[i], Xi, sw)
            self.class_count_[i] += N_i
        self.var_[:, :] += self.epsilon_
        if self.priors is None:
            self.class_prior_ = self.class_count_ / self.class_count_.sum()
        return self

    @property
    def sigma_(self):
        return self.var_

    def _joint_log_likelihood(self, X):
        jll = []
        for i in range(len(self.classes_)):
            jointi = np.log(self.class_prior_[i])
            n_ij = -0.5 * np.sum(np.log(2.0 * np.pi * self.var_[i]))
            n_ij -= 0.5 * np.sum(((X - self.theta_[i]) ** 2) / self.var_[i], 1)
            jll.append(jointi + n_ij)
        return np.array(jll).T


class _BaseDiscreteNB(_BaseNB):
    def _check_alpha(self):
        alpha = np.asarray(self.alpha, dtype=np.float64) if not np.isscalar(self.alpha) \
            else self.alpha
        if np.min(alpha) < 0:
            raise ValueError("Smoothing parameter alpha = %.1e. alpha should be > 0."
                             % np.min(alpha))
        if np.min(alpha) < 1e-10:
            warnings.warn("alpha too small will result in numeric errors, setting alpha = %.1e"
                          % 1e-10)
            return np.maximum(alpha, 1e-10)
        return alpha

    def _update_class_log_prior(self, class_prior=None):
        n_cls = len(self.classes_)
        if class_prior is not None:
            if len(class_prior) != n_cls:
                raise ValueError("Number of priors must match number of classes.")
            self.class_log_prior_ = np.log(class_prior)
        elif self.fit_prior:
            with warnings.catch_warnings():
                warnings.simplefilter("ignore", RuntimeWarning)
                log_cc = np.log(self.class_count_)
            self.class_log_prior_ = log_cc - np.log(self.class_count_.sum())
        else:
            self.class_log_prior_ = np.full(n_cls, -np.log(n_cls))

    def _binarize_y(self, y, sample_weight):
        lb = LabelBinarizer()
        Y = lb.fit_transform(y).astype(np.float64)
        self.classes_ = lb.classes_
        if Y.shape[1] == 1:
            Y = np.concatenate((1 - Y, Y), axis=1) if len(self.classes_) == 2 else \
                np.ones_like(Y)
        if sample_weight is not None:
            Y = Y * np.asarray(sample_weight, dtype=np.float64)[:, None]
        return Y

    def _prep(self, X):
        return _dense(X)

    def fit(self, X, y, sample_weight=None):
        X = self._prep(X)
        self.n_features_in_ = X.shape[1]
        y = np.asarray(y).reshape(-1)
        Y = self._binarize_y(y, sample_weight)
        n_cls = Y.shape[1]
        self._init_counters(n_cls, X.shape[1])
        self._count(X, Y)
        alpha = self._check_alpha()
        self._update_feature_log_prob(alpha)
        self._update_class_log_prior(class_prior=self.class_prior)
        return self

    def partial_fit(self, X, y, classes=None, sample_weight=None):
        X = self._prep(X)
        y = np.asarray(y).reshape(-1)
        if not hasattr(self, "classes_"):
            self.classes_ = np.asarray(classes)
            self.n_features_in_ = X.shape[1]
            self._init_counters(len(self.classes_), X.shape[1])
        Y = (y[:, None] == self.classes_[None, :]).astype(np.float64)
        if sample_weight is not None:
            Y *= np.asarray(sample_weight, dtype=np.float64)[:, None]
        self._count(X, Y)
        self._update_feature_log_prob(self._check_alpha())
        self._update_class_log_prior(class_prior=self.class_prior)
        return self

    def _init_counters(self, n_cls, n_feat):
        self.class_count_ = np.zeros(n_cls)
        self.feature_count_ = np.zeros((n_cls, n_feat))

    @property
    def n_features_(self):
        return self.n_features_in_


class MultinomialNB(_BaseDiscreteNB):

    def _more_tags(self):
        return {"requires_positive_X": True}

    def __init__(self, *, alpha=1.0, fit_prior=True, class_prior=None):
        self.alpha = alpha
        self.fit_prior = fit_prior
        self.class_prior = class_prior

    def _count(self, X, Y):
        if np.any(X < 0):
            raise ValueError("Negative values in data passed to MultinomialNB (input X)")
        self.feature_count_ += Y.T @ X
        self.class_count_ += Y.sum(axis=0)

    def _update_feature_log_prob(self, alpha):
        smoothed_fc = self.feature_count_ + alpha
        smoothed_cc = smoothed_fc.sum(axis=1)
        self.feature_log_prob_ = np.log(smoothed_fc) - np.log(smoothed_cc.reshape(-1, 1))

    def _joint_log_likelihood(self, X):
        return X @ self.feature_log_prob_.T + self.class_log_prior_


class ComplementNB(_BaseDiscreteNB):

    def _more_tags(self):
        return {"requires_positive_X": True}

    def __init__(self, *, alpha=1.0, fit_prior=True, class_prior=None, norm=False):
        self.alpha = alpha
        self.fit_prior = fit_prior
        self.class_prior = class_prior
        self.norm = norm

    def _count(self, X, Y):
        if np.any(X < 0):
            raise ValueError("Negative values in data passed to ComplementNB (input X)")
        self.feature_count_ += Y.T @ X
        self.class_count_ += Y.sum(axis=0)
        self.feature_all_ = self.feature_count_.sum(axis=0)

    def _update_feature_log_prob(self, alpha):
        comp_count = self.feature_all_ + alpha - self.feature_count_
        logged = np.log(comp_count / comp_count.sum(axis=1, keepdims=True))
        if self.norm:
            feature_log_prob = logged / logged.sum(axis=1, keepdims=True)
        else:
            feature_log_prob = -logged
        self.feature_log_prob_ = feature_log_prob

    def _joint_log_likelihood(self, X):
        jll = X @ self.feature_log_prob_.T
        if len(self.classes_) == 1:
            jll += self.class_log_prior_
        return jll


class BernoulliNB(_BaseDiscreteNB):

    def _more_tags(self):
        return {"poor_score": True}

    def __init__(self, *, alpha=1.0, binarize=0.0, fit_prior=True, class_prior=None):
        self.alpha = alpha
        self.binarize = binarize
        self.fit_prior = fit_prior
        self.class_prior = class_prior

    def _prep(self, X):
        X = _dense(X)
        if self.binarize is not None:
            X = (X > self.binarize).astype(np.float64)
        return X

    def _check_X(self, X):
        X = self._prep(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError("Expected input with %d features, got %d instead"
                             % (self.n_features_in_, X.shape[1]))
        return X

    def _count(self, X, Y):
        self.feature_count_ += Y.T @ X
        self.class_count_ += Y.sum(axis=0)

    def _update_feature_log_prob(self, alpha):
        smoothed_fc = self.feature_count_ + alpha
        smoothed_cc = self.class_count_ + alpha * 2
        self.feature_log_prob_ = np.log(smoothed_fc) - np.log(smoothed_cc.reshape(-1, 1))

    def _joint_log_likelihood(self, X):
        neg_prob = np.log(1 - np.exp(self.feature_log_prob_))
        jll = X @ (self.feature_log_prob_ - neg_prob).T
        jll += self.class_log_prior_ + neg_prob.sum(axis=1)
        return jll


class CategoricalNB(_BaseDiscreteNB):

    def _more_tags(self):
        return {"requires_positive_X": True}

    def __init__(self, *, alpha=1.0, fit_prior=True, class_prior=None, min_categories=None):
        self.alpha = alpha
        self.fit_prior = fit_prior
        self.class_prior = class_prior
        self.min_categories = min_categories

    def _prep(self, X):
        X = _dense(X)
        if np.any(X < 0):
            raise ValueError("Negative values in data passed to CategoricalNB (input X)")
        return X.astype(np.int64)

    _check_X = _prep

    def _init_counters(self, n_cls, n_feat):
        self.class_count_ = np.zeros(n_cls)
        self.category_count_ = [np.zeros((n_cls, 0)) for _ in range(n_feat)]

    def _count(self, X, Y):
        self.class_count_ += Y.sum(axis=0)
        n_cat = X.max(axis=0) + 1
        if self.min_categories is not None:
            n_cat = np.maximum(n_cat, np.broadcast_to(self.min_categories, n_cat.shape))
        for j in range(X.shape[1]):
            cc = self.category_count_[j]
            if n_cat[j] > cc.shape[1]:
                cc = np.hstack([cc, np.zeros((cc.shape[0], n_cat[j] - cc.shape[1]))])
            onehot = np.zeros((X.shape[0], cc.shape[1]))
            onehot[np.arange(X.shape[0]), X[:, j]] = 1.0
            cc += Y.T @ onehot
            self.category_count_[j] = cc
        self.n_categories_ = np.array([c.shape[1] for c in self.category_count_])

    def _update_feature_log_prob(self, alpha):
        self.feature_log_prob_ = []
        for cc in self.category_count_:
            smoothed = cc + alpha
            self.feature_log_prob_.append(np.log(smoothed)
                                          - np.log(smoothed.sum(axis=1, keepdims=True)))

    def _joint_log_likelihood(self, X):
        jll = np.zeros((X.shape[0], len(self.classes_)))
        for j, flp in enumerate(self.feature_log_prob_):
            idx = np.clip(X[:, j], 0, flp.shape[1] - 1)
            jll += flp[:, idx].T
        return jll + self.class_log_prior_


__all__ = ["GaussianNB", "MultinomialNB", "ComplementNB", "BernoulliNB", "CategoricalNB"]
