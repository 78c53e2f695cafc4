"""Baseline estimators (reference ``sklearn/dummy.py``: DummyClassifier
strategies most_frequent / prior / stratified / uniform / constant,
DummyRegressor mean / median / quantile / constant)."""

import numpy as np

from .base import BaseEstimator, ClassifierMixin, RegressorMixin
from .utils.stats import _weighted_percentile
from .utils.validation import check_is_fitted, check_random_state


def _rows(X):
    return X.shape[0] if hasattr(X, "shape") else len(X)


class DummyClassifier(ClassifierMixin, BaseEstimator):

    def _more_tags(self):
        return {"allow_nan": True, "poor_score": True}

    def __init__(self, *, strategy="prior", random_state=None, constant=None):
        self.strategy = strategy
        self.random_state = random_state
        self.constant = constant

    def fit(self, X, y, sample_weight=None):
        if self.strategy not in ("most_frequent", "stratified", "uniform", "constant", "prior"):
            raise ValueError("Unknown strategy type: %s, expected one of %s."
                             % (self.strategy, ("most_frequent", "stratified", "uniform",
                                                "constant", "prior")))
        y = np.asarray(y)
        self.n_features_in_ = X.shape[1] if hasattr(X, "shape") and len(X.shape) == 2 else None
        self._output_2d = y.ndim == 2 and y.shape[1] > 1
        if y.ndim == 1:
            y = y.reshape(-1, 1)
        self.n_outputs_ = y.shape[1]
        sw = None if sample_weight is None else np.asarray(sample_weight, dtype=np.float64)
        self.classes_, self.n_classes_, self.class_prior_ = [], [], []
        constant = self.constant
        if self.strategy == "constant":
            if constant is None:
                raise ValueError("Constant target value has to be specified when the constant "
                                 "strategy is used.")
            constant = np.reshape(constant, (-1, 1))
            if constant.shape[0] != self.n_outputs_:
                raise ValueError("Constant target value should have shape (%d, 1)."
                                 % self.n_outputs_)
        for k in range(self.n_outputs_):
            cls, inv = np.unique(y[:, k], return_inverse=True)
            prior = np.bincount(inv, weights=sw, minlength=len(cls)).astype(np.float64)
            self.classes_.append(cls)
            self.n_classes_.append(len(cls))
            self.class_prior_.append(prior / prior.sum())
            if self.strategy == "constant" and constant[k][0] not in cls:
                raise ValueError("The constant target value must be present in the training "
                                 "data. You provided constant={}. Possible values are: {}."
                                 .format(self.constant, list(cls)))
        if self.n_outputs_ == 1:
            self.n_classes_ = self.n_classes_[0]
            self.classes_ = self.classes_[0]
            self.class_prior_ = self.class_prior_[0]
        self._constant = constant
        return self

    def predict_proba(self, X):
        check_is_fitted(self)
        n = _rows(X)
        rs = check_random_state(self.random_state)
        ncls = [self.n_classes_] if self.n_outputs_ == 1 else self.n_classes_
        cls = [self.classes_] if self.n_outputs_ == 1 else self.classes_
        prior = [self.class_prior_] if self.n_outputs_ == 1 else self.class_prior_
        out = []
        for k in range(self.n_outputs_):
            if self.strategy == "most_frequent":
                p = np.zeros((n, ncls[k]))
                p[:, prior[k].argmax()] = 1.0
            elif self.strategy == "prior":
                p = np.ones((n, 1)) * prior[k]
            elif self.strategy == "stratified":
                p = rs.multinomial(1, prior[k], size=n).astype(np.float64)
            elif self.strategy == "uniform":
                p = np.ones((n, ncls[k])) / ncls[k]
            else:
                idx = int(np.where(cls[k] == self._constant[k][0])[0][0])
                p = np.zeros((n, ncls[k]))
                p[:, idx] = 1.0
            out.append(p)
        return out[0] if self.n_outputs_ == 1 else out

    def predict_log_proba(self, X):
        p = self.predict_proba(X)
        return np.log(p) if self.n_outputs_ == 1 else [np.log(q) for q in p]

    def predict(self, X):
        check_is_fitted(self)
        n = _rows(X)
        rs = check_random_state(self.random_state)
        cls = [self.classes_] if self.n_outputs_ == 1 else self.classes_
        prior = [self.class_prior_] if self.n_outputs_ == 1 else self.class_prior_
        cols = []
        for k in range(self.n_outputs_):
            if self.strategy in ("most_frequent", "prior"):
                cols.append(np.full(n, cls[k][prior[k].argmax()]))
            elif self.strategy == "stratified":
                cols.append(cls[k][rs.multinomial(1, prior[k], size=n).argmax(axis=1)])
            elif self.strategy == "uniform":
                cols.append(cls[k][rs.randint(len(cls[k]), size=n)])
            else:
                cols.append(np.full(n, self._constant[k][0]))
        y = np.stack(cols, axis=1)
        return y[:, 0] if self.n_outputs_ == 1 and not self._output_2d else y

    def score(self, X, y, sample_weight=None):
        X = np.zeros((len(y), 1)) if X is None else X
        return super().score(X, y, sample_weight)


class DummyRegressor(RegressorMixin, BaseEstimator):

    def _more_tags(self):
        return {"allow_nan": True, "poor_score": True}

    def __init__(self, *, strategy="mean", constant=None, quantile=None):
        self.strategy = strategy
        self.constant = constant
        self.quantile = quantile

    def fit(self, X, y, sample_weight=None):
        if self.strategy not in ("mean", "median", "quantile", "constant"):
            raise ValueError("Unknown strategy type: %s, expected one of ('mean', 'median', "
                             "'quantile', 'constant')." % self.strategy)
        y = np.asarray(y, dtype=np.float64)
        self.n_features_in_ = X.shape[1] if hasattr(X, "shape") and len(X.shape) == 2 else None
        self._output_2d = y.ndim == 2 and y.shape[1] > 1
        if y.ndim == 1:
            y = y.reshape(-1, 1)
        self.n_outputs_ = y.shape[1]
        sw = None if sample_weight is None else np.asarray(sample_weight, dtype=np.float64)
        if self.strategy == "mean":
            c = np.average(y, axis=0, weights=sw)
        elif self.strategy == "median":
            c = (np.median(y, axis=0) if sw is None
                 else np.atleast_1d(_weighted_percentile(y, sw, 50.0)))
        elif self.strategy == "quantile":
            if self.quantile is None or not 0 <= self.quantile <= 1:
                raise ValueError("Quantile must be a scalar in the range [0.0, 1.0], but got %s."
                                 % self.quantile)
            q = self.quantile * 100.0
            c = (np.percentile(y, axis=0, q=q) if sw is None
                 else np.atleast_1d(_weighted_percentile(y, sw, q)))
        else:
            if self.constant is None:
                raise TypeError("Constant target value has to be specified when the constant "
                                "strategy is used.")
            c = np.reshape(np.asarray(self.constant, dtype=np.float64), (-1,))
            if c.shape[0] != self.n_outputs_:
                raise ValueError("Constant target value should have shape (%d, 1)."
                                 % self.n_outputs_)
        self.constant_ = np.reshape(c, (1, -1))
        return self

    def predict(self, X, return_std=False):
        check_is_fitted(self)
        n = _rows(X)
        y = np.full((n, self.n_outputs_), self.constant_[0])
        if self.n_outputs_ == 1 and not self._output_2d:
            y = y[:, 0]
        if return_std:
            return y, np.zeros_like(y)
        return y

    def score(self, X, y, sample_weight=None):
        X = np.zeros((len(y), 1)) if X is None else X
        return super().score(X, y, sample_weight)
