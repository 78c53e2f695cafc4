"""Multi-output meta-estimators (reference ``sklearn/multioutput.py``):
``MultiOutputRegressor`` :222, ``MultiOutputClassifier`` :313 (one
estimator per target column) and the chains ``ClassifierChain`` :540 /
``RegressorChain`` :770 (each link sees X plus the previous links'
targets - true targets at fit time, or out-of-fold predictions with
``cv`` - and predictions at inference time)."""

from .parallel.tasks import Parallel
from .utils.fixes import delayed
import numpy as np
import scipy.sparse as sp

from .base import (BaseEstimator, ClassifierMixin, MetaEstimatorMixin, MultiOutputMixin,
                   RegressorMixin, clone, is_classifier)
from .model_selection import cross_val_predict
from .utils.metaestimators import available_if
from .utils.validation import check_is_fitted, check_random_state


def _np(a):
    return a.detach().cpu().numpy() if hasattr(a, "detach") else np.asarray(a)


def _has_est(attr):
    def check(self):
        if hasattr(self, "estimators_"):
            return hasattr(self.estimators_[0], attr)
        return hasattr(self.estimator if hasattr(self, "estimator") else self.base_estimator,
                       attr)
    return check


def _fit_estimator(est, X, y, sample_weight, fit_params):
    if sample_weight is not None:
        return est.fit(X, y, sample_weight=sample_weight, **fit_params)
    return est.fit(X, y, **fit_params)


class _MultiOutputEstimator(MetaEstimatorMixin, MultiOutputMixin, BaseEstimator):
    def __init__(self, estimator, *, n_jobs=None):
        self.estimator = estimator
        self.n_jobs = n_jobs

    def fit(self, X, y, sample_weight=None, **fit_params):
        y = np.asarray(y)
        if y.ndim == 1:
            raise ValueError("y must have at least two dimensions for multi-output regression "
                             "but has only one.")
        if is_classifier(self):
            self.classes_ = []
        # one independent fit per output, fanned out by the task layer
        # (reference multioutput.py:186 Parallel(n_jobs))
        self.estimators_ = Parallel(n_jobs=self.n_jobs)(
            delayed(_fit_estimator)(clone(self.estimator), X, y[:, j], sample_weight, fit_params)
            for j in range(y.shape[1]))
        if is_classifier(self):
            self.classes_ = [e.classes_ for e in self.estimators_]
        if hasattr(self.estimators_[0], "n_features_in_"):
            self.n_features_in_ = self.estimators_[0].n_features_in_
        return self

    @available_if(_has_est("partial_fit"))
    def partial_fit(self, X, y, classes=None, sample_weight=None):
        y = np.asarray(y)
        first = not hasattr(self, "estimators_")
        if first:
            self.estimators_ = [clone(self.estimator) for _ in range(y.shape[1])]
        for j, e in enumerate(self.estimators_):
            kw = {}
            if classes is not None:
                kw["classes"] = classes[j]
            if sample_weight is not None:
                kw["sample_weight"] = sample_weight
            e.partial_fit(X, y[:, j], **kw)
        return self

    def predict(self, X):
        check_is_fitted(self)
        return np.asarray([_np(e.predict(X)) for e in self.estimators_]).T


class MultiOutputRegressor(RegressorMixin, _MultiOutputEstimator):
    """One regressor per target."""

    def _more_tags(self):
        return {"multioutput_only": True}



class MultiOutputClassifier(ClassifierMixin, _MultiOutputEstimator):
    """One classifier per target."""

    def _more_tags(self):
        return {"multioutput_only": True}


    @available_if(_has_est("predict_proba"))
    def predict_proba(self, X):
        check_is_fitted(self)
        return [_np(e.predict_proba(X)) for e in self.estimators_]

    def score(self, X, y):
        y = np.asarray(y)
        if y.ndim == 1:
            raise ValueError("y must have at least two dimensions for multi target "
                             "classification but has only one")
        if y.shape[1] != len(self.estimators_):
            raise ValueError("The number of outputs of Y for fit {0} and score {1} should be "
                             "same".format(len(self.estimators_), y.shape[1]))
        return np.mean(np.all(y == self.predict(X), axis=1))


class _BaseChain(BaseEstimator):
    def __init__(self, base_estimator, *, order=None, cv=None, random_state=None):
        self.base_estimator = base_estimator
        self.order = order
        self.cv = cv
        self.random_state = random_state

    def fit(self, X, Y, **fit_params):
        X = X if sp.issparse(X) else np.asarray(X, dtype=np.float64)
        Y = np.asarray(Y)
        rs = check_random_state(self.random_state)
        self.order_ = self.order
        if isinstance(self.order_, tuple):
            self.order_ = np.array(self.order_)
        if self.order_ is None:
            self.order_ = np.arange(Y.shape[1])
        elif isinstance(self.order_, str):
            if self.order_ == "random":
                self.order_ = rs.permutation(Y.shape[1])
        elif sorted(self.order_) != list(range(Y.shape[1])):
            raise ValueError("invalid order")
        self.estimators_ = [clone(self.base_estimator) for _ in range(Y.shape[1])]
        if self.cv is None:
            Yp = Y[:, self.order_]
            Xa = sp.hstack((X, Yp)) if sp.issparse(X) else np.hstack((X, Yp))
        else:
            Xa = sp.hstack((X, np.zeros(Y.shape))) if sp.issparse(X) else \
                np.hstack((X, np.zeros(Y.shape)))
        if sp.issparse(Xa):
            Xa = Xa.tocsr()
        d = X.shape[1]
        for k, e in enumerate(self.estimators_):
            y = Y[:, self.order_[k]]
            e.fit(Xa[:, :d + k], y, **fit_params)
            if self.cv is not None and k < len(self.estimators_) - 1:
                cvp = cross_val_predict(self.base_estimator, Xa[:, :d + k], y=y, cv=self.cv)
                if sp.issparse(Xa):
                    Xa[:, d + k] = np.expand_dims(cvp, 1)
                else:
                    Xa[:, d + k] = cvp
        self.n_features_in_ = d
        return self

    def _chain(self, X, fn):
        X = X if sp.issparse(X) else np.asarray(X, dtype=np.float64)
        Yc = np.zeros((X.shape[0], len(self.estimators_)))
        outs = []
        for k, e in enumerate(self.estimators_):
            prev = Yc[:, :k]
            Xa = sp.hstack((X, prev)).tocsr() if sp.issparse(X) else np.hstack((X, prev))
            Yc[:, k] = _np(e.predict(Xa))
            if fn is not None:
                outs.append(_np(getattr(e, fn)(Xa)))
        return Yc, outs

    def predict(self, X):
        check_is_fitted(self)
        Yc, _ = self._chain(X, None)
        inv = np.empty_like(self.order_)
        inv[self.order_] = np.arange(len(self.order_))
        return Yc[:, inv]


class ClassifierChain(MetaEstimatorMixin, ClassifierMixin, _BaseChain):

    def _more_tags(self):
        return {"multioutput_only": True}

    def fit(self, X, Y):
        super().fit(X, Y)
        self.classes_ = [e.classes_ for e in self.estimators_]
        return self

    @available_if(_has_est("predict_proba"))
    def predict_proba(self, X):
        _, outs = self._chain(X, "predict_proba")
        P = np.column_stack([o[:, 1] for o in outs])
        inv = np.empty_like(self.order_)
        inv[self.order_] = np.arange(len(self.order_))
        return P[:, inv]

    @available_if(_has_est("decision_function"))
    def decision_function(self, X):
        _, outs = self._chain(X, "decision_function")
        D = np.column_stack([o.ravel() for o in outs])
        inv = np.empty_like(self.order_)
        inv[self.order_] = np.arange(len(self.order_))
        return D[:, inv]


class RegressorChain(MetaEstimatorMixin, RegressorMixin, _BaseChain):

    def _more_tags(self):
        return {"multioutput_only": True}

    def fit(self, X, Y, **fit_params):
        return super().fit(X, Y, **fit_params)


__all__ = ["MultiOutputRegressor", "MultiOutputClassifier", "ClassifierChain", "RegressorChain"]
