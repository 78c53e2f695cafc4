"""Multiclass reductions (reference ``sklearn/multiclass.py``):
``OneVsRestClassifier`` :188, ``OneVsOneClassifier`` :540 with the
vote + normalised-confidence tie breaking of ``_ovr_decision_function``
(reference utils/multiclass.py:442), ``OutputCodeClassifier`` :790.

Sub-estimators are independent tasks of the task layer
(``parallel/tasks.py``): ``n_jobs`` worker threads, task i pinned to GPU
i mod n_gpus when several GPUs are visible (reference ``Parallel(n_jobs)``
at multiclass.py:281, 339, 641, 696)."""

import numpy as np
import scipy.sparse as sp

from .parallel.tasks import Parallel
from .utils.fixes import delayed
from .base import BaseEstimator, ClassifierMixin, MetaEstimatorMixin, clone, is_regressor
from .metrics import euclidean_distances
from .preprocessing import LabelBinarizer
from .utils.metaestimators import available_if
from .utils.validation import check_is_fitted, check_random_state


def _to_np(a):
    a = a.detach().cpu().numpy() if hasattr(a, "detach") else a
    return np.asarray(a)


def _fit_binary(estimator, X, y, classes=None):
    uniq = np.unique(y)
    if len(uniq) == 1:
        if classes is not None:
            c = 0 if y[0] == -1 else y[0]
            import warnings
            warnings.warn("Label %s is present in all training examples." % str(classes[c]))
        return _ConstantPredictor().fit(X, uniq)
    est = clone(estimator)
    est.fit(X, y)
    return est


def _predict_binary(est, X):
    if is_regressor(est):
        return _to_np(est.predict(X))
    try:
        s = _to_np(est.decision_function(X)).ravel()
    except (AttributeError, NotImplementedError):
        s = _to_np(est.predict_proba(X))[:, 1]
    return s


def _ovr_decision_function(predictions, confidences, n_classes):
    n = predictions.shape[0]
    votes = np.zeros((n, n_classes))
    conf = np.zeros((n, n_classes))
    k = 0
    for i in range(n_classes):
        for j in range(i + 1, n_classes):
            conf[:, i] -= confidences[:, k]
            conf[:, j] += confidences[:, k]
            votes[predictions[:, k] == 0, i] += 1
            votes[predictions[:, k] == 1, j] += 1
            k += 1
    return votes + conf / (3 * (np.abs(conf) + 1))


class _ConstantPredictor(BaseEstimator):
    def fit(self, X, y):
        self.y_ = y
        return self

    def predict(self, X):
        return np.repeat(self.y_, X.shape[0])

    def decision_function(self, X):
        return np.repeat(self.y_, X.shape[0])

    def predict_proba(self, X):
        return np.repeat([np.hstack([1 - self.y_, self.y_])], X.shape[0], axis=0)


def _has(attr):
    def check(self):
        est = self.estimators_[0] if hasattr(self, "estimators_") else self.estimator
        return hasattr(est, attr)
    return check


class OneVsRestClassifier(MetaEstimatorMixin, ClassifierMixin, BaseEstimator):
    """One binary estimator per class (or per label for multilabel y)."""

    def __init__(self, estimator, *, n_jobs=None):
        self.estimator = estimator
        self.n_jobs = n_jobs

    def fit(self, X, y):
        self.label_binarizer_ = LabelBinarizer(sparse_output=True)
        Y = self.label_binarizer_.fit_transform(y)
        Y = Y.tocsc() if sp.issparse(Y) else sp.csc_matrix(Y)
        self.classes_ = self.label_binarizer_.classes_
        cols = (np.asarray(col.toarray()).ravel() for col in Y.T)
        # one binary problem per class, fanned out by the task layer
        # (reference multiclass.py:281 Parallel(n_jobs))
        self.estimators_ = Parallel(n_jobs=self.n_jobs)(
            delayed(_fit_binary)(self.estimator, X, c,
                                 classes=["not %s" % self.label_binarizer_.classes_[i],
                                          self.label_binarizer_.classes_[i]])
            for i, c in enumerate(cols))
        if hasattr(self.estimators_[0], "n_features_in_"):
            self.n_features_in_ = self.estimators_[0].n_features_in_
        return self

    def partial_fit(self, X, y, classes=None):
        if not hasattr(self, "estimators_"):
            if classes is None:
                raise ValueError("classes must be passed on the first call to partial_fit.")
            self.estimators_ = [clone(self.estimator) for _ in range(len(classes))]
            self.label_binarizer_ = LabelBinarizer(sparse_output=True)
            self.label_binarizer_.fit(classes)
            self.classes_ = self.label_binarizer_.classes_
        Y = self.label_binarizer_.transform(y)
        Y = (Y.toarray() if sp.issparse(Y) else np.asarray(Y))
        for i, e in enumerate(self.estimators_):
            e.partial_fit(X, Y[:, i], classes=np.array([0, 1]))
        return self

    @property
    def multilabel_(self):
        return self.label_binarizer_.y_type_.startswith("multilabel")

    @property
    def n_classes_(self):
        return len(self.classes_)

    def predict(self, X):
        check_is_fitted(self)
        n = X.shape[0]
        if self.label_binarizer_.y_type_ == "multiclass":
            maxima = np.full(n, -np.inf)
            argmax = np.zeros(n, dtype=int)
            for i, e in enumerate(self.estimators_):
                pred = _predict_binary(e, X)
                np.maximum(maxima, pred, out=maxima)
                argmax[maxima == pred] = i
            return self.classes_[argmax]
        thresh = 0 if hasattr(self.estimators_[0], "decision_function") and \
            is_classifier_like(self.estimators_[0]) else 0.5
        indicator = np.column_stack([_predict_binary(e, X) > thresh for e in self.estimators_])
        return self.label_binarizer_.inverse_transform(sp.csc_matrix(indicator.astype(int)))

    @available_if(_has("predict_proba"))
    def predict_proba(self, X):
        check_is_fitted(self)
        Y = np.array([_to_np(e.predict_proba(X))[:, 1] for e in self.estimators_]).T
        if len(self.estimators_) == 1:
            Y = np.concatenate(((1 - Y), Y), axis=1)
        if not self.multilabel_:
            Y /= np.sum(Y, axis=1)[:, np.newaxis]
        return Y

    @available_if(_has("decision_function"))
    def decision_function(self, X):
        check_is_fitted(self)
        if len(self.estimators_) == 1:
            return _to_np(self.estimators_[0].decision_function(X))
        return np.array([_to_np(e.decision_function(X)).ravel() for e in self.estimators_]).T


def is_classifier_like(est):
    return not isinstance(est, _ConstantPredictor)


def _fit_ovo_binary(estimator, X, y, i, j):
    cond = np.logical_or(y == i, y == j)
    y = y[cond]
    yb = np.empty(y.shape, int)
    yb[y == i] = 0
    yb[y == j] = 1
    idx = np.arange(X.shape[0])[cond]
    return _fit_binary(estimator, X[idx], yb, classes=[i, j]), idx


class OneVsOneClassifier(MetaEstimatorMixin, ClassifierMixin, BaseEstimator):
    """One binary estimator per class pair; predictions by vote with
    confidence tie-breaking."""

    def __init__(self, estimator, *, n_jobs=None):
        self.estimator = estimator
        self.n_jobs = n_jobs

    def fit(self, X, y):
        X = X if sp.issparse(X) else np.asarray(X)
        y = np.asarray(y)
        self.classes_ = np.unique(y)
        if len(self.classes_) == 1:
            raise ValueError("OneVsOneClassifier can not be fit when only one class is present.")
        n = self.classes_.shape[0]
        fits = Parallel(n_jobs=self.n_jobs)(
            delayed(_fit_ovo_binary)(self.estimator, X, y, self.classes_[i], self.classes_[j])
            for i in range(n) for j in range(i + 1, n))   # reference multiclass.py:641
        self.estimators_ = [f[0] for f in fits]
        self.pairwise_indices_ = None
        self.n_features_in_ = X.shape[1]
        return self

    def partial_fit(self, X, y, classes=None):
        if not hasattr(self, "estimators_"):
            if classes is None:
                raise ValueError("classes must be passed on the first call to partial_fit.")
            self.classes_ = np.unique(classes)
            n = len(self.classes_)
            self.estimators_ = [clone(self.estimator) for _ in range(n * (n - 1) // 2)]
        X, y = np.asarray(X), np.asarray(y)
        n = len(self.classes_)
        k = 0
        for i in range(n):
            for j in range(i + 1, n):
                ci, cj = self.classes_[i], self.classes_[j]
                cond = (y == ci) | (y == cj)
                if cond.any():
                    yb = (y[cond] == cj).astype(int)
                    self.estimators_[k].partial_fit(X[cond], yb, np.array([0, 1]))
                k += 1
        self.pairwise_indices_ = None
        return self

    def decision_function(self, X):
        check_is_fitted(self)
        X = X if sp.issparse(X) else np.asarray(X)
        preds = np.vstack([_to_np(e.predict(X)) for e in self.estimators_]).T
        confs = np.vstack([_predict_binary(e, X) for e in self.estimators_]).T
        Y = _ovr_decision_function(preds, confs, len(self.classes_))
        return Y[:, 1] if len(self.classes_) == 2 else Y

    def predict(self, X):
        Y = self.decision_function(X)
        if len(self.classes_) == 2:
            return self.classes_[(Y > 0).astype(int)]
        return self.classes_[Y.argmax(axis=1)]

    @property
    def n_classes_(self):
        return len(self.classes_)


class OutputCodeClassifier(MetaEstimatorMixin, ClassifierMixin, BaseEstimator):
    """Error-correcting output codes: random code book, one estimator per
    bit, nearest code word (euclidean) at predict time."""

    def __init__(self, estimator, *, code_size=1.5, random_state=None, n_jobs=None):
        self.estimator = estimator
        self.code_size = code_size
        self.random_state = random_state
        self.n_jobs = n_jobs

    def fit(self, X, y):
        X = X if sp.issparse(X) else np.asarray(X)
        y = np.asarray(y)
        if self.code_size <= 0:
            raise ValueError("code_size should be greater than 0, got {0}".format(self.code_size))
        rs = check_random_state(self.random_state)
        self.classes_ = np.unique(y)
        nc = self.classes_.shape[0]
        if nc == 0:
            raise ValueError("OutputCodeClassifier can not be fit when no class is present.")
        code_size_ = int(nc * self.code_size)
        self.code_book_ = rs.random_sample((nc, code_size_))
        self.code_book_[self.code_book_ > 0.5] = 1
        if hasattr(self.estimator, "decision_function"):
            self.code_book_[self.code_book_ != 1] = -1
        else:
            self.code_book_[self.code_book_ != 1] = 0
        cls_idx = {c: i for i, c in enumerate(self.classes_)}
        Y = np.array([self.code_book_[cls_idx[v]] for v in y], dtype=int)
        self.estimators_ = Parallel(n_jobs=self.n_jobs)(
            delayed(_fit_binary)(self.estimator, X, Y[:, i]) for i in range(Y.shape[1]))
        self.n_features_in_ = X.shape[1]
        return self

    def predict(self, X):
        check_is_fitted(self)
        X = X if sp.issparse(X) else np.asarray(X)
        Y = np.array([_predict_binary(e, X) for e in self.estimators_]).T
        return self.classes_[euclidean_distances(Y, self.code_book_).argmin(axis=1)]


__all__ = ["OneVsRestClassifier", "OneVsOneClassifier", "OutputCodeClassifier"]
