"""Probability calibration (reference ``sklearn/calibration.py``):
``CalibratedClassifierCV`` :52 with Platt sigmoid (``_sigmoid_calibration``
:418, BFGS on the prior-corrected log loss exactly as the reference) or
isotonic calibrators per class, ``calibration_curve`` :553.

The per-fold base fits run through the framework's estimators (device
resident); calibration itself is a handful of host scalars per class."""

from math import log

import numpy as np
from scipy.optimize import fmin_bfgs
from scipy.special import expit, xlogy

from .base import BaseEstimator, ClassifierMixin, MetaEstimatorMixin, RegressorMixin, clone
from .isotonic import IsotonicRegression
from .model_selection import check_cv, cross_val_predict
from .preprocessing import LabelEncoder, label_binarize
from .utils.validation import check_is_fitted


def _np(a):
    return a.detach().cpu().numpy() if hasattr(a, "detach") else np.asarray(a)


def _get_prediction_method(clf):
    if hasattr(clf, "decision_function"):
        return getattr(clf, "decision_function"), "decision_function"
    if hasattr(clf, "predict_proba"):
        return getattr(clf, "predict_proba"), "predict_proba"
    raise RuntimeError("classifier has no decision_function or predict_proba method.")


def _compute_predictions(pred_method, method_name, X, n_classes):
    pred = _np(pred_method(X))
    if method_name == "decision_function":
        if pred.ndim == 1:
            pred = pred[:, np.newaxis]
    elif method_name == "predict_proba":
        if n_classes == 2:
            pred = pred[:, 1:]
    else:
        raise ValueError(f"Invalid prediction method: {method_name}")
    return pred


def _sigmoid_calibration(predictions, y, sample_weight=None):
    F = np.asarray(predictions, dtype=np.float64).ravel()
    y = np.asarray(y).ravel()
    prior0 = float(np.sum(y <= 0))
    prior1 = y.shape[0] - prior0
    T = np.zeros(y.shape)
    T[y > 0] = (prior1 + 1.0) / (prior1 + 2.0)
    T[y <= 0] = 1.0 / (prior0 + 2.0)
    T1 = 1.0 - T

    def objective(AB):
        P = expit(-(AB[0] * F + AB[1]))
        loss = -(xlogy(T, P) + xlogy(T1, 1.0 - P))
        return (sample_weight * loss).sum() if sample_weight is not None else loss.sum()

    def grad(AB):
        P = expit(-(AB[0] * F + AB[1]))
        d = T - P
        if sample_weight is not None:
            d *= sample_weight
        return np.array([np.dot(d, F), np.sum(d)])

    AB0 = np.array([0.0, log((prior0 + 1.0) / (prior1 + 1.0))])
    AB = fmin_bfgs(objective, AB0, fprime=grad, disp=False)
    return AB[0], AB[1]


class _SigmoidCalibration(RegressorMixin, BaseEstimator):
    def fit(self, X, y, sample_weight=None):
        self.a_, self.b_ = _sigmoid_calibration(X, y, sample_weight)
        return self

    def predict(self, T):
        return expit(-(self.a_ * np.asarray(T).ravel() + self.b_))


def _fit_calibrator(clf, predictions, y, classes, method, sample_weight=None):
    Y = label_binarize(y, classes=classes)
    le = LabelEncoder().fit(classes)
    pos = le.transform(clf.classes_)
    cals = []
    for ci, pred in zip(pos, predictions.T):
        cal = IsotonicRegression(out_of_bounds="clip") if method == "isotonic" \
            else _SigmoidCalibration()
        cal.fit(pred, Y[:, ci], sample_weight=sample_weight) if method == "isotonic" \
            else cal.fit(pred, Y[:, ci], sample_weight)
        cals.append(cal)
    return _CalibratedClassifier(clf, cals, method=method, classes=classes)


class _CalibratedClassifier:
    def __init__(self, base_estimator, calibrators, *, classes, method="sigmoid"):
        self.base_estimator = base_estimator
        self.calibrators = calibrators
        self.classes = classes
        self.method = method

    def predict_proba(self, X):
        nc = len(self.classes)
        pm, name = _get_prediction_method(self.base_estimator)
        preds = _compute_predictions(pm, name, X, nc)
        pos = LabelEncoder().fit(self.classes).transform(self.base_estimator.classes_)
        n = preds.shape[0]
        proba = np.zeros((n, nc))
        for ci, p, cal in zip(pos, preds.T, self.calibrators):
            if nc == 2:
                ci += 1
            proba[:, ci] = cal.predict(p)
        if nc == 2:
            proba[:, 0] = 1.0 - proba[:, 1]
        else:
            den = np.sum(proba, axis=1)[:, np.newaxis]
            uniform = np.full_like(proba, 1 / nc)
            proba = np.divide(proba, den, out=uniform, where=den != 0)
        proba[(1.0 < proba) & (proba <= 1.0 + 1e-5)] = 1.0
        return proba


class CalibratedClassifierCV(MetaEstimatorMixin, ClassifierMixin, BaseEstimator):
    """Cross-validated probability calibration."""

    def __init__(self, base_estimator=None, *, method="sigmoid", cv=None, n_jobs=None,
                 ensemble=True):
        self.base_estimator = base_estimator
        self.method = method
        self.cv = cv
        self.n_jobs = n_jobs
        self.ensemble = ensemble

    def fit(self, X, y, sample_weight=None):
        y = np.asarray(y)
        if self.base_estimator is None:
            from .svm import LinearSVC
            base = LinearSVC(random_state=0)
        else:
            base = self.base_estimator
        if self.method not in ("sigmoid", "isotonic"):
            raise ValueError("'method' should be one of: 'sigmoid' or 'isotonic'. Got %r."
                             % self.method)
        self.calibrated_classifiers_ = []
        if self.cv == "prefit":
            check_is_fitted(base)
            self.classes_ = base.classes_
            pm, name = _get_prediction_method(base)
            preds = _compute_predictions(pm, name, X, len(self.classes_))
            self.calibrated_classifiers_.append(
                _fit_calibrator(base, preds, y, self.classes_, self.method, sample_weight))
        else:
            le = LabelEncoder().fit(y)
            self.classes_ = le.classes_
            nc = len(self.classes_)
            cv = check_cv(self.cv, y, classifier=True)
            if self.ensemble:
                for train, test in cv.split(X, y):
                    Xtr = X[train]
                    clf = clone(base)
                    if sample_weight is not None:
                        clf.fit(Xtr, y[train], sample_weight=np.asarray(sample_weight)[train])
                    else:
                        clf.fit(Xtr, y[train])
                    pm, name = _get_prediction_method(clf)
                    preds = _compute_predictions(pm, name, X[test], nc)
                    sw = None if sample_weight is None else np.asarray(sample_weight)[test]
                    self.calibrated_classifiers_.append(
                        _fit_calibrator(clf, preds, y[test], self.classes_, self.method, sw))
            else:
                this = clone(base)
                _, name = _get_prediction_method(this)
                preds = _np(cross_val_predict(this, X, y, cv=cv, method=name))
                if name == "decision_function" and preds.ndim == 1:
                    preds = preds[:, np.newaxis]
                elif name == "predict_proba" and nc == 2:
                    preds = preds[:, 1:]
                this.fit(X, y) if sample_weight is None else \
                    this.fit(X, y, sample_weight=sample_weight)
                self.calibrated_classifiers_.append(
                    _fit_calibrator(this, preds, y, self.classes_, self.method, sample_weight))
        first = self.calibrated_classifiers_[0].base_estimator
        if hasattr(first, "n_features_in_"):
            self.n_features_in_ = first.n_features_in_
        return self

    def predict_proba(self, X):
        check_is_fitted(self)
        mean = np.zeros((X.shape[0], len(self.classes_)))
        for c in self.calibrated_classifiers_:
            mean += c.predict_proba(X)
        return mean / len(self.calibrated_classifiers_)

    def predict(self, X):
        return self.classes_[np.argmax(self.predict_proba(X), axis=1)]


def calibration_curve(y_true, y_prob, *, normalize=False, n_bins=5, strategy="uniform"):
    """Fraction of positives vs mean predicted probability per bin."""
    y_true = np.asarray(y_true).ravel()
    y_prob = np.asarray(y_prob, dtype=np.float64).ravel()
    if normalize:
        y_prob = (y_prob - y_prob.min()) / (y_prob.max() - y_prob.min())
    elif y_prob.min() < 0 or y_prob.max() > 1:
        raise ValueError("y_prob has values outside [0, 1] and normalize is set to False.")
    labels = np.unique(y_true)
    if len(labels) > 2:
        raise ValueError("Only binary classification is supported. Provided labels %s." % labels)
    y_true = label_binarize(y_true, classes=labels)[:, 0]
    if strategy == "quantile":
        q = np.linspace(0, 1, n_bins + 1)
        bins = np.percentile(y_prob, q * 100)
        bins[-1] = bins[-1] + 1e-8
    elif strategy == "uniform":
        bins = np.linspace(0.0, 1.0 + 1e-8, n_bins + 1)
    else:
        raise ValueError("Invalid entry to 'strategy' input. Strategy must be either 'quantile' "
                         "or 'uniform'.")
    ids = np.digitize(y_prob, bins) - 1
    sums = np.bincount(ids, weights=y_prob, minlength=len(bins))
    true = np.bincount(ids, weights=y_true, minlength=len(bins))
    total = np.bincount(ids, minlength=len(bins))
    nz = total != 0
    return true[nz] / total[nz], sums[nz] / total[nz]


__all__ = ["CalibratedClassifierCV", "calibration_curve"]
