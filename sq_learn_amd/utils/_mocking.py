"""Test doubles of the reference (``sklearn/utils/_mocking.py``): a minimal
DataFrame stand-in with ``iloc`` slicing, a classifier that asserts on what
``fit`` / ``predict`` receive, and a wrapper that hides ``sample_weight``."""

import numpy as np

from ..base import BaseEstimator, ClassifierMixin
from .validation import _num_samples, check_array, check_is_fitted


class ArraySlicingWrapper:
    """``df.iloc``: row slicing that keeps the MockDataFrame type."""

    def __init__(self, array):
        self.array = array

    def __getitem__(self, aslice):
        return MockDataFrame(self.array[aslice])


class MockDataFrame:
    """An array that is not an ndarray: ``iloc``, ``shape``, ``ndim``,
    ``take``, ``__array__`` and elementwise comparisons, like a DataFrame."""

    def __init__(self, array):
        self.array = array
        self.values = array
        self.shape = array.shape
        self.ndim = array.ndim
        self.iloc = ArraySlicingWrapper(array)

    def __len__(self):
        return len(self.array)

    def __array__(self, dtype=None, copy=None):
        return np.asarray(self.array, dtype=dtype)

    def __eq__(self, other):
        return MockDataFrame(self.array == other.array)

    def __ne__(self, other):
        return not self == other

    def take(self, indices, axis=0):
        return MockDataFrame(self.array.take(indices, axis=axis))


class CheckingClassifier(ClassifierMixin, BaseEstimator):
    """Predicts the first class; runs ``check_X`` / ``check_y`` (callables
    returning bool or the validated array) on what it receives and can
    require specific fit parameters - for testing meta-estimators."""

    def __init__(self, *, check_y=None, check_y_params=None, check_X=None, check_X_params=None,
                 methods_to_check="all", foo_param=0, expected_fit_params=None):
        self.check_y = check_y
        self.check_y_params = check_y_params
        self.check_X = check_X
        self.check_X_params = check_X_params
        self.methods_to_check = methods_to_check
        self.foo_param = foo_param
        self.expected_fit_params = expected_fit_params

    def _check(self, method, X, y=None):
        if self.methods_to_check != "all" and method not in self.methods_to_check:
            return X, y
        for fn, params, arr, name in ((self.check_X, self.check_X_params, X, "X"),
                                      (self.check_y, self.check_y_params, y, "y")):
            if fn is None or arr is None:
                continue
            res = fn(arr, **(params or {}))
            if isinstance(res, (bool, np.bool_)):
                assert res, f"check_{name} failed in {method}"
            elif name == "X":
                X = res
            else:
                y = res
        return X, y

    def fit(self, X, y, sample_weight=None, **fit_params):
        assert _num_samples(X) == _num_samples(y)
        if self.methods_to_check == "all" or "fit" in self.methods_to_check:
            X, y = self._check("fit", X, y)
        self.n_features_in_ = np.shape(X)[1]
        self.classes_ = np.unique(check_array(y, ensure_2d=False, allow_nd=True, dtype=None))
        if self.expected_fit_params:
            missing = set(self.expected_fit_params) - set(fit_params)
            if missing:
                raise AssertionError(f"Expected fit parameter(s) {sorted(missing)} not seen.")
            for key, value in fit_params.items():
                if _num_samples(value) != _num_samples(X):
                    raise AssertionError(f"Fit parameter {key} has length {_num_samples(value)}"
                                         f"; expected {_num_samples(X)}.")
        return self

    def predict(self, X):
        check_is_fitted(self)
        X, _ = self._check("predict", X)
        return self.classes_[np.zeros(_num_samples(X), dtype=int)]

    def predict_proba(self, X):
        check_is_fitted(self)
        X, _ = self._check("predict_proba", X)
        proba = np.zeros((_num_samples(X), len(self.classes_)))
        proba[:, 0] = 1
        return proba

    def decision_function(self, X):
        check_is_fitted(self)
        X, _ = self._check("decision_function", X)
        if len(self.classes_) == 2:
            return np.zeros(_num_samples(X))
        dec = np.zeros((_num_samples(X), len(self.classes_)))
        dec[:, 0] = 1
        return dec

    def score(self, X=None, Y=None):
        self._check("score", X, Y)
        return 1.0 if self.foo_param > 1 else 0.0

    def _more_tags(self):
        return {"_skip_test": True, "X_types": ["1dlabel"]}


class NoSampleWeightWrapper(BaseEstimator):
    """Forwards fit / predict / predict_proba to ``est`` without
    sample_weight."""

    def __init__(self, est=None):
        self.est = est

    def fit(self, X, y):
        return self.est.fit(X, y)

    def predict(self, X):
        return self.est.predict(X)

    def predict_proba(self, X):
        return self.est.predict_proba(X)

    def _more_tags(self):
        return {"_skip_test": True}
