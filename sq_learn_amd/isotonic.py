"""Isotonic regression (reference ``isotonic.py`` +
``_isotonic.pyx``).

The pool-adjacent-violators pass and the duplicate aggregation run in the
host-native library (``csrc/host/isotonic.cpp``); interpolation of the
fitted step function uses scipy as the reference does."""

import math
import warnings

import numpy as np
from scipy import interpolate
from scipy.stats import spearmanr

from .base import BaseEstimator, RegressorMixin, TransformerMixin
from .ops import _host
from .utils.validation import check_array, check_consistent_length

__all__ = ["check_increasing", "isotonic_regression", "IsotonicRegression"]


def check_increasing(x, y):
    """Sign of the Spearman correlation of (x, y) (warns when its 95%
    Fisher interval spans zero)."""
    rho, _ = spearmanr(x, y)
    increasing_bool = rho >= 0
    if rho not in [-1.0, 1.0] and len(x) > 3:
        F = 0.5 * math.log((1.0 + rho) / (1.0 - rho))
        F_se = 1 / math.sqrt(len(x) - 3)
        lo, hi = math.tanh(F - 1.96 * F_se), math.tanh(F + 1.96 * F_se)
        if np.sign(lo) != np.sign(hi):
            warnings.warn("Confidence interval of the Spearman correlation coefficient spans "
                          "zero. Determination of ``increasing`` may be suspect.")
    return increasing_bool


def _weights(sample_weight, y, dtype):
    if sample_weight is None:
        return np.ones(len(y), dtype=dtype)
    w = np.asarray(sample_weight, dtype=dtype)
    if w.ndim == 0:
        return np.full(len(y), w, dtype=dtype)
    if w.shape != (len(y),):
        raise ValueError(f"sample_weight.shape == {w.shape}, expected {(len(y),)}!")
    return w.copy()


def _pava_inplace(y, w):
    L = _host.lib()
    if y.dtype == np.float32:
        L.sqh_pava_f32(_host.ptr(y), _host.ptr(w), y.size)
    else:
        L.sqh_pava_f64(_host.ptr(y), _host.ptr(w), y.size)


def isotonic_regression(y, *, sample_weight=None, y_min=None, y_max=None, increasing=True):
    """Solve min sum w_i (y_i - yhat_i)^2 s.t. yhat monotone (and within
    [y_min, y_max])."""
    order = np.s_[:] if increasing else np.s_[::-1]
    y = check_array(y, ensure_2d=False, dtype=[np.float64, np.float32])
    y = np.array(y[order], dtype=y.dtype)
    w = np.ascontiguousarray(_weights(sample_weight, y, y.dtype)[order])
    _pava_inplace(y, w)
    if y_min is not None or y_max is not None:
        np.clip(y, -np.inf if y_min is None else y_min, np.inf if y_max is None else y_max, y)
    return y[order]


def _make_unique(X, y, w):
    n = len(X)
    dt = X.dtype
    X, y, w = (np.ascontiguousarray(a, dtype=dt) for a in (X, y, w))
    xo, yo, wo = np.empty(n, dt), np.empty(n, dt), np.empty(n, dt)
    L = _host.lib()
    fn = L.sqh_make_unique_f32 if dt == np.float32 else L.sqh_make_unique_f64
    u = fn(_host.ptr(X), _host.ptr(y), _host.ptr(w), n, float(np.finfo(dt).resolution),
           _host.ptr(xo), _host.ptr(yo), _host.ptr(wo))
    return xo[:u], yo[:u], wo[:u]


class IsotonicRegression(RegressorMixin, TransformerMixin, BaseEstimator):
    """Isotonic regression model (y_min, y_max, increasing True/False/'auto',
    out_of_bounds 'nan' | 'clip' | 'raise')."""

    def __init__(self, *, y_min=None, y_max=None, increasing=True, out_of_bounds="nan"):
        self.y_min = y_min
        self.y_max = y_max
        self.increasing = increasing
        self.out_of_bounds = out_of_bounds

    def _check_input_data_shape(self, X):
        if not (X.ndim == 1 or (X.ndim == 2 and X.shape[1] == 1)):
            raise ValueError("Isotonic regression input X should be a 1d array or 2d array "
                             "with 1 feature")

    def _check_oob(self):
        if self.out_of_bounds not in ["raise", "nan", "clip"]:
            raise ValueError("The argument ``out_of_bounds`` must be in 'nan', 'clip', "
                             "'raise'; got {0}".format(self.out_of_bounds))

    def _build_f(self, X, y):
        self._check_oob()
        if len(y) == 1:
            self.f_ = lambda x: y.repeat(x.shape)
        else:
            self.f_ = interpolate.interp1d(X, y, kind="linear",
                                           bounds_error=self.out_of_bounds == "raise")

    def _build_y(self, X, y, sample_weight, trim_duplicates=True):
        self._check_input_data_shape(X)
        X = X.reshape(-1)
        self.increasing_ = (check_increasing(X, y) if self.increasing == "auto"
                            else self.increasing)
        w = _weights(sample_weight, X, X.dtype)
        mask = w > 0
        X, y, w = X[mask], y[mask], w[mask]
        order = np.lexsort((y, X))
        X, y, w = X[order], y[order], w[order]
        X, y, w = _make_unique(X, y, w)
        y = isotonic_regression(y, sample_weight=w, y_min=self.y_min, y_max=self.y_max,
                                increasing=self.increasing_)
        self.X_min_, self.X_max_ = np.min(X), np.max(X)
        if trim_duplicates:
            keep = np.ones((len(y),), dtype=bool)
            keep[1:-1] = np.logical_or(np.not_equal(y[1:-1], y[:-2]),
                                       np.not_equal(y[1:-1], y[2:]))
            return X[keep], y[keep]
        return X, y

    def fit(self, X, y, sample_weight=None):
        X = check_array(X, dtype=[np.float64, np.float32], ensure_2d=False)
        y = check_array(y, dtype=X.dtype, ensure_2d=False)
        check_consistent_length(X, y, sample_weight)
        X, y = self._build_y(X, y, sample_weight)
        self.X_thresholds_, self.y_thresholds_ = X, y
        self._build_f(X, y)
        return self

    def transform(self, T):
        dtype = self.X_thresholds_.dtype if hasattr(self, "X_thresholds_") else np.float64
        T = check_array(T, dtype=dtype, ensure_2d=False)
        self._check_input_data_shape(T)
        T = T.reshape(-1)
        self._check_oob()
        if self.out_of_bounds == "clip":
            T = np.clip(T, self.X_min_, self.X_max_)
        return np.asarray(self.f_(T)).astype(T.dtype)

    def predict(self, T):
        return self.transform(T)

    def __getstate__(self):
        state = super().__getstate__()
        state.pop("f_", None)
        return state

    def __setstate__(self, state):
        super().__setstate__(state)
        if hasattr(self, "X_thresholds_") and hasattr(self, "y_thresholds_"):
            self._build_f(self.X_thresholds_, self.y_thresholds_)

    def _more_tags(self):
        return {"X_types": ["1darray"]}
