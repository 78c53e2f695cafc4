"""Remaining scalers / transformers of the reference's
``preprocessing/_data.py`` (MaxAbsScaler, RobustScaler, Binarizer,
KernelCenterer, QuantileTransformer, PowerTransformer, add_dummy_feature
and the functional forms), ``_discretization.py`` (KBinsDiscretizer),
``_function_transformer.py`` (SplineTransformer is in ``_polynomial.py``).
Dense numpy (fp64) implementations; statistics follow the reference."""

import warnings

import numpy as np
import scipy.sparse as sp
from scipy import optimize, stats
from scipy.interpolate import BSpline

from ..base import BaseEstimator, TransformerMixin
from ..utils.validation import check_array, check_is_fitted, check_random_state


def _dense(X, copy=False):
    if hasattr(X, "detach"):
        X = X.detach().cpu().numpy()
    X = np.array(X, dtype=np.float64, copy=copy) if copy else np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X.reshape(-1, 1)
    return X


def _nf(est, X):
    if X.shape[1] != est.n_features_in_:
        raise ValueError(f"X has {X.shape[1]} features, but {type(est).__name__} is expecting "
                         f"{est.n_features_in_} features as input.")


def _handle_zeros_in_scale(scale):
    scale = np.asarray(scale, dtype=np.float64).copy()
    scale[scale == 0.0] = 1.0
    return scale


class MaxAbsScaler(TransformerMixin, BaseEstimator):

    def _more_tags(self):
        return {"allow_nan": True}

    def __init__(self, *, copy=True):
        self.copy = copy

    def fit(self, X, y=None):
        X = _dense(X)
        self.n_features_in_ = X.shape[1]
        self.max_abs_ = np.nanmax(np.abs(X), axis=0)
        self.scale_ = _handle_zeros_in_scale(self.max_abs_)
        self.n_samples_seen_ = X.shape[0]
        return self

    def partial_fit(self, X, y=None):
        X = _dense(X)
        m = np.nanmax(np.abs(X), axis=0)
        if hasattr(self, "max_abs_"):
            m = np.maximum(self.max_abs_, m)
            self.n_samples_seen_ += X.shape[0]
        else:
            self.n_features_in_ = X.shape[1]
            self.n_samples_seen_ = X.shape[0]
        self.max_abs_ = m
        self.scale_ = _handle_zeros_in_scale(m)
        return self

    def transform(self, X):
        check_is_fitted(self)
        X = _dense(X)
        _nf(self, X)
        return X / self.scale_

    def inverse_transform(self, X):
        return _dense(X) * self.scale_


class RobustScaler(TransformerMixin, BaseEstimator):

    def _more_tags(self):
        return {"allow_nan": True}

    def __init__(self, *, with_centering=True, with_scaling=True, quantile_range=(25.0, 75.0),
                 copy=True, unit_variance=False):
        self.with_centering = with_centering
        self.with_scaling = with_scaling
        self.quantile_range = quantile_range
        self.copy = copy
        self.unit_variance = unit_variance

    def fit(self, X, y=None):
        X = _dense(X)
        self.n_features_in_ = X.shape[1]
        q_min, q_max = self.quantile_range
        if not 0 <= q_min <= q_max <= 100:
            raise ValueError("Invalid quantile range: %s" % str(self.quantile_range))
        self.center_ = np.nanmedian(X, axis=0) if self.with_centering else None
        if self.with_scaling:
            q = np.nanpercentile(X, [q_min, q_max], axis=0)
            self.scale_ = _handle_zeros_in_scale(q[1] - q[0])
            if self.unit_variance:
                adjust = stats.norm.ppf(q_max / 100.0) - stats.norm.ppf(q_min / 100.0)
                self.scale_ = self.scale_ / adjust
        else:
            self.scale_ = None
        return self

    def transform(self, X):
        check_is_fitted(self)
        X = _dense(X, copy=True)
        _nf(self, X)
        if self.with_centering:
            X -= self.center_
        if self.with_scaling:
            X /= self.scale_
        return X

    def inverse_transform(self, X):
        X = _dense(X, copy=True)
        if self.with_scaling:
            X *= self.scale_
        if self.with_centering:
            X += self.center_
        return X


def binarize(X, *, threshold=0.0, copy=True):
    X = _dense(X, copy=copy)
    return (X > threshold).astype(np.float64)


class Binarizer(TransformerMixin, BaseEstimator):

    def _more_tags(self):
        return {"stateless": True}

    def __init__(self, *, threshold=0.0, copy=True):
        self.threshold = threshold
        self.copy = copy

    def fit(self, X, y=None):
        self.n_features_in_ = _dense(X).shape[1]
        return self

    def transform(self, X, copy=None):
        X = _dense(X)
        if hasattr(self, "n_features_in_"):
            _nf(self, X)
        return binarize(X, threshold=self.threshold)


class KernelCenterer(TransformerMixin, BaseEstimator):
    def fit(self, K, y=None):
        K = _dense(K)
        n = K.shape[0]
        self.K_fit_rows_ = K.sum(axis=0) / n
        self.K_fit_all_ = self.K_fit_rows_.sum() / n
        self.n_features_in_ = K.shape[1]
        return self

    def transform(self, K, copy=True):
        check_is_fitted(self)
        K = _dense(K, copy=True)
        K_pred_cols = (K.sum(axis=1) / self.K_fit_rows_.shape[0])[:, None]
        K -= self.K_fit_rows_
        K -= K_pred_cols
        K += self.K_fit_all_
        return K


def add_dummy_feature(X, value=1.0):
    X = _dense(X)
    return np.hstack((np.full((X.shape[0], 1), value), X))


class QuantileTransformer(TransformerMixin, BaseEstimator):

    def _more_tags(self):
        return {"allow_nan": True}

    def __init__(self, *, n_quantiles=1000, output_distribution="uniform",
                 ignore_implicit_zeros=False, subsample=int(1e5), random_state=None, copy=True):
        self.n_quantiles = n_quantiles
        self.output_distribution = output_distribution
        self.ignore_implicit_zeros = ignore_implicit_zeros
        self.subsample = subsample
        self.random_state = random_state
        self.copy = copy

    def fit(self, X, y=None):
        if self.n_quantiles <= 0:
            raise ValueError("Invalid value for 'n_quantiles': %d. The number of quantiles "
                             "must be at least one." % self.n_quantiles)
        if self.output_distribution not in ("uniform", "normal"):
            raise ValueError("'output_distribution' has to be either 'normal' or 'uniform'. "
                             "Got '{}' instead.".format(self.output_distribution))
        X = _dense(X)
        n = X.shape[0]
        self.n_features_in_ = X.shape[1]
        if self.n_quantiles > n:
            warnings.warn("n_quantiles (%s) is greater than the total number of samples (%s). "
                          "n_quantiles is set to n_samples." % (self.n_quantiles, n))
        self.n_quantiles_ = max(1, min(self.n_quantiles, n))
        rng = check_random_state(self.random_state)
        self.references_ = np.linspace(0, 1, self.n_quantiles_, endpoint=True)
        refs = self.references_ * 100
        qs = []
        for col in X.T:
            if self.subsample < n:
                col = col.take(rng.choice(n, size=self.subsample, replace=False))
            qs.append(np.nanpercentile(col, refs))
        self.quantiles_ = np.maximum.accumulate(np.transpose(qs))
        return self

    def _transform_col(self, col, q, inverse):
        lb, ub = 0.0, 1.0
        out_normal = self.output_distribution == "normal"
        if not inverse:
            lo, hi = q[0], q[-1]
        else:
            lo, hi = lb, ub
            if out_normal:
                col = stats.norm.cdf(col)
        lower = col - 1e-7 < lo
        upper = col + 1e-7 > hi
        if out_normal and not inverse:
            lower = col == lo
            upper = col == hi
        isfin = ~np.isnan(col)
        res = col.copy()
        if not inverse:
            res[isfin] = 0.5 * (np.interp(col[isfin], q, self.references_)
                                - np.interp(-col[isfin], -q[::-1], -self.references_[::-1]))
        else:
            res[isfin] = np.interp(col[isfin], self.references_, q)
        res[upper] = ub if not inverse else q[-1]
        res[lower] = lb if not inverse else q[0]
        if out_normal and not inverse:
            clip_min = stats.norm.ppf(1e-7 - np.spacing(1))
            clip_max = stats.norm.ppf(1 - (1e-7 - np.spacing(1)))
            with np.errstate(invalid="ignore", divide="ignore"):
                res = stats.norm.ppf(res)
            res = np.clip(res, clip_min, clip_max)
        return res

    def transform(self, X):
        check_is_fitted(self)
        X = _dense(X, copy=True)
        _nf(self, X)
        for j in range(X.shape[1]):
            X[:, j] = self._transform_col(X[:, j], self.quantiles_[:, j], False)
        return X

    def inverse_transform(self, X):
        check_is_fitted(self)
        X = _dense(X, copy=True)
        for j in range(X.shape[1]):
            X[:, j] = self._transform_col(X[:, j], self.quantiles_[:, j], True)
        return X


def quantile_transform(X, *, axis=0, n_quantiles=1000, output_distribution="uniform",
                       ignore_implicit_zeros=False, subsample=int(1e5), random_state=None,
                       copy=True):
    n = QuantileTransformer(n_quantiles=n_quantiles, output_distribution=output_distribution,
                            subsample=subsample, random_state=random_state, copy=copy)
    X = _dense(X)
    return n.fit_transform(X) if axis == 0 else n.fit_transform(X.T).T


class PowerTransformer(TransformerMixin, BaseEstimator):

    def _more_tags(self):
        return {"allow_nan": True}

    def __init__(self, method="yeo-johnson", *, standardize=True, copy=True):
        self.method = method
        self.standardize = standardize
        self.copy = copy

    @staticmethod
    def _yj(x, lmbda):
        out = np.zeros_like(x)
        pos = x >= 0
        if abs(lmbda) < np.spacing(1.0):
            out[pos] = np.log1p(x[pos])
        else:
            out[pos] = (np.power(x[pos] + 1, lmbda) - 1) / lmbda
        if abs(lmbda - 2) > np.spacing(1.0):
            out[~pos] = -(np.power(-x[~pos] + 1, 2 - lmbda) - 1) / (2 - lmbda)
        else:
            out[~pos] = -np.log1p(-x[~pos])
        return out

    @staticmethod
    def _yj_inv(x, lmbda):
        out = np.zeros_like(x)
        pos = x >= 0
        if abs(lmbda) < np.spacing(1.0):
            out[pos] = np.exp(x[pos]) - 1
        else:
            out[pos] = np.power(x[pos] * lmbda + 1, 1 / lmbda) - 1
        if abs(lmbda - 2) > np.spacing(1.0):
            out[~pos] = 1 - np.power(-(2 - lmbda) * x[~pos] + 1, 1 / (2 - lmbda))
        else:
            out[~pos] = 1 - np.exp(-x[~pos])
        return out

    def _yj_optimize(self, x):
        x = x[~np.isnan(x)]
        n = x.shape[0]

        def nll(lmbda):
            xt = self._yj(x, lmbda)
            var = np.var(xt)
            if var == 0:
                return np.inf
            return -(-n / 2 * np.log(var) + (lmbda - 1) * (np.sign(x) * np.log1p(np.abs(x))).sum())

        return optimize.brent(nll, brack=(-2, 2))

    def fit(self, X, y=None):
        self._fit(X, force_transform=False)
        return self

    def fit_transform(self, X, y=None):
        return self._fit(X, force_transform=True)

    def _fit(self, X, force_transform):
        X = _dense(X, copy=True)
        self.n_features_in_ = X.shape[1]
        if self.method == "box-cox":
            if np.nanmin(X) <= 0:
                raise ValueError("The Box-Cox transformation can only be applied to strictly "
                                 "positive data")
            self.lambdas_ = np.array([stats.boxcox(col[~np.isnan(col)])[1] for col in X.T])
        elif self.method == "yeo-johnson":
            with np.errstate(invalid="ignore", over="ignore"):
                self.lambdas_ = np.array([self._yj_optimize(col) for col in X.T])
        else:
            raise ValueError("'method' must be one of ('box-cox', 'yeo-johnson'), got {} "
                             "instead.".format(self.method))
        Xt = self._apply(X)
        if self.standardize:
            self._mean = np.nanmean(Xt, axis=0)
            self._scale = _handle_zeros_in_scale(np.nanstd(Xt, axis=0))
            Xt = (Xt - self._mean) / self._scale
        return Xt

    def _apply(self, X):
        out = np.empty_like(X)
        for j, lm in enumerate(self.lambdas_):
            out[:, j] = (stats.boxcox(X[:, j], lm) if self.method == "box-cox"
                         else self._yj(X[:, j], lm))
        return out

    def transform(self, X):
        check_is_fitted(self)
        X = _dense(X, copy=True)
        _nf(self, X)
        Xt = self._apply(X)
        if self.standardize:
            Xt = (Xt - self._mean) / self._scale
        return Xt

    def inverse_transform(self, X):
        check_is_fitted(self)
        X = _dense(X, copy=True)
        if self.standardize:
            X = X * self._scale + self._mean
        out = np.empty_like(X)
        for j, lm in enumerate(self.lambdas_):
            if self.method == "box-cox":
                from scipy.special import inv_boxcox
                out[:, j] = inv_boxcox(X[:, j], lm)
            else:
                out[:, j] = self._yj_inv(X[:, j], lm)
        return out


def power_transform(X, method="yeo-johnson", *, standardize=True, copy=True):
    return PowerTransformer(method=method, standardize=standardize, copy=copy).fit_transform(X)


def maxabs_scale(X, *, axis=0, copy=True):
    X = _dense(X)
    return MaxAbsScaler().fit_transform(X) if axis == 0 else MaxAbsScaler().fit_transform(X.T).T


def robust_scale(X, *, axis=0, with_centering=True, with_scaling=True,
                 quantile_range=(25.0, 75.0), copy=True, unit_variance=False):
    s = RobustScaler(with_centering=with_centering, with_scaling=with_scaling,
                     quantile_range=quantile_range, unit_variance=unit_variance)
    X = _dense(X)
    return s.fit_transform(X) if axis == 0 else s.fit_transform(X.T).T


class FunctionTransformer(TransformerMixin, BaseEstimator):

    def _more_tags(self):
        return {"stateless": True, "allow_nan": True}

    def __init__(self, func=None, inverse_func=None, *, validate=False, accept_sparse=False,
                 check_inverse=True, kw_args=None, inv_kw_args=None):
        self.func = func
        self.inverse_func = inverse_func
        self.validate = validate
        self.accept_sparse = accept_sparse
        self.check_inverse = check_inverse
        self.kw_args = kw_args
        self.inv_kw_args = inv_kw_args

    def fit(self, X, y=None):
        if self.validate:
            X = check_array(X, accept_sparse=self.accept_sparse)
            self.n_features_in_ = X.shape[1]
        if self.check_inverse and not (self.func is None or self.inverse_func is None):
            idx = np.arange(0, X.shape[0], max(1, X.shape[0] // 100))
            Xs = X[idx]
            back = self.inverse_transform(self.transform(Xs))
            if not np.allclose(np.asarray(Xs, dtype=float), np.asarray(back, dtype=float)):
                warnings.warn("The provided functions are not strictly inverse of each other. "
                              "If you are sure you want to proceed regardless, set "
                              "'check_inverse=False'.", UserWarning)
        return self

    def transform(self, X):
        if self.validate:
            X = check_array(X, accept_sparse=self.accept_sparse)
        f = self.func if self.func is not None else (lambda x: x)
        return f(X, **(self.kw_args or {}))

    def inverse_transform(self, X):
        f = self.inverse_func if self.inverse_func is not None else (lambda x: x)
        return f(X, **(self.inv_kw_args or {}))


class KBinsDiscretizer(TransformerMixin, BaseEstimator):
    def __init__(self, n_bins=5, *, encode="onehot", strategy="quantile", dtype=None):
        self.n_bins = n_bins
        self.encode = encode
        self.strategy = strategy
        self.dtype = dtype

    def fit(self, X, y=None):
        X = _dense(X)
        self.n_features_in_ = X.shape[1]
        if self.encode not in ("onehot", "onehot-dense", "ordinal"):
            raise ValueError("Valid options for 'encode' are ('onehot', 'onehot-dense', "
                             "'ordinal'). Got encode={!r} instead.".format(self.encode))
        if self.strategy not in ("uniform", "quantile", "kmeans"):
            raise ValueError("Valid options for 'strategy' are ('uniform', 'quantile', "
                             "'kmeans'). Got strategy={!r} instead.".format(self.strategy))
        n_bins = np.full(X.shape[1], self.n_bins, dtype=int) if np.isscalar(self.n_bins) \
            else np.asarray(self.n_bins, dtype=int)
        if np.any(n_bins < 2):
            raise ValueError("KBinsDiscretizer received an invalid number of bins.")
        edges = np.empty(X.shape[1], dtype=object)
        for j in range(X.shape[1]):
            col = X[:, j]
            lo, hi = col.min(), col.max()
            if lo == hi:
                warnings.warn("Feature %d is constant and will be replaced with 0." % j)
                n_bins[j] = 1
                edges[j] = np.array([-np.inf, np.inf])
                continue
            if self.strategy == "uniform":
                e = np.linspace(lo, hi, n_bins[j] + 1)
            elif self.strategy == "quantile":
                e = np.asarray(np.percentile(col, np.linspace(0, 100, n_bins[j] + 1)))
            else:
                from ..models.cluster import KMeans
                uni = np.linspace(lo, hi, n_bins[j] + 1)
                init = (uni[1:] + uni[:-1])[:, None] * 0.5
                km = KMeans(n_clusters=n_bins[j], init=init, n_init=1, algorithm="full",
                            device="cpu")
                c = np.sort(km.fit(col[:, None]).cluster_centers_[:, 0])
                e = np.r_[lo, (c[1:] + c[:-1]) * 0.5, hi]
            if self.strategy in ("quantile", "kmeans"):
                mask = np.ediff1d(e, to_begin=np.inf) > 1e-8
                e = e[mask]
                if len(e) - 1 != n_bins[j]:
                    warnings.warn("Bins whose width are too small (i.e., <= 1e-8) in feature %d "
                                  "are removed. Consider decreasing the number of bins." % j)
                    n_bins[j] = len(e) - 1
            edges[j] = e
        self.bin_edges_ = edges
        self.n_bins_ = n_bins
        if "onehot" in self.encode:
            from ._encoders import OneHotEncoder
            self._encoder = OneHotEncoder(categories=[np.arange(i) for i in self.n_bins_],
                                          sparse=self.encode == "onehot")
            self._encoder.fit(np.zeros((1, len(self.n_bins_))))
        return self

    def transform(self, X):
        check_is_fitted(self)
        X = _dense(X, copy=True)
        _nf(self, X)
        Xt = np.zeros_like(X)
        for j in range(X.shape[1]):
            e = self.bin_edges_[j]
            Xt[:, j] = np.digitize(X[:, j] + 1e-8 * 0, e[1:-1], right=False)
            Xt[:, j] = np.clip(Xt[:, j], 0, self.n_bins_[j] - 1)
        if self.encode == "ordinal":
            return Xt
        return self._encoder.transform(Xt)

    def inverse_transform(self, Xt):
        check_is_fitted(self)
        if "onehot" in self.encode:
            Xt = self._encoder.inverse_transform(Xt)
        Xt = np.asarray(Xt, dtype=np.float64)
        out = np.empty_like(Xt)
        for j in range(Xt.shape[1]):
            e = self.bin_edges_[j]
            centers = (e[1:] + e[:-1]) * 0.5
            out[:, j] = centers[Xt[:, j].astype(int)]
        return out
