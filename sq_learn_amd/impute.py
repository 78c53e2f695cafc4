"""Missing-value imputation (reference ``sklearn/impute``: SimpleImputer
mean / median / most_frequent / constant, MissingIndicator, KNNImputer
with nan-euclidean distances, IterativeImputer (round-robin regression,
BayesianRidge by default))."""

import warnings

import numpy as np
from scipy import stats

from .base import BaseEstimator, TransformerMixin, clone
from .utils.validation import check_is_fitted, check_random_state


def _mask(X, missing_values):
    if missing_values is np.nan or (isinstance(missing_values, float) and np.isnan(missing_values)):
        return np.isnan(X) if X.dtype.kind == "f" else np.zeros(X.shape, dtype=bool)
    return X == missing_values


def _arr(X, force_float=True):
    if hasattr(X, "detach"):
        X = X.detach().cpu().numpy()
    if hasattr(X, "toarray"):
        X = X.toarray()
    X = np.asarray(X)
    if force_float and X.dtype.kind in "iub":
        X = X.astype(np.float64)
    return X


class MissingIndicator(TransformerMixin, BaseEstimator):

    def _more_tags(self):
        return {"allow_nan": True}

    def __init__(self, *, missing_values=np.nan, features="missing-only", sparse="auto",
                 error_on_new=True):
        self.missing_values = missing_values
        self.features = features
        self.sparse = sparse
        self.error_on_new = error_on_new

    def fit(self, X, y=None):
        X = _arr(X)
        self.n_features_in_ = X.shape[1]
        m = _mask(X, self.missing_values)
        self._n_features = X.shape[1]
        self.features_ = (np.flatnonzero(m.any(axis=0)) if self.features == "missing-only"
                          else np.arange(X.shape[1]))
        return self

    def transform(self, X):
        check_is_fitted(self)
        X = _arr(X)
        self._check_n_features(X, reset=False)
        m = _mask(X, self.missing_values)
        if self.features == "missing-only":
            new = np.setdiff1d(np.flatnonzero(m.any(axis=0)), self.features_)
            if self.error_on_new and new.size:
                raise ValueError("The features {} have missing values in transform but have no "
                                 "missing values in fit.".format(new))
        return m[:, self.features_]

    def fit_transform(self, X, y=None):
        return self.fit(X).transform(X)


class SimpleImputer(TransformerMixin, BaseEstimator):

    def _more_tags(self):
        return {"allow_nan": True}

    def __init__(self, *, missing_values=np.nan, strategy="mean", fill_value=None, verbose=0,
                 copy=True, add_indicator=False):
        self.missing_values = missing_values
        self.strategy = strategy
        self.fill_value = fill_value
        self.verbose = verbose
        self.copy = copy
        self.add_indicator = add_indicator

    def fit(self, X, y=None):
        if self.strategy not in ("mean", "median", "most_frequent", "constant"):
            raise ValueError("Can only use these strategies: ['mean', 'median', "
                             "'most_frequent', 'constant']  got strategy=%s" % self.strategy)
        X = _arr(X, force_float=self.strategy in ("mean", "median"))
        self.n_features_in_ = X.shape[1]
        m = _mask(X, self.missing_values)
        stats_ = np.empty(X.shape[1], dtype=object if X.dtype.kind == "O" else np.float64)
        for j in range(X.shape[1]):
            col = X[~m[:, j], j]
            if self.strategy == "constant":
                fv = self.fill_value
                if fv is None:
                    fv = 0 if X.dtype.kind in "iuf" else "missing_value"
                stats_[j] = fv
            elif col.size == 0:
                stats_[j] = np.nan
            elif self.strategy == "mean":
                stats_[j] = col.mean()
            elif self.strategy == "median":
                stats_[j] = np.median(col)
            else:
                vals, counts = np.unique(col, return_counts=True)
                stats_[j] = vals[np.argmax(counts)]
        self.statistics_ = stats_
        if self.add_indicator:
            self.indicator_ = MissingIndicator(missing_values=self.missing_values,
                                               error_on_new=False).fit(X)
        return self

    def transform(self, X):
        check_is_fitted(self)
        X = _arr(X, force_float=self.strategy in ("mean", "median"))
        if X.shape[1] != self.statistics_.shape[0]:
            raise ValueError("X has %d features per sample, expected %d"
                             % (X.shape[1], self.statistics_.shape[0]))
        m = _mask(X, self.missing_values)
        valid = np.array([not (isinstance(s, float) and np.isnan(s)) for s in self.statistics_]) \
            if self.strategy != "constant" else np.ones(X.shape[1], dtype=bool)
        if not valid.all():
            warnings.warn("Skipping features without any observed values: %s. At least one "
                          "non-missing value is needed for imputation with strategy='%s'."
                          % (np.flatnonzero(~valid), self.strategy))
        Xo = X.astype(object) if (self.strategy == "constant" and X.dtype.kind != "O"
                                  and isinstance(self.statistics_[0], str)) else X.copy()
        for j in np.flatnonzero(valid):
            Xo[m[:, j], j] = self.statistics_[j]
        Xo = Xo[:, valid]
        if self.add_indicator:
            Xo = np.hstack([Xo, self.indicator_.transform(X)])
        return Xo

    def inverse_transform(self, X):
        check_is_fitted(self)
        if not self.add_indicator:
            raise ValueError("'inverse_transform' works only when 'SimpleImputer' is "
                             "instantiated with 'add_indicator=True'.")
        X = _arr(X)
        n = self.statistics_.shape[0]
        out = X[:, :n].copy()
        ind = X[:, n:].astype(bool)
        out[:, self.indicator_.features_][ind] = self.missing_values
        full = out.copy()
        for k, j in enumerate(self.indicator_.features_):
            full[ind[:, k], j] = self.missing_values
        return full


def nan_euclidean_distances(X, Y=None, *, squared=False, missing_values=np.nan, copy=True):
    X = _arr(X)
    Y = X if Y is None else _arr(Y)
    mx, my = _mask(X, missing_values), _mask(Y, missing_values)
    Xz, Yz = np.where(mx, 0, X), np.where(my, 0, Y)
    d = ((Xz ** 2) @ (~my).T + (~mx) @ (Yz ** 2).T - 2 * Xz @ Yz.T)
    np.clip(d, 0, None, out=d)
    present = (~mx).astype(float) @ (~my).astype(float).T
    with np.errstate(divide="ignore", invalid="ignore"):
        d = d * X.shape[1] / present
    d[present == 0] = np.nan
    if Y is X or (Y.shape == X.shape and np.shares_memory(X, Y)):
        np.fill_diagonal(d, 0.0)
    return d if squared else np.sqrt(d)


class KNNImputer(TransformerMixin, BaseEstimator):

    def _more_tags(self):
        return {"allow_nan": True}

    def __init__(self, *, missing_values=np.nan, n_neighbors=5, weights="uniform",
                 metric="nan_euclidean", copy=True, add_indicator=False):
        self.missing_values = missing_values
        self.n_neighbors = n_neighbors
        self.weights = weights
        self.metric = metric
        self.copy = copy
        self.add_indicator = add_indicator

    def fit(self, X, y=None):
        X = _arr(X)
        self.n_features_in_ = X.shape[1]
        self._fit_X = X
        self._mask_fit_X = _mask(X, self.missing_values)
        self._valid_mask = ~np.all(self._mask_fit_X, axis=0)
        if self.add_indicator:
            self.indicator_ = MissingIndicator(missing_values=self.missing_values,
                                               error_on_new=False).fit(X)
        return self

    def transform(self, X):
        check_is_fitted(self)
        X = _arr(X).copy()
        self._check_n_features(X, reset=False)
        m = _mask(X, self.missing_values)
        Xo = X.copy()
        rows = np.flatnonzero(m[:, self._valid_mask].any(axis=1))
        if rows.size:
            D = nan_euclidean_distances(X[rows], self._fit_X, missing_values=self.missing_values)
            for j in np.flatnonzero(self._valid_mask):
                r_need = np.flatnonzero(m[rows, j])
                if not r_need.size:
                    continue
                donors = np.flatnonzero(~self._mask_fit_X[:, j])
                for r in r_need:
                    dd = D[r, donors]
                    ok = ~np.isnan(dd)
                    if not ok.any():
                        Xo[rows[r], j] = np.mean(self._fit_X[donors, j])
                        continue
                    dcand, idx = dd[ok], donors[ok]
                    k = min(self.n_neighbors, len(idx))
                    sel = np.argsort(dcand, kind="stable")[:k]
                    vals = self._fit_X[idx[sel], j]
                    if self.weights == "distance":
                        w = 1.0 / np.maximum(dcand[sel], 1e-300)
                        if np.any(dcand[sel] == 0):
                            w = (dcand[sel] == 0).astype(float)
                    elif callable(self.weights):
                        w = self.weights(dcand[sel])
                    else:
                        w = np.ones(k)
                    Xo[rows[r], j] = np.sum(w * vals) / np.sum(w)
        Xo = Xo[:, self._valid_mask]
        if self.add_indicator:
            Xo = np.hstack([Xo, self.indicator_.transform(X)])
        return Xo


class IterativeImputer(TransformerMixin, BaseEstimator):

    def _more_tags(self):
        return {"allow_nan": True}

    def __init__(self, estimator=None, *, missing_values=np.nan, sample_posterior=False,
                 max_iter=10, tol=1e-3, n_nearest_features=None, initial_strategy="mean",
                 imputation_order="ascending", skip_complete=False, min_value=-np.inf,
                 max_value=np.inf, verbose=0, random_state=None, add_indicator=False):
        self.estimator = estimator
        self.missing_values = missing_values
        self.sample_posterior = sample_posterior
        self.max_iter = max_iter
        self.tol = tol
        self.n_nearest_features = n_nearest_features
        self.initial_strategy = initial_strategy
        self.imputation_order = imputation_order
        self.skip_complete = skip_complete
        self.min_value = min_value
        self.max_value = max_value
        self.verbose = verbose
        self.random_state = random_state
        self.add_indicator = add_indicator

    def _order(self, mask):
        frac = mask.mean(axis=0)
        idx = np.flatnonzero(frac) if self.skip_complete else np.arange(mask.shape[1])
        if self.imputation_order == "roman":
            return idx
        if self.imputation_order == "arabic":
            return idx[::-1]
        if self.imputation_order == "ascending":
            return idx[np.argsort(frac[idx], kind="mergesort")]
        if self.imputation_order == "descending":
            return idx[np.argsort(frac[idx], kind="mergesort")[::-1]]
        if self.imputation_order == "random":
            return self.random_state_.permutation(idx)
        raise ValueError("Got an invalid imputation order: '{0}'".format(self.imputation_order))

    def fit_transform(self, X, y=None):
        X = _arr(X)
        self.n_features_in_ = X.shape[1]
        self.random_state_ = check_random_state(self.random_state)
        if self.estimator is None:
            from .models.linear_model import BayesianRidge
            est = BayesianRidge()
        else:
            est = self.estimator
        mask = _mask(X, self.missing_values)
        self.initial_imputer_ = SimpleImputer(missing_values=self.missing_values,
                                              strategy=self.initial_strategy).fit(X)
        Xt = self.initial_imputer_.transform(X)
        valid = self.initial_imputer_.statistics_.astype(float)
        valid = ~np.isnan(valid)
        mask_v = mask[:, valid]
        self._valid = valid
        if self.max_iter == 0 or not mask_v.any():
            self.n_iter_ = 0
            self.imputation_sequence_ = []
            return Xt
        order = self._order(mask_v)
        self.imputation_sequence_ = []
        abs_corr_mat = None
        normalized_tol = self.tol * np.max(np.abs(X[~mask]))
        for it in range(1, self.max_iter + 1):
            X_prev = Xt.copy()
            if self.imputation_order == "random":
                order = self._order(mask_v)
            for f in order:
                others = np.delete(np.arange(Xt.shape[1]), f)
                miss = mask_v[:, f]
                if not miss.any():
                    continue
                e = clone(est).fit(Xt[~miss][:, others], Xt[~miss, f])
                if self.sample_posterior:
                    mus, sigmas = e.predict(Xt[miss][:, others], return_std=True)
                    pred = self.random_state_.normal(mus, np.maximum(sigmas, 1e-300))
                else:
                    pred = e.predict(Xt[miss][:, others])
                Xt[miss, f] = np.clip(pred, self.min_value, self.max_value)
                self.imputation_sequence_.append((f, others, e))
            self.n_iter_ = it
            inf_norm = np.linalg.norm(Xt - X_prev, ord=np.inf, axis=None)
            if not self.sample_posterior and inf_norm < normalized_tol:
                break
        else:
            if not self.sample_posterior:
                from .exceptions import ConvergenceWarning
                warnings.warn("[IterativeImputer] Early stopping criterion not reached.",
                              ConvergenceWarning)
        if self.add_indicator:
            self.indicator_ = MissingIndicator(missing_values=self.missing_values,
                                               error_on_new=False).fit(X)
            Xt = np.hstack([Xt, self.indicator_.transform(X)])
        return Xt

    def fit(self, X, y=None):
        self.fit_transform(X)
        return self

    def transform(self, X):
        check_is_fitted(self)
        X = _arr(X)
        self._check_n_features(X, reset=False)
        mask = _mask(X, self.missing_values)[:, self._valid]
        Xt = self.initial_imputer_.transform(X)
        for f, others, e in self.imputation_sequence_:
            miss = mask[:, f]
            if miss.any():
                Xt[miss, f] = np.clip(e.predict(Xt[miss][:, others]), self.min_value,
                                      self.max_value)
        if self.add_indicator:
            Xt = np.hstack([Xt, self.indicator_.transform(X)])
        return Xt


__all__ = ["SimpleImputer", "MissingIndicator", "KNNImputer", "IterativeImputer",
           "nan_euclidean_distances"]

from .utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
