"""Column-wise composition and target transformation (reference
``compose/_column_transformer.py`` - ``ColumnTransformer`` :37,
``make_column_transformer`` :870, ``make_column_selector`` :960 - and
``compose/_target.py`` - ``TransformedTargetRegressor`` :19).

Column selections accept ints, names (pandas input), slices, boolean
masks, callables and ``make_column_selector``; outputs are stacked dense
or as CSR when the overall density falls below ``sparse_threshold``.
"""



import numpy as np
import scipy.sparse as sp

from .base import BaseEstimator, RegressorMixin, TransformerMixin, clone
from .pipeline import _name_estimators
from .preprocessing import FunctionTransformer
from .utils.metaestimators import _BaseComposition
from .utils.validation import check_is_fitted


def _is_pandas(X):
    return hasattr(X, "iloc") and hasattr(X, "columns")


def _n_cols(X):
    return X.shape[1]


def _col_indices(X, key):
    """Resolve a column spec to integer positions."""
    n = _n_cols(X)
    if callable(key):
        key = key(X)
    if key is None:
        return []
    if isinstance(key, slice):
        if _is_pandas(X) and (isinstance(key.start, str) or isinstance(key.stop, str)):
            cols = list(X.columns)
            start = cols.index(key.start) if key.start is not None else 0
            stop = cols.index(key.stop) + 1 if key.stop is not None else n
            return list(range(start, stop))
        return list(range(n))[key]
    if isinstance(key, (int, np.integer)):
        return [int(key)]
    if isinstance(key, str):
        if not _is_pandas(X):
            raise ValueError("Specifying the columns using strings is only supported for pandas "
                             "DataFrames")
        return [list(X.columns).index(key)]
    key = list(key) if not isinstance(key, np.ndarray) else key
    if len(key) == 0:
        return []
    arr = np.asarray(key)
    if arr.dtype == bool:
        return list(np.flatnonzero(arr))
    if arr.dtype.kind in "iu":
        return [int(i) for i in arr]
    if not _is_pandas(X):
        raise ValueError("Specifying the columns using strings is only supported for pandas "
                         "DataFrames")
    cols = list(X.columns)
    return [cols.index(k) for k in key]


def _take(X, idx, keep_frame):
    if _is_pandas(X):
        sub = X.iloc[:, idx]
        return sub if keep_frame else sub.to_numpy()
    if sp.issparse(X):
        return X.tocsc()[:, idx].tocsr()
    return np.asarray(X)[:, idx]


class make_column_selector:
    """Callable selecting columns by name regex and/or dtype."""

    def __init__(self, pattern=None, *, dtype_include=None, dtype_exclude=None):
        self.pattern = pattern
        self.dtype_include = dtype_include
        self.dtype_exclude = dtype_exclude

    def __call__(self, df):
        if not hasattr(df, "iloc"):
            raise ValueError("make_column_selector can only be applied to pandas dataframes")
        sub = df.iloc[:1]
        if self.dtype_include is not None or self.dtype_exclude is not None:
            sub = sub.select_dtypes(include=self.dtype_include, exclude=self.dtype_exclude)
        cols = sub.columns
        if self.pattern is not None:
            cols = cols[cols.str.contains(self.pattern, regex=True)]
        return cols.tolist()


class ColumnTransformer(TransformerMixin, _BaseComposition):
    """Apply transformers to column subsets and concatenate the results."""

    def __init__(self, transformers, *, remainder="drop", sparse_threshold=0.3, n_jobs=None,
                 transformer_weights=None, verbose=False, verbose_feature_names_out=True):
        self.transformers = transformers
        self.remainder = remainder
        self.sparse_threshold = sparse_threshold
        self.n_jobs = n_jobs
        self.transformer_weights = transformer_weights
        self.verbose = verbose
        self.verbose_feature_names_out = verbose_feature_names_out

    @property
    def _transformers(self):
        return [(n, t) for n, t, _ in self.transformers]

    @_transformers.setter
    def _transformers(self, value):
        self.transformers = [(n, t, c) for (n, t), (_, _, c) in zip(value, self.transformers)]

    def get_params(self, deep=True):
        return self._get_params("_transformers", deep=deep)

    def set_params(self, **kwargs):
        self._set_params("_transformers", **kwargs)
        return self

    def _validate(self, X):
        names = [n for n, _, _ in self.transformers]
        self._validate_names(names)
        for _, t, _ in self.transformers:
            if t in ("drop", "passthrough"):
                continue
            if not (hasattr(t, "fit") or hasattr(t, "fit_transform")) or not hasattr(t, "transform"):
                raise TypeError("All estimators should implement fit and transform, or can be "
                                "'drop' or 'passthrough' specifiers. '%s' (type %s) doesn't."
                                % (t, type(t)))
        if not (self.remainder in ("drop", "passthrough") or hasattr(self.remainder, "transform")):
            raise ValueError("The remainder keyword needs to be one of 'drop', 'passthrough', or "
                             "estimator. '%s' was passed instead" % self.remainder)

    def _iter(self, X, fitted):
        trans = self.transformers_ if fitted else self.transformers
        for name, t, cols in trans:
            if fitted:
                idx = self._columns[name]
            else:
                idx = _col_indices(X, cols)
            yield name, t, cols, idx

    def _fit_transform(self, X, y, fit):
        outs, fitted = [], []
        self._columns = {}
        used = set()
        specs = list(self.transformers)
        for name, t, cols in specs:
            idx = _col_indices(X, cols)
            self._columns[name] = idx
            used.update(idx)
        rem = [i for i in range(_n_cols(X)) if i not in used]
        self._remainder = ("remainder", self.remainder, rem)
        if rem and self.remainder != "drop":
            specs = specs + [self._remainder]
            self._columns["remainder"] = rem
        for name, t, cols in specs:
            idx = self._columns[name]
            if t == "drop" or (len(idx) == 0 and t != "passthrough"):
                fitted.append((name, t, cols))
                continue
            keep_frame = isinstance(cols, (str, list)) and _is_pandas(X)
            Xs = _take(X, idx, keep_frame)
            if t == "passthrough":
                est = FunctionTransformer(accept_sparse=True, check_inverse=False,
                                          feature_names_out="one-to-one") \
                    if _ft_has_names() else FunctionTransformer(accept_sparse=True,
                                                                check_inverse=False)
                est = est.fit(Xs)
                out = Xs if not hasattr(Xs, "to_numpy") else Xs.to_numpy()
            else:
                est = clone(t)
                out = est.fit_transform(Xs, y) if hasattr(est, "fit_transform") else \
                    est.fit(Xs, y).transform(Xs)
            w = (self.transformer_weights or {}).get(name)
            if w is not None:
                out = out * w
            outs.append(out)
            fitted.append((name, est, cols))
        self.transformers_ = [f for f in fitted if f[0] != "remainder"]
        if rem and self.remainder != "drop":
            self.transformers_.append(next(f for f in fitted if f[0] == "remainder"))
        else:
            self.transformers_.append(("remainder", self.remainder, rem))
        self._out_widths = [o.shape[1] for o in outs]
        return self._hstack(outs, X.shape[0])

    def _hstack(self, outs, n):
        if not outs:
            return np.zeros((n, 0))
        if any(sp.issparse(o) for o in outs):
            nnz = sum(o.nnz if sp.issparse(o) else np.count_nonzero(o) for o in outs)
            total = sum(o.shape[0] * o.shape[1] for o in outs)
            density = nnz / total if total else 0
            self.sparse_output_ = density < self.sparse_threshold
        else:
            self.sparse_output_ = False
        if self.sparse_output_:
            return sp.hstack([sp.csr_matrix(o) for o in outs]).tocsr()
        return np.hstack([o.toarray() if sp.issparse(o) else np.asarray(o) for o in outs])

    def fit(self, X, y=None):
        self.fit_transform(X, y)
        return self

    def fit_transform(self, X, y=None):
        self._validate(X)
        self.n_features_in_ = _n_cols(X)
        if _is_pandas(X):
            self.feature_names_in_ = np.asarray(X.columns, dtype=object)
        return self._fit_transform(X, y, True)

    def transform(self, X):
        check_is_fitted(self, "transformers_")
        if _n_cols(X) != self.n_features_in_ and not _is_pandas(X):
            raise ValueError("X has %d features, but ColumnTransformer is expecting %d features "
                             "as input." % (_n_cols(X), self.n_features_in_))
        outs = []
        for name, est, cols in self.transformers_:
            idx = self._columns.get(name, [])
            if est == "drop" or len(idx) == 0:
                continue
            if _is_pandas(X) and hasattr(self, "feature_names_in_"):
                names = list(self.feature_names_in_[idx])
                Xs = X[names] if isinstance(cols, (str, list)) else X[names].to_numpy()
            else:
                Xs = _take(X, idx, False)
            out = est.transform(Xs)
            if hasattr(out, "to_numpy"):
                out = out.to_numpy()
            w = (self.transformer_weights or {}).get(name)
            if w is not None:
                out = out * w
            outs.append(out)
        return self._hstack(outs, X.shape[0])

    @property
    def named_transformers_(self):
        return {n: t for n, t, _ in self.transformers_}

    def get_feature_names_out(self, input_features=None):
        check_is_fitted(self, "transformers_")
        names_in = getattr(self, "feature_names_in_",
                           np.array(["x%d" % i for i in range(self.n_features_in_)], dtype=object))
        out = []
        for name, est, _ in self.transformers_:
            idx = self._columns.get(name, [])
            if est == "drop" or len(idx) == 0:
                continue
            sub = names_in[idx]
            if hasattr(est, "get_feature_names_out"):
                try:
                    sub = est.get_feature_names_out(sub)
                except TypeError:
                    sub = est.get_feature_names_out()
            elif not isinstance(est, FunctionTransformer):
                raise AttributeError("Transformer %s (type %s) does not provide "
                                     "get_feature_names_out." % (name, type(est).__name__))
            out += ["%s__%s" % (name, s) if self.verbose_feature_names_out else str(s)
                    for s in sub]
        return np.asarray(out, dtype=object)


def _ft_has_names():
    import inspect
    return "feature_names_out" in inspect.signature(FunctionTransformer.__init__).parameters


def make_column_transformer(*transformers, remainder="drop", sparse_threshold=0.3, n_jobs=None,
                            verbose=False, verbose_feature_names_out=True):
    trans, cols = zip(*transformers)
    names = [n for n, _ in _name_estimators(trans)]
    return ColumnTransformer(list(zip(names, trans, cols)), n_jobs=n_jobs, remainder=remainder,
                             sparse_threshold=sparse_threshold, verbose=verbose,
                             verbose_feature_names_out=verbose_feature_names_out)


class TransformedTargetRegressor(RegressorMixin, BaseEstimator):
    """Fit a regressor on transformed targets; predictions are mapped back."""

    def __init__(self, regressor=None, *, transformer=None, func=None, inverse_func=None,
                 check_inverse=True):
        self.regressor = regressor
        self.transformer = transformer
        self.func = func
        self.inverse_func = inverse_func
        self.check_inverse = check_inverse

    def _fit_transformer(self, y):
        if self.transformer is not None and (self.func is not None
                                             or self.inverse_func is not None):
            raise ValueError("'transformer' and functions 'func'/'inverse_func' cannot both be "
                             "set.")
        if self.transformer is not None:
            self.transformer_ = clone(self.transformer)
        else:
            if self.func is not None and self.inverse_func is None:
                raise ValueError("When 'func' is provided, 'inverse_func' must also be provided")
            self.transformer_ = FunctionTransformer(func=self.func,
                                                    inverse_func=self.inverse_func,
                                                    validate=True,
                                                    check_inverse=self.check_inverse)
        self.transformer_.fit(y)
        if self.check_inverse:
            idx = slice(None, None, max(1, y.shape[0] // 10))
            ys = y[idx]
            back = self.transformer_.inverse_transform(self.transformer_.transform(ys))
            if not np.allclose(ys, np.asarray(back).reshape(ys.shape)):
                import warnings
                warnings.warn("The provided functions or transformer are not strictly inverse of "
                              "each other. If you are sure you want to proceed regardless, set "
                              "'check_inverse=False'", UserWarning)

    def fit(self, X, y, **fit_params):
        y = np.asarray(y, dtype=np.float64)
        self._training_dim = y.ndim
        y2 = y.reshape(-1, 1) if y.ndim == 1 else y
        self._fit_transformer(y2)
        yt = np.asarray(self.transformer_.transform(y2))
        if yt.ndim == 2 and yt.shape[1] == 1:
            yt = yt.ravel()
        if self.regressor is None:
            from .linear_model import LinearRegression
            self.regressor_ = LinearRegression()
        else:
            self.regressor_ = clone(self.regressor)
        self.regressor_.fit(X, yt, **fit_params)
        if hasattr(self.regressor_, "n_features_in_"):
            self.n_features_in_ = self.regressor_.n_features_in_
        return self

    def predict(self, X, **predict_params):
        check_is_fitted(self)
        pred = np.asarray(self.regressor_.predict(X, **predict_params))
        p2 = pred.reshape(-1, 1) if pred.ndim == 1 else pred
        out = np.asarray(self.transformer_.inverse_transform(p2))
        if self._training_dim == 1 and out.ndim == 2 and out.shape[1] == 1:
            out = out.ravel()
        return out


__all__ = ["ColumnTransformer", "make_column_transformer", "make_column_selector",
           "TransformedTargetRegressor"]

from .utils._aliases import alias_submodules  # noqa: E402
alias_submodules(__name__, "_column_transformer", "_target")
