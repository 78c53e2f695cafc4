"""Categorical / label encoders (reference ``preprocessing/_encoders.py``:
OneHotEncoder, OrdinalEncoder; ``preprocessing/_label.py``: LabelEncoder,
LabelBinarizer, label_binarize, MultiLabelBinarizer)."""

import numbers

import numpy as np
import scipy.sparse as sp

from ..base import BaseEstimator, TransformerMixin
from ..utils.validation import check_is_fitted


def _to_2d_object(X):
    if hasattr(X, "iloc"):
        X = X.values
    X = np.asarray(X.detach().cpu().numpy() if hasattr(X, "detach") else X)
    if X.ndim != 2:
        raise ValueError("Expected 2D array, got %dD array instead" % X.ndim)
    return X


def _unique_sorted(col):
    if col.dtype.kind == "O":
        vals = sorted(set(col.tolist()), key=lambda v: (str(type(v)), v))
        return np.array(vals, dtype=object)
    return np.unique(col)


def _encode(col, cats, handle_unknown):
    idx = np.searchsorted(cats, col) if cats.dtype.kind != "O" else None
    if idx is None:
        lookup = {v: i for i, v in enumerate(cats.tolist())}
        codes = np.array([lookup.get(v, -1) for v in col.tolist()], dtype=np.int64)
    else:
        idx = np.clip(idx, 0, max(len(cats) - 1, 0))
        codes = np.where(cats[idx] == col, idx, -1) if len(cats) else np.full(len(col), -1)
    unknown = codes < 0
    if unknown.any() and handle_unknown == "error":
        raise ValueError("Found unknown categories {} during transform"
                         .format(list(np.unique(col[unknown]))))
    return codes, unknown


class _BaseEncoder(TransformerMixin, BaseEstimator):
    def _fit_categories(self, X):
        X = _to_2d_object(X)
        self.n_features_in_ = X.shape[1]
        if isinstance(self.categories, str) and self.categories == "auto":
            self.categories_ = [_unique_sorted(X[:, j]) for j in range(X.shape[1])]
        else:
            if len(self.categories) != X.shape[1]:
                raise ValueError("Shape mismatch: if categories is an array, it has to be of "
                                 "shape (n_features,).")
            self.categories_ = [np.asarray(c) for c in self.categories]
            if self.handle_unknown == "error":
                for j, c in enumerate(self.categories_):
                    diff = set(np.unique(X[:, j]).tolist()) - set(c.tolist())
                    if diff:
                        raise ValueError("Found unknown categories {} in column {} during fit"
                                         .format(sorted(diff, key=str), j))
        return X

    def _transform_codes(self, X):
        X = _to_2d_object(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError(f"X has {X.shape[1]} features, but {type(self).__name__} is "
                             f"expecting {self.n_features_in_} features as input.")
        codes = np.empty(X.shape, dtype=np.int64)
        unknown = np.zeros(X.shape, dtype=bool)
        hu = "error" if self.handle_unknown == "error" else "ignore"
        for j, c in enumerate(self.categories_):
            codes[:, j], unknown[:, j] = _encode(X[:, j], c, hu)
        return codes, unknown


class OneHotEncoder(_BaseEncoder):

    def _more_tags(self):
        return {"allow_nan": True}

    def __init__(self, *, categories="auto", drop=None, sparse=True, dtype=np.float64,
                 handle_unknown="error"):
        self.categories = categories
        self.drop = drop
        self.sparse = sparse
        self.dtype = dtype
        self.handle_unknown = handle_unknown

    def fit(self, X, y=None):
        if self.handle_unknown not in ("error", "ignore"):
            raise ValueError("handle_unknown should be either 'error' or 'ignore', got {0}."
                             .format(self.handle_unknown))
        self._fit_categories(X)
        self.drop_idx_ = self._compute_drop_idx()
        return self

    def _compute_drop_idx(self):
        if self.drop is None:
            return None
        if isinstance(self.drop, str):
            if self.drop == "first":
                return np.zeros(len(self.categories_), dtype=object)
            if self.drop == "if_binary":
                return np.array([0 if len(c) == 2 else None for c in self.categories_],
                                dtype=object)
            raise ValueError("Wrong input for parameter `drop`. Expected 'first', 'if_binary', "
                             "None or array of objects, got {}".format(self.drop))
        out = []
        for c, v in zip(self.categories_, self.drop):
            hit = np.where(c == v)[0]
            if not len(hit):
                raise ValueError("The following categories were supposed to be dropped, but "
                                 "were not found in the training data.")
            out.append(hit[0])
        return np.array(out, dtype=object)

    def _sizes(self):
        sizes = [len(c) for c in self.categories_]
        if self.drop_idx_ is not None:
            sizes = [s - (0 if d is None else 1) for s, d in zip(sizes, self.drop_idx_)]
        return sizes

    def transform(self, X):
        check_is_fitted(self)
        codes, unknown = self._transform_codes(X)
        n = codes.shape[0]
        sizes = self._sizes()
        offs = np.concatenate([[0], np.cumsum(sizes)])
        rows, cols = [], []
        for j in range(codes.shape[1]):
            c = codes[:, j].copy()
            keep = ~unknown[:, j]
            if self.drop_idx_ is not None and self.drop_idx_[j] is not None:
                d = int(self.drop_idx_[j])
                keep &= c != d
                c = np.where(c > d, c - 1, c)
            r = np.where(keep)[0]
            rows.append(r)
            cols.append(c[keep] + offs[j])
        r = np.concatenate(rows) if rows else np.zeros(0, dtype=np.int64)
        cc = np.concatenate(cols) if cols else np.zeros(0, dtype=np.int64)
        out = sp.csr_matrix((np.ones(len(r), dtype=self.dtype), (r, cc)), shape=(n, offs[-1]))
        out.sort_indices()
        return out if self.sparse else out.toarray()

    def inverse_transform(self, X):
        check_is_fitted(self)
        X = X.toarray() if sp.issparse(X) else np.asarray(X)
        sizes = self._sizes()
        out = np.empty((X.shape[0], len(sizes)), dtype=object)
        j0 = 0
        for j, s in enumerate(sizes):
            block = X[:, j0:j0 + s]
            cats = self.categories_[j]
            if self.drop_idx_ is not None and self.drop_idx_[j] is not None:
                keep = np.delete(np.arange(len(cats)), int(self.drop_idx_[j]))
                lab = np.where(block.sum(1) == 0, int(self.drop_idx_[j]),
                               keep[np.argmax(block, axis=1)] if s else 0)
            else:
                lab = np.argmax(block, axis=1)
            vals = cats[lab].astype(object)
            if self.handle_unknown == "ignore" and (self.drop_idx_ is None
                                                    or self.drop_idx_[j] is None):
                vals[block.sum(1) == 0] = None
            out[:, j] = vals
            j0 += s
        try:
            return out.astype(np.result_type(*[c.dtype for c in self.categories_]))
        except (TypeError, ValueError):
            return out

    def get_feature_names(self, input_features=None):
        check_is_fitted(self)
        input_features = input_features or ["x%d" % i for i in range(len(self.categories_))]
        names = []
        for j, cats in enumerate(self.categories_):
            for k, c in enumerate(cats):
                if self.drop_idx_ is not None and self.drop_idx_[j] is not None and \
                        k == int(self.drop_idx_[j]):
                    continue
                names.append("%s_%s" % (input_features[j], c))
        return np.array(names, dtype=object)

    get_feature_names_out = get_feature_names


class OrdinalEncoder(_BaseEncoder):

    def _more_tags(self):
        return {"allow_nan": True}

    def __init__(self, *, categories="auto", dtype=np.float64, handle_unknown="error",
                 unknown_value=None):
        self.categories = categories
        self.dtype = dtype
        self.handle_unknown = handle_unknown
        self.unknown_value = unknown_value

    def fit(self, X, y=None):
        if self.handle_unknown not in ("error", "use_encoded_value"):
            raise ValueError("handle_unknown should be either 'error' or 'use_encoded_value', "
                             "got {}.".format(self.handle_unknown))
        if self.handle_unknown == "use_encoded_value" and not (
                isinstance(self.unknown_value, numbers.Integral) or
                (isinstance(self.unknown_value, float) and np.isnan(self.unknown_value))):
            raise TypeError("unknown_value should be an integer or np.nan when "
                            "handle_unknown is 'use_encoded_value', got {}."
                            .format(self.unknown_value))
        self._fit_categories(X)
        return self

    def transform(self, X):
        check_is_fitted(self)
        codes, unknown = self._transform_codes(X)
        out = codes.astype(self.dtype)
        if unknown.any():
            out[unknown] = self.unknown_value
        return out

    def inverse_transform(self, X):
        X = np.asarray(X)
        out = np.empty(X.shape, dtype=object)
        for j, c in enumerate(self.categories_):
            col = X[:, j]
            bad = ~np.isfinite(col.astype(float)) | (col < 0)
            idx = np.where(bad, 0, col).astype(np.int64)
            vals = c[idx].astype(object)
            vals[bad] = None
            out[:, j] = vals
        return out


class LabelEncoder(TransformerMixin, BaseEstimator):

    def _more_tags(self):
        return {"X_types": ["1dlabels"]}

    def fit(self, y):
        self.classes_ = _unique_sorted(np.asarray(y).ravel())
        return self

    def fit_transform(self, y):
        return self.fit(y).transform(y)

    def transform(self, y):
        check_is_fitted(self)
        y = np.asarray(y).ravel()
        if len(y) == 0:
            return np.array([], dtype=np.int64)
        codes, unknown = _encode(y, self.classes_, "ignore")
        if unknown.any():
            raise ValueError("y contains previously unseen labels: %s"
                             % str(list(np.unique(y[unknown]))))
        return codes

    def inverse_transform(self, y):
        check_is_fitted(self)
        y = np.asarray(y)
        if len(y) == 0:
            return np.array([])
        diff = np.setdiff1d(y, np.arange(len(self.classes_)))
        if len(diff):
            raise ValueError("y contains previously unseen labels: %s" % str(diff))
        return self.classes_[y]


def label_binarize(y, *, classes, neg_label=0, pos_label=1, sparse_output=False):
    y = np.asarray(y)
    classes = np.asarray(classes)
    if neg_label >= pos_label:
        raise ValueError("neg_label={0} must be strictly less than pos_label={1}."
                         .format(neg_label, pos_label))
    multilabel = y.ndim == 2 and y.shape[1] > 1
    if multilabel:
        Y = (y != 0).astype(int)
        out = np.where(Y == 1, pos_label, neg_label)
        return sp.csr_matrix(out) if sparse_output else out
    y = y.ravel()
    n_classes = len(classes)
    if n_classes == 1:
        out = np.full((len(y), 1), neg_label)
        if sparse_output:
            return sp.csr_matrix(out)
        return out
    if n_classes == 2:
        out = np.where(y == classes[1], pos_label, neg_label).reshape(-1, 1)
        return sp.csr_matrix(out) if sparse_output else out
    codes, unknown = _encode(y, np.sort(classes) if classes.dtype.kind != "O" else classes,
                             "ignore")
    sorted_cls = np.sort(classes) if classes.dtype.kind != "O" else classes
    order = np.searchsorted(sorted_cls, classes) if classes.dtype.kind != "O" else \
        np.arange(n_classes)
    out = np.full((len(y), n_classes), neg_label)
    inv = np.empty(n_classes, dtype=np.int64)
    inv[order] = np.arange(n_classes)
    ok = ~unknown
    out[np.where(ok)[0], inv[codes[ok]]] = pos_label
    return sp.csr_matrix(out) if sparse_output else out


class LabelBinarizer(TransformerMixin, BaseEstimator):

    def _more_tags(self):
        return {"X_types": ["1dlabels"]}

    def __init__(self, *, neg_label=0, pos_label=1, sparse_output=False):
        self.neg_label = neg_label
        self.pos_label = pos_label
        self.sparse_output = sparse_output

    def fit(self, y):
        y = np.asarray(y)
        self.y_type_ = ("multilabel-indicator" if y.ndim == 2 and y.shape[1] > 1 else
                        ("binary" if len(np.unique(y)) <= 2 else "multiclass"))
        self.classes_ = (np.arange(y.shape[1]) if self.y_type_ == "multilabel-indicator"
                         else _unique_sorted(y.ravel()))
        return self

    def fit_transform(self, y):
        return self.fit(y).transform(y)

    def transform(self, y):
        check_is_fitted(self)
        return label_binarize(y, classes=self.classes_, neg_label=self.neg_label,
                              pos_label=self.pos_label, sparse_output=self.sparse_output)

    def inverse_transform(self, Y, threshold=None):
        check_is_fitted(self)
        Y = Y.toarray() if sp.issparse(Y) else np.asarray(Y)
        if threshold is None:
            threshold = (self.pos_label + self.neg_label) / 2.0
        if self.y_type_ == "multilabel-indicator":
            return (Y > threshold).astype(int)
        if self.y_type_ == "binary" or Y.shape[1] == 1:
            return self.classes_[(Y.ravel() > threshold).astype(int)]
        return self.classes_[np.argmax(Y, axis=1)]


class MultiLabelBinarizer(TransformerMixin, BaseEstimator):

    def _more_tags(self):
        return {"X_types": ["2dlabels"]}

    def __init__(self, *, classes=None, sparse_output=False):
        self.classes = classes
        self.sparse_output = sparse_output

    def fit(self, y):
        if self.classes is None:
            cls = sorted(set(v for row in y for v in row))
        else:
            cls = list(self.classes)
        self.classes_ = np.empty(len(cls), dtype=object if any(isinstance(c, str) for c in cls)
                                 else int)
        self.classes_[:] = cls
        return self

    def fit_transform(self, y):
        return self.fit(y).transform(y)

    def transform(self, y):
        check_is_fitted(self)
        lookup = {c: i for i, c in enumerate(self.classes_.tolist())}
        rows, cols = [], []
        for i, row in enumerate(y):
            for v in set(row):
                if v in lookup:
                    rows.append(i)
                    cols.append(lookup[v])
        out = sp.csr_matrix((np.ones(len(rows), dtype=int), (rows, cols)),
                            shape=(len(y), len(self.classes_)))
        return out if self.sparse_output else out.toarray()

    def inverse_transform(self, yt):
        yt = yt.toarray() if sp.issparse(yt) else np.asarray(yt)
        return [tuple(self.classes_[np.flatnonzero(r)]) for r in yt]
