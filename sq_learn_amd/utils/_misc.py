"""Public array utilities of the reference ``sklearn.utils`` namespace
(``utils/__init__.py``: resample / shuffle / safe indexing / masks,
``utils/validation.py`` helpers, ``utils/deprecation.py``)."""

import functools
import numbers
import warnings

import numpy as np
import scipy.sparse as sp

from .validation import check_array, check_consistent_length, check_random_state


def _safe_indexing(X, indices, *, axis=0):
    """Rows (axis=0) or columns (axis=1) of an array, sparse matrix,
    dataframe or list."""
    if indices is None:
        return X
    if hasattr(X, "iloc"):
        return X.iloc[indices] if axis == 0 else X.iloc[:, indices]
    if hasattr(X, "shape"):
        idx = np.asarray(indices)
        return X[idx] if axis == 0 else X[:, idx]
    idx = np.asarray(indices)
    if idx.dtype == bool:
        idx = np.flatnonzero(idx)
    return [X[i] for i in idx]


def resample(*arrays, replace=True, n_samples=None, random_state=None, stratify=None):
    """Bootstrap / subsample arrays consistently (reference
    ``utils/__init__.py`` ``resample``)."""
    from ..model_selection._split import _approximate_mode
    max_n = n_samples
    rs = check_random_state(random_state)
    if len(arrays) == 0:
        return None
    first = arrays[0]
    n = first.shape[0] if hasattr(first, "shape") else len(first)
    if max_n is None:
        max_n = n
    elif max_n > n and not replace:
        raise ValueError("Cannot sample %d out of arrays with dim %d when replace is False"
                         % (max_n, n))
    check_consistent_length(*arrays)
    if stratify is None:
        if replace:
            indices = rs.randint(0, n, size=(max_n,))
        else:
            indices = np.arange(n)
            rs.shuffle(indices)
            indices = indices[:max_n]
    else:
        y = np.asarray(stratify)
        if y.ndim == 2:
            y = np.array([" ".join(row.astype("str")) for row in y])
        classes, y_idx = np.unique(y, return_inverse=True)
        counts = np.bincount(y_idx)
        cls_idx = np.split(np.argsort(y_idx, kind="mergesort"), np.cumsum(counts)[:-1])
        n_i = _approximate_mode(counts, max_n, rs)
        indices = []
        for i in range(len(classes)):
            indices.extend(rs.choice(cls_idx[i], n_i[i], replace=replace))
        indices = rs.permutation(indices)
    arrays = [a.tocsr() if sp.issparse(a) else a for a in arrays]
    out = [_safe_indexing(a, indices) for a in arrays]
    return out[0] if len(out) == 1 else out


def shuffle(*arrays, random_state=None, n_samples=None):
    """Consistent permutation of several arrays."""
    return resample(*arrays, replace=False, n_samples=n_samples, random_state=random_state)


def safe_mask(X, mask):
    mask = np.asarray(mask)
    if np.issubdtype(mask.dtype, np.signedinteger):
        return mask
    if hasattr(X, "toarray"):
        mask = np.arange(mask.shape[0])[mask]
    return mask


def safe_sqr(X, *, copy=True):
    if sp.issparse(X):
        X = X.copy() if copy else X
        X.data **= 2
        return X
    return X ** 2 if copy else np.power(X, 2, out=X)


def indexable(*iterables):
    out = []
    for X in iterables:
        if sp.issparse(X):
            out.append(X.tocsr())
        elif hasattr(X, "__getitem__") or hasattr(X, "iloc") or X is None:
            out.append(X)
        else:
            out.append(np.array(X))
    check_consistent_length(*out)
    return out


def as_float_array(X, *, copy=True, force_all_finite=True):
    if sp.issparse(X):
        return X.astype(np.float64) if X.dtype.kind not in "f" else (X.copy() if copy else X)
    X = np.asarray(X)
    if X.dtype.kind == "f":
        return X.copy() if copy else X
    dt = np.float32 if X.dtype in (np.int8, np.int16, np.uint8, np.uint16) else np.float64
    return X.astype(dt)


def assert_all_finite(X, *, allow_nan=False):
    data = X.data if sp.issparse(X) else np.asarray(X)
    if data.dtype.kind in "fc":
        bad = np.isinf(data).any() if allow_nan else not np.isfinite(data).all()
        if bad:
            raise ValueError("Input contains %s." % ("infinity or a value too large for %r"
                                                     % data.dtype if allow_nan or
                                                     not np.isnan(data).any() else "NaN"))


def check_symmetric(array, *, tol=1e-10, raise_warning=True, raise_exception=False):
    if array.ndim != 2 or array.shape[0] != array.shape[1]:
        raise ValueError("array must be 2-dimensional and square. shape = {0}"
                         .format(array.shape))
    if sp.issparse(array):
        diff = array - array.T
        sym = np.all(abs(diff.data) < tol) if diff.format in ("csr", "csc", "coo") else \
            np.all(abs(diff.tocsr().data) < tol)
    else:
        sym = np.allclose(array, array.T, atol=tol)
    if not sym:
        if raise_exception:
            raise ValueError("Array must be symmetric")
        if raise_warning:
            warnings.warn("Array is not symmetric, and will be converted to symmetric by "
                          "average with its transpose.", stacklevel=2)
        array = 0.5 * (array + array.T)
        if sp.issparse(array):
            array = array.asformat(array.format)
    return array


class deprecated:
    """Decorator marking a function or class as deprecated."""

    def __init__(self, extra=""):
        self.extra = extra

    def __call__(self, obj):
        msg = "%s is deprecated" % getattr(obj, "__name__", "object")
        if self.extra:
            msg += "; %s" % self.extra
        if isinstance(obj, type):
            init = obj.__init__

            @functools.wraps(init)
            def wrapped(*a, **k):
                warnings.warn(msg, category=FutureWarning)
                return init(*a, **k)
            obj.__init__ = wrapped
            return obj

        @functools.wraps(obj)
        def wrapped(*a, **k):
            warnings.warn(msg, category=FutureWarning)
            return obj(*a, **k)
        return wrapped


def is_scalar_nan(x):
    return isinstance(x, numbers.Real) and np.isnan(x)


__all__ = ["resample", "shuffle", "safe_mask", "safe_sqr", "indexable", "as_float_array",
           "assert_all_finite", "check_symmetric", "deprecated", "is_scalar_nan", "check_array"]
