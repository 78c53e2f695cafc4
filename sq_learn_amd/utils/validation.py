"""Input validation (reference ``sklearn/utils/validation.py``:
``check_array`` :462, ``check_X_y`` :765, ``check_random_state`` :926,
``check_is_fitted`` :1035, ``_check_sample_weight`` :1333).

Accepts NumPy arrays, array-likes and torch tensors.  Tensors stay tensors
(and stay on their device: a 10M-row shard on an MI355X is never copied to
the host for validation); everything else becomes a NumPy array.
"""

import numbers
import warnings

import numpy as np
import torch

from .._config import get_config
from ..exceptions import NotFittedError, DataConversionWarning

_FLOAT_TORCH = (torch.float64, torch.float32, torch.bfloat16, torch.float16)


def _num_samples(x):
    if hasattr(x, "shape") and len(x.shape) > 0:
        return int(x.shape[0])
    if hasattr(x, "__len__"):
        return len(x)
    raise TypeError(f"Expected sequence or array-like, got {type(x)}")


def _assert_all_finite(X, allow_nan=False):
    if get_config()["assume_finite"]:
        return
    if isinstance(X, torch.Tensor):
        if not X.is_floating_point():
            return
        bad = ~torch.isfinite(X) if not allow_nan else torch.isinf(X)
        if bool(bad.any()):
            raise ValueError("Input contains NaN, infinity or a value too large for "
                             f"dtype('{X.dtype}').")
        return
    X = np.asarray(X)
    if X.dtype.kind in "fc":
        ok = np.isfinite(X).all() if not allow_nan else not np.isinf(X).any()
        if not ok:
            raise ValueError("Input contains NaN, infinity or a value too large for "
                             f"dtype('{X.dtype}').")


def _np_dtype_of(d):
    if d in ("numeric",):
        return d
    return d


def check_array(array, accept_sparse=False, *, accept_large_sparse=True, dtype="numeric",
                order=None, copy=False, force_all_finite=True, ensure_2d=True,
                allow_nd=False, ensure_min_samples=1, ensure_min_features=1,
                estimator=None):
    """Validate an array / tensor.  ``dtype`` may be 'numeric', None, a dtype
    or a list of acceptable dtypes (the first is used for conversion)."""
    try:
        import scipy.sparse as sp
        if sp.issparse(array):
            if not accept_sparse:
                raise TypeError("A sparse matrix was passed, but dense data is required. "
                                "Use X.toarray() to convert to a dense numpy array.")
            return array
    except ImportError:  # pragma: no cover
        pass

    if isinstance(array, torch.Tensor):
        t = array
        if dtype == "numeric":
            if not (t.is_floating_point() or t.dtype in (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool)):
                raise ValueError(f"Unsupported tensor dtype {t.dtype}")
        elif dtype is not None:
            wanted = dtype if isinstance(dtype, (list, tuple)) else [dtype]
            tw = [_to_torch_dtype(w) for w in wanted]
            if t.dtype not in tw:
                t = t.to(tw[0])
                copy = False
        if ensure_2d:
            if t.ndim == 0:
                raise ValueError(f"Expected 2D array, got scalar array instead:\narray={t}.")
            if t.ndim == 1:
                raise ValueError("Expected 2D array, got 1D array instead. Reshape your data "
                                 "either using array.reshape(-1, 1) if your data has a single "
                                 "feature or array.reshape(1, -1) if it contains a single sample.")
        if not allow_nd and t.ndim >= 3:
            raise ValueError(f"Found array with dim {t.ndim}. Expected <= 2.")
        if force_all_finite:
            _assert_all_finite(t, allow_nan=force_all_finite == "allow-nan")
        _check_min(t, ensure_min_samples, ensure_min_features, ensure_2d)
        if order == "C" and not t.is_contiguous():
            t = t.contiguous()
            copy = False
        return t.clone() if copy else t

    # numpy / array-like
    dtype_orig = getattr(array, "dtype", None)
    if not hasattr(dtype_orig, "kind"):
        dtype_orig = None
    if dtype == "numeric":
        dtype_target = np.float64 if (dtype_orig is not None and dtype_orig.kind == "O") else None
    elif isinstance(dtype, (list, tuple)):
        if dtype_orig is not None and any(np.dtype(d) == dtype_orig for d in dtype if not isinstance(d, torch.dtype)):
            dtype_target = None
        else:
            dtype_target = dtype[0]
    else:
        dtype_target = dtype
    if isinstance(dtype_target, torch.dtype):
        dtype_target = {torch.float64: np.float64, torch.float32: np.float32}.get(dtype_target, np.float32)
    with warnings.catch_warnings():
        try:
            arr = np.asarray(array, order=order, dtype=dtype_target)
        except ComplexWarning:  # pragma: no cover
            raise ValueError(f"Complex data not supported\n{array}\n")
    if arr.dtype.kind == "c":
        raise ValueError(f"Complex data not supported\n{array}\n")
    if ensure_2d:
        if arr.ndim == 0:
            raise ValueError(f"Expected 2D array, got scalar array instead:\narray={array}.\n"
                             "Reshape your data either using array.reshape(-1, 1) if your data "
                             "has a single feature or array.reshape(1, -1) if it contains a single sample.")
        if arr.ndim == 1:
            raise ValueError(f"Expected 2D array, got 1D array instead:\narray={array}.\n"
                             "Reshape your data either using array.reshape(-1, 1) if your data "
                             "has a single feature or array.reshape(1, -1) if it contains a single sample.")
    if dtype == "numeric" and arr.dtype.kind in "USV":
        raise ValueError("dtype='numeric' is not compatible with arrays of bytes/strings.")
    if not allow_nd and arr.ndim >= 3:
        raise ValueError(f"Found array with dim {arr.ndim}. Expected <= 2.")
    if force_all_finite and arr.dtype.kind in "fc":
        _assert_all_finite(arr, allow_nan=force_all_finite == "allow-nan")
    _check_min(arr, ensure_min_samples, ensure_min_features, ensure_2d)
    if copy and np.may_share_memory(arr, array):
        arr = np.array(arr, order=order, copy=True)
    return arr


class ComplexWarning(Warning):
    pass


def _check_min(a, ensure_min_samples, ensure_min_features, ensure_2d):
    if ensure_min_samples > 0 and a.ndim >= 1:
        n = a.shape[0]
        if n < ensure_min_samples:
            raise ValueError(f"Found array with {n} sample(s) (shape={tuple(a.shape)}) while a "
                             f"minimum of {ensure_min_samples} is required.")
    if ensure_min_features > 0 and a.ndim == 2 and ensure_2d:
        f = a.shape[1]
        if f < ensure_min_features:
            raise ValueError(f"Found array with {f} feature(s) (shape={tuple(a.shape)}) while a "
                             f"minimum of {ensure_min_features} is required.")


def _to_torch_dtype(d):
    if isinstance(d, torch.dtype):
        return d
    return {np.dtype(np.float64): torch.float64, np.dtype(np.float32): torch.float32,
            np.dtype(np.int64): torch.int64, np.dtype(np.int32): torch.int32}[np.dtype(d)]


def column_or_1d(y, *, warn=False):
    if isinstance(y, torch.Tensor):
        if y.ndim == 1:
            return y
        if y.ndim == 2 and y.shape[1] == 1:
            if warn:
                warnings.warn("A column-vector y was passed when a 1d array was expected.",
                              DataConversionWarning, stacklevel=2)
            return y.reshape(-1)
        raise ValueError(f"y should be a 1d array, got an array of shape {tuple(y.shape)} instead.")
    y = np.asarray(y)
    if y.ndim == 1:
        return y
    if y.ndim == 2 and y.shape[1] == 1:
        if warn:
            warnings.warn("A column-vector y was passed when a 1d array was expected.",
                          DataConversionWarning, stacklevel=2)
        return np.ravel(y)
    raise ValueError(f"y should be a 1d array, got an array of shape {y.shape} instead.")


def check_consistent_length(*arrays):
    lengths = [_num_samples(x) for x in arrays if x is not None]
    if len(set(lengths)) > 1:
        raise ValueError("Found input variables with inconsistent numbers of samples: "
                         f"{[int(v) for v in lengths]}")


def check_X_y(X, y, accept_sparse=False, *, dtype="numeric", order=None, copy=False,
              force_all_finite=True, ensure_2d=True, allow_nd=False, multi_output=False,
              ensure_min_samples=1, ensure_min_features=1, y_numeric=False, estimator=None,
              **_ignored):
    if y is None:
        raise ValueError("y cannot be None")
    X = check_array(X, accept_sparse=accept_sparse, dtype=dtype, order=order, copy=copy,
                    force_all_finite=force_all_finite, ensure_2d=ensure_2d, allow_nd=allow_nd,
                    ensure_min_samples=ensure_min_samples, ensure_min_features=ensure_min_features)
    if multi_output:
        y = check_array(y, dtype=None, ensure_2d=False, force_all_finite=True)
    else:
        y = column_or_1d(y, warn=True)
        if not isinstance(y, torch.Tensor):
            _assert_all_finite(y) if y.dtype.kind in "fc" else None
    if y_numeric and not isinstance(y, torch.Tensor) and y.dtype.kind == "O":
        y = y.astype(np.float64)
    check_consistent_length(X, y)
    return X, y


def check_random_state(seed):
    """numpy RandomState from None / int / RandomState (reference :926)."""
    if seed is None or seed is np.random:
        return np.random.mtrand._rand
    if isinstance(seed, numbers.Integral):
        return np.random.RandomState(seed)
    if isinstance(seed, np.random.RandomState):
        return seed
    if isinstance(seed, np.random.Generator):
        return np.random.RandomState(seed.integers(0, 2 ** 31 - 1))
    raise ValueError(f"{seed!r} cannot be used to seed a numpy.random.RandomState instance")


def seed_from_random_state(random_state):
    """Integer seed for the counter-based stochastic layer.

    ``int`` -> that int; ``None`` -> the global config seed; a RandomState ->
    one draw from it (so the estimator stays reproducible w.r.t. it)."""
    if random_state is None:
        return get_config()["seed"]
    if isinstance(random_state, numbers.Integral):
        return int(random_state) & ((1 << 64) - 1)
    rs = check_random_state(random_state)
    return int(rs.randint(0, 2 ** 31 - 1))


def check_is_fitted(estimator, attributes=None, *, msg=None, all_or_any=all):
    if isinstance(estimator, type):
        raise TypeError(f"{estimator} is a class, not an instance.")
    if msg is None:
        msg = ("This %(name)s instance is not fitted yet. Call 'fit' with appropriate "
               "arguments before using this estimator.")
    if not hasattr(estimator, "fit"):
        raise TypeError(f"{estimator} is not an estimator instance.")
    if attributes is not None:
        if not isinstance(attributes, (list, tuple)):
            attributes = [attributes]
        fitted = all_or_any([hasattr(estimator, a) for a in attributes])
    else:
        fitted = [v for v in vars(estimator) if v.endswith("_") and not v.startswith("__")]
    if not fitted:
        raise NotFittedError(msg % {"name": type(estimator).__name__})


def _check_sample_weight(sample_weight, X, dtype=None, copy=False):
    n = _num_samples(X)
    if isinstance(X, torch.Tensor):
        dt = X.dtype if X.is_floating_point() else torch.float64
        if dt in (torch.bfloat16, torch.float16):
            dt = torch.float32
        if sample_weight is None:
            return torch.ones(n, dtype=dt, device=X.device)
        if isinstance(sample_weight, numbers.Number):
            return torch.full((n,), float(sample_weight), dtype=dt, device=X.device)
        sw = torch.as_tensor(sample_weight, dtype=dt, device=X.device).reshape(-1)
        if sw.shape[0] != n:
            raise ValueError(f"sample_weight.shape == {tuple(sw.shape)}, expected ({n},)!")
        return sw.clone() if copy else sw
    if dtype is None:
        dtype = [np.float64, np.float32]
    dt = dtype[0] if isinstance(dtype, list) else dtype
    if sample_weight is None:
        return np.ones(n, dtype=dt)
    if isinstance(sample_weight, numbers.Number):
        return np.full(n, sample_weight, dtype=dt)
    sw = check_array(sample_weight, ensure_2d=False, dtype=dt, order="C", copy=copy)
    if sw.ndim != 1:
        raise ValueError("Sample weights must be 1D array or scalar")
    if sw.shape != (n,):
        raise ValueError(f"sample_weight.shape == {sw.shape}, expected {(n,)}!")
    return sw


def check_scalar(x, name, target_type, *, min_val=None, max_val=None):
    if not isinstance(x, target_type):
        raise TypeError(f"`{name}` must be an instance of {target_type}, not {type(x)}.")
    if min_val is not None and x < min_val:
        raise ValueError(f"`{name}`= {x}, must be >= {min_val}.")
    if max_val is not None and x > max_val:
        raise ValueError(f"`{name}`= {x}, must be <= {max_val}.")


def check_memory(memory):
    """``memory`` as an object with a joblib.Memory-style ``cache`` method
    (reference ``utils/validation.py:316``): None or a str path -> a
    joblib.Memory (identity-caching stub when joblib is absent); objects
    with ``cache`` pass through."""
    if memory is None or isinstance(memory, str):
        try:
            import joblib
            return joblib.Memory(location=memory, verbose=0)
        except ImportError:  # pragma: no cover
            if memory is not None:
                raise ValueError("a cache directory needs joblib")

            class _NoCache:
                location = None

                def cache(self, func=None, **kw):
                    return func if func is not None else (lambda f: f)
            return _NoCache()
    if not hasattr(memory, "cache"):
        raise ValueError("'memory' should be None, a string or have the same interface as "
                         "joblib.Memory. Got memory='{}' instead.".format(memory))
    return memory


def has_fit_parameter(estimator, parameter):
    """Whether ``estimator.fit`` accepts an argument named ``parameter``
    (reference ``utils/validation.py:1003``)."""
    import inspect
    return parameter in inspect.signature(estimator.fit).parameters


def check_non_negative(X, whom):
    """Raise ValueError when ``X`` (dense, sparse or tensor) has a negative
    entry (reference ``utils/validation.py:1153``)."""
    import scipy.sparse as sp
    if sp.issparse(X):
        data = X.data if X.format in ("csr", "csc", "coo", "bsr") else X.tocsr().data
        xmin = data.min() if data.size else 0
        if X.nnz < X.shape[0] * X.shape[1]:
            xmin = min(xmin, 0)
    elif isinstance(X, torch.Tensor):
        xmin = float(X.min()) if X.numel() else 0
    else:
        X = np.asarray(X)
        xmin = X.min() if X.size else 0
    if xmin < 0:
        raise ValueError("Negative values in data passed to %s" % whom)


def __getattr__(name):
    # helpers implemented in utils/_misc.py, exposed here like the reference
    if name in ("indexable", "as_float_array", "assert_all_finite", "check_symmetric"):
        from . import _misc
        return getattr(_misc, name)
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
