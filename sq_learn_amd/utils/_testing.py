"""Testing helpers used by estimator test suites (reference
``utils/_testing.py``): numpy's array assertions, warning / exception
assertions, ``ignore_warnings`` (decorator and context manager),
``set_random_state``, dense-vs-sparse comparison, memmap-backed data,
running a Python snippet in a child interpreter, ``raises`` and minimal
estimators implementing only the API contract."""

import contextlib
import functools
import os
import re
import shutil
import subprocess
import sys
import tempfile
import unittest
import warnings

import numpy as np
import scipy.sparse as sp
from numpy.testing import (assert_allclose, assert_almost_equal, assert_approx_equal,  # noqa: F401
                           assert_array_almost_equal, assert_array_equal, assert_array_less)

SkipTest = unittest.case.SkipTest
_case = unittest.TestCase("__init__")
assert_raises = _case.assertRaises
assert_raises_regex = _case.assertRaisesRegex
assert_raises_regexp = _case.assertRaisesRegex
assert_dict_equal = _case.assertDictEqual


def assert_warns(warning_class, func, *args, **kw):
    """Call ``func``; fail unless it warned with ``warning_class``."""
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        out = func(*args, **kw)
    if not any(issubclass(w.category, warning_class) for w in rec):
        raise AssertionError(f"No {warning_class.__name__} was raised by {func.__name__}")
    return out


def assert_warns_message(warning_class, message, func, *args, **kw):
    """As assert_warns, and the message contains ``message`` (or the
    callable ``message(msg)`` is true)."""
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        out = func(*args, **kw)
    hits = [w for w in rec if issubclass(w.category, warning_class)]
    if not hits:
        raise AssertionError(f"No {warning_class.__name__} was raised by {func.__name__}")
    ok = any(message(str(w.message)) if callable(message) else message in str(w.message)
             for w in hits)
    if not ok:
        raise AssertionError(f"No {warning_class.__name__} with message {message!r}; got "
                             f"{[str(w.message) for w in hits]}")
    return out


def assert_no_warnings(func, *args, **kw):
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        out = func(*args, **kw)
    rec = [w for w in rec if not issubclass(w.category, FutureWarning)]
    if rec:
        raise AssertionError(f"Got warnings when calling {func.__name__}: "
                             f"{[str(w.message) for w in rec]}")
    return out


class _IgnoreWarnings:
    """Context manager / decorator silencing ``category`` warnings."""

    def __init__(self, category):
        self.category = category
        self._cm = None

    def __call__(self, fn):
        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            with warnings.catch_warnings():
                warnings.simplefilter("ignore", self.category)
                return fn(*args, **kwargs)
        return wrapper

    def __enter__(self):
        self._cm = warnings.catch_warnings()
        self._cm.__enter__()
        warnings.simplefilter("ignore", self.category)

    def __exit__(self, *exc):
        self._cm.__exit__(*exc)


def ignore_warnings(obj=None, category=Warning):
    """``@ignore_warnings``, ``@ignore_warnings(category=...)`` or ``with
    ignore_warnings():``."""
    if isinstance(obj, type) and issubclass(obj, Warning):
        raise ValueError("'obj' should be a callable where you want to ignore warnings. You "
                         f"passed a warning class instead: 'obj={obj.__name__}'. If you want "
                         "to pass a warning class to ignore_warnings, you should use "
                         f"'category={obj.__name__}'")
    if callable(obj):
        return _IgnoreWarnings(category)(obj)
    return _IgnoreWarnings(category)


def assert_raise_message(exceptions, message, function, *args, **kwargs):
    """``function`` raises one of ``exceptions`` whose text contains
    ``message``."""
    try:
        function(*args, **kwargs)
    except exceptions as e:
        if message not in str(e):
            raise AssertionError(f"Error message does not include the expected string: "
                                 f"{message!r}. Observed error message: {str(e)!r}")
    else:
        names = (exceptions.__name__ if isinstance(exceptions, type)
                 else " or ".join(e.__name__ for e in exceptions))
        raise AssertionError(f"{names} not raised by {function.__name__}")


def assert_allclose_dense_sparse(x, y, rtol=1e-07, atol=1e-9, err_msg=""):
    """Both dense or both sparse (then same pattern after canonicalising)
    and numerically close."""
    if sp.issparse(x) and sp.issparse(y):
        x, y = x.tocsr(), y.tocsr()
        x.sum_duplicates()
        y.sum_duplicates()
        assert_array_equal(x.indices, y.indices, err_msg=err_msg)
        assert_array_equal(x.indptr, y.indptr, err_msg=err_msg)
        assert_allclose(x.data, y.data, rtol=rtol, atol=atol, err_msg=err_msg)
    elif not sp.issparse(x) and not sp.issparse(y):
        assert_allclose(x, y, rtol=rtol, atol=atol, err_msg=err_msg)
    else:
        raise ValueError("Can only compare two sparse matrices, not a sparse matrix and an "
                         "array.")


def set_random_state(estimator, random_state=0):
    """Set every ``*random_state`` parameter of ``estimator``."""
    if "random_state" in estimator.get_params():
        estimator.set_params(random_state=random_state)


class TempMemmap:
    """Context manager yielding ``data`` backed by a temporary memmap."""

    def __init__(self, data, mmap_mode="r"):
        self.mmap_mode = mmap_mode
        self.data = data

    def __enter__(self):
        data, self.folder = create_memmap_backed_data(self.data, mmap_mode=self.mmap_mode,
                                                      return_folder=True)
        return data

    def __exit__(self, *exc):
        shutil.rmtree(self.folder, ignore_errors=True)


def create_memmap_backed_data(data, mmap_mode="r", return_folder=False):
    """A copy of the array ``data`` memory-mapped from a temporary file."""
    folder = tempfile.mkdtemp(prefix="sq_learn_amd_")
    path = os.path.join(folder, "data.npy")
    np.save(path, np.asarray(data))
    out = np.load(path, mmap_mode=mmap_mode)
    return (out, folder) if return_folder else out


def check_skip_network():
    if int(os.environ.get("SKLEARN_SKIP_NETWORK_TESTS", "1")):
        raise SkipTest("Text tutorial requires large dataset download")


def assert_run_python_script(source_code, timeout=60):
    """Run ``source_code`` in a fresh interpreter (this repository on the
    path); fail with its output on a non-zero exit."""
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ)
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    with tempfile.NamedTemporaryFile("w", suffix=".py", delete=False) as f:
        f.write(source_code)
        path = f.name
    try:
        proc = subprocess.run([sys.executable, path], capture_output=True, text=True,
                              timeout=timeout, env=env, cwd=root)
    finally:
        os.unlink(path)
    if proc.returncode != 0:
        raise RuntimeError(f"script errored with output:\n{proc.stdout}{proc.stderr}")


class _Raises(contextlib.AbstractContextManager):
    def __init__(self, expected, match, may_pass, err_msg):
        self.expected = expected if isinstance(expected, (list, tuple)) else [expected]
        self.match = [match] if isinstance(match, str) else match
        self.may_pass = may_pass
        self.err_msg = err_msg
        self.raised_and_matched = False

    def __exit__(self, exc_type, exc, tb):
        if exc_type is None:
            if self.may_pass:
                return True
            raise AssertionError(self.err_msg or
                                 f"Did not raise: {[e.__name__ for e in self.expected]}")
        if not any(issubclass(exc_type, e) for e in self.expected):
            if self.err_msg is not None:
                raise AssertionError(self.err_msg) from exc
            return False
        if self.match is not None:
            if not any(re.search(m, str(exc)) for m in self.match):
                raise AssertionError(self.err_msg or
                                     f"The error message should contain one of the patterns "
                                     f"{self.match}; got {str(exc)!r}") from exc
        self.raised_and_matched = True
        return True


def raises(expected_exc_type, match=None, may_pass=False, err_msg=None):
    """Context manager: the block raises ``expected_exc_type`` (one of a
    list), its message matches one of ``match``; ``may_pass`` allows no
    exception at all."""
    return _Raises(expected_exc_type, match, may_pass, err_msg)


class MinimalClassifier:
    """A classifier implementing only the estimator contract (no
    BaseEstimator): predicts the majority class."""

    _estimator_type = "classifier"

    def __init__(self, param=None):
        self.param = param

    def get_params(self, deep=True):
        return {"param": self.param}

    def set_params(self, **params):
        for k, v in params.items():
            setattr(self, k, v)
        return self

    def fit(self, X, y):
        y = np.asarray(y)
        self.classes_, counts = np.unique(y, return_counts=True)
        self._most_frequent = int(np.argmax(counts))
        return self

    def predict_proba(self, X):
        n = np.asarray(X).shape[0]
        p = np.zeros((n, len(self.classes_)))
        p[:, self._most_frequent] = 1.0
        return p

    def predict(self, X):
        return self.classes_[np.argmax(self.predict_proba(X), axis=1)]

    def score(self, X, y):
        return float(np.mean(self.predict(X) == np.asarray(y)))


class MinimalRegressor:
    """A regressor implementing only the contract: predicts the mean."""

    _estimator_type = "regressor"

    def __init__(self, param=None):
        self.param = param

    def get_params(self, deep=True):
        return {"param": self.param}

    def set_params(self, **params):
        for k, v in params.items():
            setattr(self, k, v)
        return self

    def fit(self, X, y):
        self.is_fitted_ = True
        self._mean = float(np.mean(y))
        return self

    def predict(self, X):
        return np.full(np.asarray(X).shape[0], self._mean)

    def score(self, X, y):
        y = np.asarray(y, dtype=float)
        p = self.predict(X)
        den = ((y - y.mean()) ** 2).sum()
        return 1.0 - ((y - p) ** 2).sum() / den if den > 0 else 0.0


class MinimalTransformer:
    """A transformer implementing only the contract: the identity."""

    def __init__(self, param=None):
        self.param = param

    def get_params(self, deep=True):
        return {"param": self.param}

    def set_params(self, **params):
        for k, v in params.items():
            setattr(self, k, v)
        return self

    def fit(self, X, y=None):
        self.is_fitted_ = True
        return self

    def transform(self, X, y=None):
        return np.asarray(X)

    def fit_transform(self, X, y=None):
        return self.fit(X, y).transform(X, y)


__all__ = ["assert_raises", "assert_raises_regexp", "assert_array_equal", "assert_almost_equal",
           "assert_array_almost_equal", "assert_array_less", "assert_approx_equal",
           "assert_allclose", "assert_run_python_script", "SkipTest"]


def assert_warns_div0(func, *args, **kw):
    """func(*args) must emit a RuntimeWarning about division by zero /
    invalid values (or none at all, where the platform does not warn)."""
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        result = func(*args, **kw)
    msgs = [str(w.message) for w in rec if issubclass(w.category, RuntimeWarning)]
    if rec and not any(("divide" in m) or ("invalid value" in m) for m in msgs):
        raise AssertionError(f"expected a division-by-zero warning, got {msgs}")
    return result


def check_docstring_parameters(func, doc=None, ignore=None):
    """Names of the signature parameters of ``func`` that its numpydoc
    ``Parameters`` section does not document (and vice versa), as a list of
    error strings (empty = consistent)."""
    import inspect
    ignore = set(ignore or ())
    try:
        sig = inspect.signature(func)
    except (TypeError, ValueError):
        return []
    params = [p for p in sig.parameters if p not in ("self", "cls", "args", "kwargs")
              and p not in ignore]
    text = doc if doc is not None else (inspect.getdoc(func) or "")
    m = re.search(r"Parameters\n-+\n(.*?)(\n\n[A-Z][a-z]+\n-+\n|\Z)", text, re.S)
    documented = []
    if m:
        for line in m.group(1).split("\n"):
            mm = re.match(r"^(\w+)\s*(:|$)", line)
            if mm:
                documented.append(mm.group(1))
    documented = [d for d in documented if d not in ignore]
    errors = []
    if m and params != documented:
        missing = [p for p in params if p not in documented]
        extra = [d for d in documented if d not in params]
        if missing:
            errors.append(f"{getattr(func, '__qualname__', func)}: undocumented {missing}")
        if extra:
            errors.append(f"{getattr(func, '__qualname__', func)}: documented but absent {extra}")
    return errors
