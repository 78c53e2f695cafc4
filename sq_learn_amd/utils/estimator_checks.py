"""Public estimator-conformance checks (reference ``utils/estimator_checks.py``:
``parametrize_with_checks`` :431, ``check_estimator`` :486).

Each check is ``check_xxx(name, estimator)`` and raises ``AssertionError``
(or the estimator's own error) on a violation of the estimator contract the
framework's estimators share with scikit-learn:

* API: constructor stores its parameters untouched, ``get_params`` /
  ``set_params`` / ``clone`` round trips, ``fit`` returns ``self`` and does not
  modify the public parameters, unfitted use raises ``NotFittedError``;
* data handling: ``n_features_in_``, float32 input, empty input and NaN/inf
  are rejected with ``ValueError``;
* reproducibility: fitting twice with a fixed ``random_state`` gives the same
  outputs; a pickled fitted estimator predicts / transforms identically;
* type-specific behaviour: classifiers learn an easy problem (accuracy >
  0.83) and expose ``classes_``; regressors reach R^2 > 0.5 on a linear
  problem; clusterers' ``fit_predict`` equals ``labels_``; transformers'
  ``fit_transform`` equals ``fit().transform``.

Estimator tags (``_get_tags()``) adapt the data: ``requires_positive_X``,
``requires_positive_y``, ``requires_y``, ``binary_only``, ``X_types``
(non-'2darray' inputs skip the array checks), ``multioutput_only``,
``stateless`` / ``requires_fit`` (no not-fitted error expected),
``poor_score`` (no score threshold), ``non_deterministic`` (skips the
idempotence check) and ``_xfail_checks`` ({check name: reason}) like the
reference.
"""

import copy
import pickle
import warnings
from functools import partial

import numpy as np

from ..base import clone, is_classifier, is_regressor, is_clusterer, is_outlier_detector
from ..exceptions import NotFittedError

__all__ = ["check_estimator", "parametrize_with_checks"]


# ------------------------------------------------------------------ data
def _blobs(n=90, d=5, centers=3, seed=0):
    rng = np.random.RandomState(seed)
    C = rng.uniform(-6, 6, (centers, d))
    y = np.arange(n) % centers
    X = C[y] + rng.randn(n, d)
    return X, y


def _tags(est):
    try:
        return est._get_tags()
    except Exception:
        return {}


def _X_y(est, n=90, d=5):
    tags = _tags(est)
    X, y = _blobs(n, d, centers=2 if tags.get("binary_only") else 3)
    if tags.get("requires_positive_X") or tags.get("positive_X"):
        X = np.abs(X)
    if is_regressor(est):
        rng = np.random.RandomState(1)
        w = rng.randn(d)
        y = X @ w + 0.1 * rng.randn(n)
        if tags.get("requires_positive_y"):
            y = np.abs(y) + 1.0
    elif tags.get("binary_only"):
        y = np.where(y == 0, -1, 1)
    return X, y


def _needs_y(est):
    import inspect
    try:
        p = inspect.signature(est.fit).parameters
    except (TypeError, ValueError):
        return False
    yp = p.get("y", p.get("Y"))
    return yp is not None and yp.default is inspect.Parameter.empty


def _fit(est, X, y):
    if is_classifier(est) or is_regressor(est) or _tags(est).get("requires_y") or _needs_y(est):
        return est.fit(X, y)
    try:
        return est.fit(X, y)
    except TypeError:
        return est.fit(X)


def _set_random_state(est, seed=0):
    params = est.get_params(deep=False)
    if "random_state" in params and params["random_state"] is None:
        est.set_params(random_state=seed)
    return est


def _outputs(est, X):
    out = {}
    for meth in ("predict", "transform", "decision_function", "predict_proba", "score_samples"):
        f = getattr(est, meth, None)
        if f is None:
            continue
        try:
            v = f(X)
        except (AttributeError, NotImplementedError, NotFittedError):
            continue
        if isinstance(v, dict) or v is None:
            continue
        if hasattr(v, "toarray"):
            v = v.toarray()
        try:
            out[meth] = np.asarray(v, dtype=float)
        except (TypeError, ValueError):
            continue
    return out


# ------------------------------------------------------------------ API checks
def check_no_attributes_set_in_init(name, est):
    """__init__ stores every parameter under its own name and nothing else
    public (reference :2860)."""
    est = clone(est)
    params = est.get_params(deep=False)
    init_params = set(type(est)._get_param_names())
    assert set(params) == init_params, f"{name}: get_params keys differ from __init__ signature"
    for k in init_params:
        assert hasattr(est, k), f"{name}: __init__ parameter {k!r} not stored"
    # parameters of the parent classes' __init__ (set through super().__init__
    # with fixed values, e.g. CCA's mode) are allowed, like the reference
    import inspect
    parents = set()
    for base in type(est).__mro__[1:]:
        if "__init__" in vars(base) and base is not object:
            try:
                parents |= set(inspect.signature(vars(base)["__init__"]).parameters) - {"self"}
            except (TypeError, ValueError):
                pass
    extra = [a for a in vars(est) if not a.startswith("_") and a not in init_params
             and a not in parents]
    assert not extra, f"{name}: __init__ sets non-parameter attributes {extra}"


def check_get_params_invariance(name, est):
    shallow = est.get_params(deep=False)
    deep = est.get_params(deep=True)
    assert all(item in deep.items() or k in deep for k, item in shallow.items()), name


def check_set_params(name, est):
    est = clone(est)
    orig = est.get_params(deep=False)
    ret = est.set_params(**orig)
    assert ret is est, f"{name}: set_params does not return self"
    after = est.get_params(deep=False)
    for k, v in orig.items():
        assert after[k] is v or _same(after[k], v), f"{name}: set_params changed {k}"


def _same(a, b):
    """Parameter equality; estimators compare by type and parameters (a
    clone or deep copy is a different object with the same configuration)."""
    if hasattr(a, "get_params") and hasattr(b, "get_params"):
        if type(a) is not type(b):
            return False
        pa, pb = a.get_params(deep=False), b.get_params(deep=False)
        return pa.keys() == pb.keys() and all(_same(pa[k], pb[k]) for k in pa)
    if isinstance(a, (list, tuple)) and isinstance(b, (list, tuple)):
        return len(a) == len(b) and all(_same(x, y) for x, y in zip(a, b))
    if isinstance(a, dict) and isinstance(b, dict):
        return a.keys() == b.keys() and all(_same(a[k], b[k]) for k in a)
    try:
        if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
            return np.array_equal(np.asarray(a), np.asarray(b))
        r = a == b
        if isinstance(r, bool):
            return r or (a != a and b != b)
        return bool(np.all(r))
    except Exception:
        return a is b


def check_parameters_default_constructible(name, est):
    c = clone(est)
    assert type(c) is type(est)
    for k, v in est.get_params(deep=False).items():
        cv = c.get_params(deep=False)[k]
        if hasattr(v, "get_params"):
            assert type(cv) is type(v)
        else:
            assert _same(cv, v), f"{name}: clone changed parameter {k}"
    repr(est)


def check_fit_returns_self(name, est):
    est = _set_random_state(clone(est))
    X, y = _X_y(est)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        assert _fit(est, X, y) is est, f"{name}: fit does not return self"


def check_dont_overwrite_parameters(name, est):
    est = _set_random_state(clone(est))
    before = copy.deepcopy(est.get_params(deep=False))
    X, y = _X_y(est)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        _fit(est, X, y)
    after = est.get_params(deep=False)
    for k, v in before.items():
        if hasattr(v, "get_params"):
            continue
        assert _same(after[k], v), f"{name}: fit modified parameter {k}"


def check_estimators_unfitted(name, est):
    tags = _tags(est)
    if tags.get("stateless") or tags.get("requires_fit") is False:
        return
    est = clone(est)
    X, _ = _X_y(est)
    for meth in ("predict", "transform"):
        f = getattr(est, meth, None)
        if f is None:
            continue
        try:
            f(X)
        except (NotFittedError, AttributeError, ValueError, TypeError, RuntimeError,
                IndexError, KeyError):
            continue
        raise AssertionError(f"{name}.{meth} did not raise before fit")


# ------------------------------------------------------------------ data checks
def check_n_features_in(name, est):
    est = _set_random_state(clone(est))
    X, y = _X_y(est)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        _fit(est, X, y)
    if hasattr(est, "n_features_in_"):
        assert est.n_features_in_ == X.shape[1], name


def check_estimators_dtypes(name, est):
    X, y = _X_y(est)
    for dt in (np.float32, np.float64):
        e = _set_random_state(clone(est))
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            _fit(e, X.astype(dt), y)
            _outputs(e, X.astype(dt))


def check_estimators_empty_data_messages(name, est):
    est = clone(est)
    X = np.empty((0, 3))
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            est.fit(X, np.empty(0))
    except (ValueError, IndexError, RuntimeError, TypeError):
        return
    raise AssertionError(f"{name} accepted an empty dataset")


def check_estimators_nan_inf(name, est):
    if _tags(est).get("allow_nan"):
        return
    X, y = _X_y(est)
    for bad in (np.nan, np.inf):
        Xb = X.copy()
        Xb[0, 0] = bad
        e = _set_random_state(clone(est))
        try:
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                _fit(e, Xb, y)
        except (ValueError, FloatingPointError, RuntimeError):
            continue
        raise AssertionError(f"{name} accepted {bad} in X")


# ------------------------------------------------------------------ reproducibility
def check_fit_idempotent(name, est):
    if _tags(est).get("non_deterministic"):
        return
    X, y = _X_y(est)
    outs = []
    for _ in range(2):
        e = _set_random_state(clone(est), 7)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            _fit(e, X, y)
            outs.append(_outputs(e, X))
    for k in outs[0]:
        np.testing.assert_allclose(outs[0][k], outs[1][k], rtol=1e-7, atol=1e-9,
                                   err_msg=f"{name}.{k} differs between two fits")


def check_estimators_pickle(name, est):
    e = _set_random_state(clone(est))
    X, y = _X_y(est)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        _fit(e, X, y)
        a = _outputs(e, X)
        e2 = pickle.loads(pickle.dumps(e))
        b = _outputs(e2, X)
    for k in a:
        np.testing.assert_allclose(a[k], b[k], atol=1e-9, err_msg=f"{name}.{k} after pickle")


# ------------------------------------------------------------------ type checks
def check_classifiers_train(name, est):
    e = _set_random_state(clone(est))
    X, y = _X_y(est)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        e.fit(X, y)
        pred = np.asarray(e.predict(X))
    assert pred.shape == y.shape, f"{name}: predict shape"
    if not _tags(est).get("poor_score"):
        assert np.mean(pred == y) > 0.83, f"{name}: training accuracy {np.mean(pred == y):.2f}"
    n_cls = len(np.unique(y))
    assert hasattr(e, "classes_") and len(e.classes_) == n_cls, f"{name}: classes_"


def check_regressors_train(name, est):
    e = _set_random_state(clone(est))
    X, y = _X_y(est)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        e.fit(X, y)
        pred = np.asarray(e.predict(X)).reshape(y.shape)
    r2 = 1 - np.sum((pred - y) ** 2) / np.sum((y - y.mean()) ** 2)
    if not _tags(est).get("poor_score"):
        assert r2 > 0.5, f"{name}: training R^2 {r2:.2f}"


def check_clustering(name, est):
    e = _set_random_state(clone(est))
    X, y = _X_y(est)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        e.fit(X)
        lab = np.asarray(e.labels_)
        assert lab.shape == (X.shape[0],), f"{name}: labels_ shape"
        e2 = _set_random_state(clone(est))
        lab2 = np.asarray(e2.fit_predict(X))
    if not _tags(est).get("non_deterministic"):
        np.testing.assert_array_equal(lab, lab2, err_msg=f"{name}: fit_predict != labels_")


def check_transformer_general(name, est):
    e = _set_random_state(clone(est))
    X, y = _X_y(est)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        try:
            try:   # y is passed like the reference's check; unsupervised ones ignore it
                a = e.fit_transform(X, y)
            except TypeError:
                a = e.fit_transform(X)
            e2 = _set_random_state(clone(est))
            _fit(e2, X, y)
            b = e2.transform(X)
        except AttributeError:   # e.g. a Pipeline whose last step has no transform
            return
    if hasattr(a, "toarray"):
        a, b = a.toarray(), b.toarray()
    if isinstance(a, dict) or isinstance(b, dict):
        return
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    assert a.shape[0] == X.shape[0], f"{name}: transform row count"
    if not _tags(est).get("non_deterministic"):
        # atol 1e-2 like the reference's _check_transformer (iterative
        # transformers re-solve for the training codes in transform)
        np.testing.assert_allclose(np.abs(a), np.abs(b), rtol=1e-2, atol=1e-2,
                                   err_msg=f"{name}: fit_transform != fit().transform")


def check_outliers_fit_predict(name, est):
    e = _set_random_state(clone(est))
    X, _ = _X_y(est)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        p = np.asarray(e.fit_predict(X))
    assert set(np.unique(p)) <= {-1, 1}, f"{name}: outlier labels must be +-1"


# ------------------------------------------------------------------ driver
_API = (check_no_attributes_set_in_init, check_get_params_invariance, check_set_params,
        check_parameters_default_constructible)
_FITTING = (check_fit_returns_self, check_dont_overwrite_parameters, check_estimators_unfitted,
            check_n_features_in, check_estimators_dtypes, check_estimators_empty_data_messages,
            check_estimators_nan_inf, check_fit_idempotent, check_estimators_pickle)


def _yield_all_checks(est):
    yield from _API
    tags = _tags(est)
    if "2darray" not in tags.get("X_types", ["2darray"]):
        return
    if tags.get("multioutput_only") or tags.get("_skip_fit_checks"):
        return
    yield from _FITTING
    if is_classifier(est):
        yield check_classifiers_train
    elif is_regressor(est):
        yield check_regressors_train
    if is_clusterer(est) and hasattr(est, "fit_predict"):
        yield check_clustering
    if is_outlier_detector(est):
        yield check_outliers_fit_predict
    if hasattr(est, "transform") and hasattr(est, "fit_transform") and not is_clusterer(est):
        yield check_transformer_general


def _xfail(est, check):
    reasons = _tags(est).get("_xfail_checks", {}) or {}
    name = check.func.__name__ if isinstance(check, partial) else check.__name__
    return reasons.get(name)


def check_estimator(estimator, generate_only=False):
    """Run every applicable check on ``estimator`` (an instance), raising on
    the first failure (checks listed in the ``_xfail_checks`` tag are
    skipped).  ``generate_only=True`` returns a generator of
    ``(estimator, check)`` pairs instead, ``check(estimator)`` running one."""
    if isinstance(estimator, type):
        raise TypeError("Passing a class was deprecated in the reference; pass an instance")
    name = type(estimator).__name__

    def gen():
        for chk in _yield_all_checks(estimator):
            yield estimator, partial(chk, name)

    if generate_only:
        return gen()
    for est, chk in gen():
        if _xfail(est, chk):
            continue
        chk(est)
    return None


def parametrize_with_checks(estimators):
    """pytest decorator parametrizing a test ``(estimator, check)`` over every
    check of every estimator instance; xfail-tagged checks are marked
    ``pytest.mark.xfail`` (reference :431)."""
    import pytest
    if any(isinstance(e, type) for e in estimators):
        raise TypeError("parametrize_with_checks takes estimator instances, not classes")
    params = []
    for est in estimators:
        for e, chk in check_estimator(est, generate_only=True):
            reason = _xfail(e, chk)
            pid = f"{type(e).__name__}-{chk.func.__name__}"
            marks = [pytest.mark.xfail(reason=reason)] if reason else []
            params.append(pytest.param(e, chk, id=pid, marks=marks))
    return pytest.mark.parametrize("estimator, check", params)
