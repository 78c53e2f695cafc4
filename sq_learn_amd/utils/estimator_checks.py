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


# ------------------------------------------------------------------ individual checks
# The reference's finer-grained public checks (``utils/estimator_checks.py``,
# same names and ``(name, estimator_orig)`` signature).  They are importable
# one by one; ``check_estimator`` runs the core set above.  Each adapts to
# the estimator type the same way (_X_y / _fit / tags) and returns silently
# when the estimator does not expose what the check is about.
def _fitted(est, X=None, y=None):
    est = _set_random_state(clone(est))
    if X is None:
        X, y = _X_y(est)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        _fit(est, X, y)
    return est, X, y


def _supervised(est):
    return is_classifier(est) or is_regressor(est)


def _has_sample_weight(est):
    import inspect
    try:
        return "sample_weight" in inspect.signature(est.fit).parameters
    except (TypeError, ValueError):
        return False


def _expect_value_error(fn):
    try:
        fn()
    except (ValueError, TypeError):
        return
    raise AssertionError("expected a ValueError")


def check_estimators_fit_returns_self(name, estimator_orig, readonly_memmap=False):
    est = _set_random_state(clone(estimator_orig))
    X, y = _X_y(est)
    if readonly_memmap:
        X = X.copy()
        X.setflags(write=False)
    assert _fit(est, X, y) is est


def check_supervised_y_no_nan(name, estimator_orig):
    if not _supervised(estimator_orig):
        return
    est = clone(estimator_orig)
    X, _ = _X_y(est)
    for bad in (np.inf, np.nan):
        y = np.full(X.shape[0], bad)
        _expect_value_error(lambda: est.fit(X, y))


def check_supervised_y_2d(name, estimator_orig):
    """A column-vector y fits like the 1-D y (possibly with a
    DataConversionWarning) and predicts the same."""
    if not _supervised(estimator_orig):
        return
    est, X, y = _fitted(estimator_orig)
    p1 = est.predict(X)
    est2 = _set_random_state(clone(estimator_orig))
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        try:
            est2.fit(X, y[:, None])
        except ValueError:
            return   # multioutput-only refusal is allowed
    np.testing.assert_allclose(np.ravel(est2.predict(X)), np.ravel(p1), rtol=1e-6, atol=1e-6)


def check_estimator_sparse_data(name, estimator_orig):
    """CSR input either works or is refused with TypeError / ValueError."""
    import scipy.sparse as sp
    est = _set_random_state(clone(estimator_orig))
    X, y = _X_y(est)
    X[X < 0.5] = 0
    Xs = sp.csr_matrix(X)
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            _fit(est, Xs, y)
    except (TypeError, ValueError):
        return
    for meth in ("predict", "transform"):
        if hasattr(est, meth):
            out = getattr(est, meth)(Xs)
            assert out.shape[0] == X.shape[0]


def _sw_fit(est, X, y, sw):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        if _supervised(est) or _needs_y(est):
            return est.fit(X, y, sample_weight=sw)
        return est.fit(X, sample_weight=sw)


def check_sample_weights_pandas_series(name, estimator_orig):
    if not _has_sample_weight(estimator_orig):
        return
    import pandas as pd
    est = _set_random_state(clone(estimator_orig))
    X, y = _X_y(est)
    _sw_fit(est, pd.DataFrame(X), pd.Series(y), pd.Series(np.ones(len(y))))


def check_sample_weights_not_an_array(name, estimator_orig):
    if not _has_sample_weight(estimator_orig):
        return
    est = _set_random_state(clone(estimator_orig))
    X, y = _X_y(est)
    _sw_fit(est, X, y, list(np.ones(len(y))))


def check_sample_weights_list(name, estimator_orig):
    check_sample_weights_not_an_array(name, estimator_orig)


def check_sample_weights_shape(name, estimator_orig):
    if not _has_sample_weight(estimator_orig):
        return
    est = _set_random_state(clone(estimator_orig))
    X, y = _X_y(est)
    _sw_fit(est, X, y, np.ones(len(y)))
    _expect_value_error(lambda: _sw_fit(clone(est), X, y, np.ones(2 * len(y))))
    _expect_value_error(lambda: _sw_fit(clone(est), X, y, np.ones((len(y), 2))))


def check_sample_weights_invariance(name, estimator_orig, kind="ones"):
    """kind='ones': unit weights == no weights; kind='zeros': rows of weight
    zero are as if removed."""
    if not _has_sample_weight(estimator_orig):
        return
    X, y = _X_y(estimator_orig)
    if kind == "ones":
        e1 = _set_random_state(clone(estimator_orig))
        e2 = _set_random_state(clone(estimator_orig))
        _sw_fit(e1, X, y, np.ones(len(y)))
        _sw_fit(e2, X, y, None)
        Xt = X
    else:
        Xd = np.vstack([X, X[:10] + 1.0])
        yd = np.concatenate([y, y[:10]])
        sw = np.concatenate([np.ones(len(y)), np.zeros(10)])
        e1 = _set_random_state(clone(estimator_orig))
        e2 = _set_random_state(clone(estimator_orig))
        _sw_fit(e1, Xd, yd, sw)
        _sw_fit(e2, X, y, None)
        Xt = X
    o1, o2 = _outputs(e1, Xt), _outputs(e2, Xt)
    for k in o1:
        if k in o2:
            np.testing.assert_allclose(o1[k], o2[k], rtol=1e-6, atol=1e-6,
                                       err_msg=f"{name}.{k} changes with {kind} weights")


def check_dtype_object(name, estimator_orig):
    """Numeric data in an object array is accepted; strings are refused."""
    est = _set_random_state(clone(estimator_orig))
    X, y = _X_y(est)
    if _tags(est).get("X_types", ["2darray"]) != ["2darray"]:
        return
    _fit(est, X.astype(object), y)
    Xs = X.astype(object)
    Xs[0, 0] = "not a number"
    _expect_value_error(lambda: _fit(clone(est), Xs, y))


def check_complex_data(name, estimator_orig):
    est = clone(estimator_orig)
    X, y = _X_y(est)
    _expect_value_error(lambda: _fit(est, X + 1j, y))


def check_dict_unchanged(name, estimator_orig):
    """predict / transform / ... leave the fitted estimator's __dict__ as is."""
    est, X, _ = _fitted(estimator_orig)
    before = copy.deepcopy({k: v for k, v in est.__dict__.items()
                            if not callable(v)})
    _outputs(est, X)
    for k, v in before.items():
        assert _same(v, est.__dict__.get(k)), f"{name}: {k} changed by a predict-type call"


def check_fit2d_predict1d(name, estimator_orig):
    est, X, _ = _fitted(estimator_orig)
    for meth in ("predict", "transform", "decision_function", "predict_proba"):
        if hasattr(est, meth):
            _expect_value_error(lambda: getattr(est, meth)(X[0]))


def _subset_or_order(name, estimator_orig, perm):
    est, X, _ = _fitted(estimator_orig)
    full = _outputs(est, X)
    part = _outputs(est, X[perm])
    for k, v in full.items():
        if k in part and v.ndim >= 1 and v.shape[0] == X.shape[0]:
            np.testing.assert_allclose(part[k], v[perm], rtol=1e-6, atol=1e-6,
                                       err_msg=f"{name}.{k}")


def check_methods_subset_invariance(name, estimator_orig):
    """Predicting on a batch equals predicting on its rows' superset."""
    _subset_or_order(name, estimator_orig, np.arange(0, 90, 3))


def check_methods_sample_order_invariance(name, estimator_orig):
    _subset_or_order(name, estimator_orig, np.random.RandomState(0).permutation(90))


def check_fit2d_1sample(name, estimator_orig):
    """One row: either fits or raises a ValueError."""
    est = _set_random_state(clone(estimator_orig))
    X, y = _X_y(est)
    try:
        _fit(est, X[:1], y[:1])
    except ValueError:
        pass


def check_fit2d_1feature(name, estimator_orig):
    est = _set_random_state(clone(estimator_orig))
    X, y = _X_y(est)
    try:
        _fit(est, X[:, :1], y)
    except ValueError:
        pass


def check_fit1d(name, estimator_orig):
    est = clone(estimator_orig)
    X, y = _X_y(est)
    _expect_value_error(lambda: _fit(est, X[:, 0], y))


def check_transformer_data_not_an_array(name, transformer):
    if not hasattr(transformer, "transform"):
        return
    est, X, y = _fitted(transformer)
    est2, _, _ = _fitted(transformer, [list(r) for r in X], list(y))
    np.testing.assert_allclose(np.asarray(est.transform(X)), np.asarray(est2.transform(X)),
                               rtol=1e-6, atol=1e-8)


def check_transformers_unfitted(name, transformer):
    if not hasattr(transformer, "transform") or _tags(transformer).get("stateless"):
        return
    X, _ = _X_y(transformer)
    try:
        clone(transformer).transform(X)
    except (AttributeError, ValueError, NotFittedError):
        return
    raise AssertionError(f"{name}.transform did not fail before fit")


def check_pipeline_consistency(name, estimator_orig):
    """Inside a one-step Pipeline the outputs equal the bare estimator's."""
    from ..pipeline import make_pipeline
    est, X, y = _fitted(estimator_orig)
    pipe = make_pipeline(_set_random_state(clone(estimator_orig)))
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        _fit(pipe, X, y)
    a, b = _outputs(est, X), _outputs(pipe, X)
    for k in a:
        if k in b:
            np.testing.assert_allclose(a[k], b[k], rtol=1e-6, atol=1e-6)


def check_fit_score_takes_y(name, estimator_orig):
    import inspect
    for meth in ("fit", "score", "partial_fit", "fit_predict", "fit_transform"):
        f = getattr(estimator_orig, meth, None)
        if f is None:
            continue
        args = [p for p in inspect.signature(f).parameters if p != "self"]
        if args and args[0] in ("args", "kwargs"):
            continue
        assert args[1:2] in (["y"], ["Y"]) or len(args) < 2 or meth == "partial_fit", \
            f"{name}.{meth} second argument is {args[1:2]}, expected y"


def check_transformer_preserve_dtypes(name, transformer):
    if not hasattr(transformer, "transform"):
        return
    preserves = _tags(transformer).get("preserves_dtype", [])
    X, y = _X_y(transformer)
    for dt in preserves:
        est, _, _ = _fitted(transformer, X.astype(dt), y)
        out = np.asarray(est.transform(X.astype(dt)))
        assert out.dtype == dt, f"{name} does not preserve {dt}"


def check_nonsquare_error(name, estimator_orig):
    """Pairwise estimators refuse a non-square 'precomputed' matrix."""
    if not _tags(estimator_orig).get("pairwise"):
        return
    X, y = _X_y(estimator_orig)
    _expect_value_error(lambda: _fit(clone(estimator_orig), X, y))


def check_estimators_partial_fit_n_features(name, estimator_orig):
    if not hasattr(estimator_orig, "partial_fit"):
        return
    est = _set_random_state(clone(estimator_orig))
    X, y = _X_y(est)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        if is_classifier(est):
            est.partial_fit(X, y, classes=np.unique(y))
        elif _supervised(est):
            est.partial_fit(X, y)
        else:
            est.partial_fit(X)
    with np.testing.assert_raises(ValueError):
        if _supervised(est):
            est.partial_fit(X[:, :-1], y)
        else:
            est.partial_fit(X[:, :-1])


def check_classifier_multioutput(name, estimator):
    if not is_classifier(estimator) or not _tags(estimator).get("multioutput"):
        return
    X, y = _X_y(estimator)
    Y = np.stack([y, (y + 1) % 3], axis=1)
    est, _, _ = _fitted(estimator, X, Y)
    assert np.asarray(est.predict(X)).shape == Y.shape


def check_regressor_multioutput(name, estimator):
    if not is_regressor(estimator) or not _tags(estimator).get("multioutput"):
        return
    X, y = _X_y(estimator)
    Y = np.stack([y, -y], axis=1)
    est, _, _ = _fitted(estimator, X, Y)
    assert np.asarray(est.predict(X)).shape == Y.shape


def check_clusterer_compute_labels_predict(name, clusterer_orig):
    est, X, _ = _fitted(clusterer_orig)
    if hasattr(est, "predict") and hasattr(est, "labels_"):
        np.testing.assert_array_equal(est.predict(X), est.labels_)


def check_classifiers_one_label(name, classifier_orig):
    """A single class: fit either succeeds (and predicts it) or raises a
    ValueError."""
    if not is_classifier(classifier_orig):
        return
    X, _ = _X_y(classifier_orig)
    y = np.ones(X.shape[0])
    est = _set_random_state(clone(classifier_orig))
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            est.fit(X, y)
    except ValueError:
        return
    np.testing.assert_array_equal(est.predict(X), y)


def check_outlier_corruption(num_outliers, expected_outliers, decision):
    """Ties at the decision threshold may explain a count mismatch."""
    if num_outliers == expected_outliers:
        return
    start = min(num_outliers, expected_outliers)
    end = max(num_outliers, expected_outliers)
    s = np.sort(decision)
    assert np.all(s[start:end + 1] == s[start]), \
        f"{num_outliers} outliers found, {expected_outliers} expected"


def check_outliers_train(name, estimator_orig, readonly_memmap=True):
    if not is_outlier_detector(estimator_orig):
        return
    est, X, _ = _fitted(estimator_orig)
    pred = est.predict(X)
    assert set(np.unique(pred)) <= {-1, 1}
    if hasattr(est, "decision_function") and hasattr(est, "score_samples"):
        dec, ss = est.decision_function(X), est.score_samples(X)
        np.testing.assert_allclose(dec, ss - est.offset_, rtol=1e-6, atol=1e-8)
        np.testing.assert_array_equal(pred, np.where(dec < 0, -1, 1))


def check_classifiers_multilabel_representation_invariance(name, classifier_orig):
    if not is_classifier(classifier_orig) or not _tags(classifier_orig).get("multilabel"):
        return
    X, y = _X_y(classifier_orig)
    Y = np.stack([(y == c).astype(int) for c in np.unique(y)], axis=1)
    est, _, _ = _fitted(classifier_orig, X, Y)
    p1 = est.predict(X)
    est2, _, _ = _fitted(classifier_orig, X, Y.tolist())
    np.testing.assert_array_equal(p1, est2.predict(X))


def check_classifiers_predictions(X, y, name, classifier_orig):
    est, _, _ = _fitted(classifier_orig, X, y)
    pred = est.predict(X)
    assert set(np.unique(pred)) <= set(np.unique(y))
    assert np.mean(pred == y) > 0.8


def check_classifiers_classes(name, classifier_orig):
    if not is_classifier(classifier_orig):
        return
    X, y = _X_y(classifier_orig)
    labels = np.array(["one", "two", "three"])[y % 3] if len(np.unique(y)) > 2 else \
        np.array(["neg", "pos"])[(y > 0).astype(int)]
    est, _, _ = _fitted(classifier_orig, X, labels)
    np.testing.assert_array_equal(est.classes_, np.unique(labels))
    assert set(est.predict(X)) <= set(labels)


def check_regressors_int(name, regressor_orig):
    if not is_regressor(regressor_orig):
        return
    X, y = _X_y(regressor_orig)
    yi = np.round(y * 10).astype(int)
    e1, _, _ = _fitted(regressor_orig, X, yi)
    e2, _, _ = _fitted(regressor_orig, X, yi.astype(float))
    np.testing.assert_allclose(e1.predict(X), e2.predict(X), rtol=1e-6, atol=1e-6)


def check_regressors_no_decision_function(name, regressor_orig):
    if not is_regressor(regressor_orig):
        return
    est, X, _ = _fitted(regressor_orig)
    for m in ("decision_function", "predict_proba", "predict_log_proba"):
        assert not hasattr(est, m) or m == "decision_function" and \
            type(est).__name__.endswith("SVR") is False, f"{name} regressor exposes {m}"


def check_class_weight_classifiers(name, classifier_orig):
    """Up-weighting one class raises its recall."""
    if not is_classifier(classifier_orig) or \
            "class_weight" not in classifier_orig.get_params(deep=False):
        return
    X, y = _X_y(classifier_orig)
    X = X + 2.5 * np.random.RandomState(2).randn(*X.shape)   # overlapping classes
    base, _, _ = _fitted(classifier_orig, X, y)
    w = {c: 1.0 for c in np.unique(y)}
    w[0] = 100.0
    est = _set_random_state(clone(classifier_orig)).set_params(class_weight=w)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        est.fit(X, y)
    assert np.mean(est.predict(X)[y == 0] == 0) >= np.mean(base.predict(X)[y == 0] == 0) - 1e-12


def check_class_weight_balanced_classifiers(name, classifier_orig, X_train, y_train, X_test,
                                            y_test, weights):
    from ..metrics import f1_score
    e1 = _set_random_state(clone(classifier_orig))
    e2 = _set_random_state(clone(classifier_orig)).set_params(class_weight="balanced")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        e1.fit(X_train, y_train)
        e2.fit(X_train, y_train)
    assert f1_score(y_test, e2.predict(X_test), average="weighted") > \
        f1_score(y_test, e1.predict(X_test), average="weighted")


def check_class_weight_balanced_linear_classifier(name, Classifier):
    """class_weight='balanced' equals the explicit n / (n_classes n_c)
    weights."""
    X = np.array([[-1.0, -1.0], [-1.0, 0], [-0.8, -1.0], [1.0, 1.0], [1.0, 0.0]])
    y = np.array([1, 1, 1, -1, -1])
    est = Classifier() if isinstance(Classifier, type) else clone(Classifier)
    params = est.get_params(deep=False)
    for k, v in (("fit_intercept", False), ("max_iter", 1000), ("random_state", 0)):
        if k in params:
            est.set_params(**{k: v})
    e1 = clone(est).set_params(class_weight="balanced").fit(X, y)
    n, classes = len(y), np.unique(y)
    cw = {c: n / (len(classes) * np.sum(y == c)) for c in classes}
    e2 = clone(est).set_params(class_weight=cw).fit(X, y)
    np.testing.assert_allclose(e1.coef_, e2.coef_, rtol=1e-6, atol=1e-8)


def check_estimators_overwrite_params(name, estimator_orig):
    check_dont_overwrite_parameters(name, estimator_orig)


def check_sparsify_coefficients(name, estimator_orig):
    if not hasattr(estimator_orig, "sparsify"):
        return
    est, X, _ = _fitted(estimator_orig)
    p = est.predict(X)
    est.sparsify()
    np.testing.assert_array_equal(est.predict(X), p)
    est.densify()
    np.testing.assert_array_equal(est.predict(X), p)


def check_estimators_data_not_an_array(name, estimator_orig, X=None, y=None, obj_type=None):
    if X is None:
        X, y = _X_y(estimator_orig)
    e1, _, _ = _fitted(estimator_orig, X, y)
    e2, _, _ = _fitted(estimator_orig, [list(r) for r in X], list(y))
    a, b = _outputs(e1, X), _outputs(e2, X)
    for k in a:
        if k in b:
            np.testing.assert_allclose(a[k], b[k], rtol=1e-6, atol=1e-6)


def check_classifier_data_not_an_array(name, estimator_orig):
    if is_classifier(estimator_orig):
        check_estimators_data_not_an_array(name, estimator_orig)


def check_regressor_data_not_an_array(name, estimator_orig):
    if is_regressor(estimator_orig):
        check_estimators_data_not_an_array(name, estimator_orig)


def check_non_transformer_estimators_n_iter(name, estimator_orig):
    if hasattr(estimator_orig, "transform") or "max_iter" not in \
            estimator_orig.get_params(deep=False):
        return
    est, _, _ = _fitted(estimator_orig)
    if hasattr(est, "n_iter_"):
        assert np.all(np.asarray(est.n_iter_) >= 1)


def check_transformer_n_iter(name, estimator_orig):
    if not hasattr(estimator_orig, "transform") or "max_iter" not in \
            estimator_orig.get_params(deep=False):
        return
    est, _, _ = _fitted(estimator_orig)
    if hasattr(est, "n_iter_"):
        assert np.all(np.asarray(est.n_iter_) >= 1)


def check_classifiers_regression_target(name, estimator_orig):
    """A continuous target is refused with 'Unknown label type'."""
    if not is_classifier(estimator_orig):
        return
    X, _ = _X_y(estimator_orig)
    y = np.linspace(0, 1, X.shape[0]) + 0.123
    try:
        clone(estimator_orig).fit(X, y)
    except ValueError as e:
        assert "label" in str(e).lower() or "target" in str(e).lower(), str(e)
        return
    raise AssertionError(f"{name} accepted a continuous target")


def check_decision_proba_consistency(name, estimator_orig):
    """decision_function and predict_proba rank the rows the same way."""
    if not (hasattr(estimator_orig, "decision_function") and
            hasattr(estimator_orig, "predict_proba")):
        return
    X, y = _blobs(100, 5, centers=2)
    est, _, _ = _fitted(estimator_orig, X, y)
    try:
        a = est.predict_proba(X)[:, 1]
        b = est.decision_function(X)
    except (AttributeError, NotImplementedError):
        return
    from scipy.stats import rankdata
    np.testing.assert_array_equal(rankdata(np.round(a, 10)), rankdata(np.round(b, 10)))


def check_fit_non_negative(name, estimator_orig):
    if not _tags(estimator_orig).get("requires_positive_X"):
        return
    X, y = _X_y(estimator_orig)
    X = X.copy()
    X[0, 0] = -1.0
    _expect_value_error(lambda: _fit(clone(estimator_orig), X, y))


def check_requires_y_none(name, estimator_orig):
    """fit(X, None) on a y-requiring estimator raises a clear ValueError."""
    if not (_supervised(estimator_orig) or _tags(estimator_orig).get("requires_y")):
        return
    X, _ = _X_y(estimator_orig)
    try:
        clone(estimator_orig).fit(X, None)
    except (ValueError, TypeError):
        return
    raise AssertionError(f"{name}.fit(X, None) did not raise")


def check_n_features_in_after_fitting(name, estimator_orig):
    est, X, y = _fitted(estimator_orig)
    assert est.n_features_in_ == X.shape[1]
    for meth in ("predict", "transform", "decision_function", "predict_proba", "score_samples"):
        if hasattr(est, meth):
            try:
                getattr(est, meth)(X[:, :-1])
            except (ValueError, IndexError, RuntimeError):
                continue
            except (AttributeError, NotImplementedError):
                continue
            raise AssertionError(f"{name}.{meth} accepted the wrong n_features")


def check_estimator_get_tags_default_keys(name, estimator_orig):
    tags = _tags(estimator_orig)
    if not tags:
        return
    for key in ("requires_fit", "X_types", "non_deterministic", "multioutput"):
        assert key in tags, f"{name} tags lack {key}"
