"""``cross_validate`` / ``cross_val_score`` / ``cross_val_predict``
(reference ``model_selection/_validation.py:47-280``); searches live in
``_search.py``.

The reference fans folds out over joblib worker processes
(``_validation.py:248``).  Here a fold's fit already fills the GPU (one
process per GPU, data resident in HBM), so folds run sequentially in this
process; ``n_jobs`` is accepted for API compatibility and ignored.  Scoring
strings cover the metrics this framework implements.
"""

import time
import warnings

import numpy as np

from ..parallel.tasks import Parallel
from ..utils.fixes import delayed
from ..base import clone, is_classifier
from ..exceptions import FitFailedWarning
from ..utils import metrics as M
from ._split import _safe_index, check_cv

_SCORERS = {
    "accuracy": (M.accuracy_score, 1.0, "predict"),
    "r2": (M.r2_score, 1.0, "predict"),
    "neg_mean_squared_error": (M.mean_squared_error, -1.0, "predict"),
    "adjusted_rand_score": (M.adjusted_rand_score, 1.0, "predict"),
}


class _PassthroughScorer:
    """est.score (picklable, so fitted searches can be checkpointed)."""

    def __call__(self, est, X, y=None):
        return est.score(X, y) if y is not None else est.score(X)


class _SimpleScorer:
    def __init__(self, name):
        self.name = name

    def __call__(self, est, X, y):
        fn, sign, method = _SCORERS[self.name]
        return sign * fn(y, getattr(est, method)(X))


def get_scorer(scoring):
    if scoring is None:
        return _PassthroughScorer()
    if callable(scoring):
        return scoring
    if scoring not in _SCORERS:
        from ..utils.metrics_extra import get_scorer_ext
        return get_scorer_ext(scoring)
    return _SimpleScorer(scoring)


def _fit_and_score(est, X, y, train, test, scorers, fit_params, return_train_score,
                   error_score):
    Xtr, Xte = _safe_index(X, train), _safe_index(X, test)
    ytr, yte = _safe_index(y, train), _safe_index(y, test)
    t0 = time.perf_counter()
    try:
        if ytr is None:
            est.fit(Xtr, **fit_params)
        else:
            est.fit(Xtr, ytr, **fit_params)
    except Exception as e:
        if error_score == "raise":
            raise
        warnings.warn(f"Estimator fit failed. The score on this train-test partition will be "
                      f"set to {error_score}. Details: {e!r}", FitFailedWarning)
        nan = {k: error_score for k in scorers}
        return {"fit_time": time.perf_counter() - t0, "score_time": 0.0, "test": nan,
                "train": dict(nan) if return_train_score else None, "estimator": est}
    fit_time = time.perf_counter() - t0
    t1 = time.perf_counter()
    def score(s, Xs, ys):
        try:
            return float(s(est, Xs, ys))
        except Exception as e:
            if error_score == "raise":
                raise
            warnings.warn(f"Scoring failed. The score on this train-test partition for these "
                          f"parameters will be set to {error_score}. Details: {e!r}",
                          UserWarning)
            return error_score
    test_scores = {k: score(s, Xte, yte) for k, s in scorers.items()}
    score_time = time.perf_counter() - t1
    train_scores = ({k: score(s, Xtr, ytr) for k, s in scorers.items()}
                    if return_train_score else None)
    return {"fit_time": fit_time, "score_time": score_time, "test": test_scores,
            "train": train_scores, "estimator": est}


def cross_validate(estimator, X, y=None, *, groups=None, scoring=None, cv=None, n_jobs=None,
                   verbose=0, fit_params=None, pre_dispatch="2*n_jobs", return_train_score=False,
                   return_estimator=False, error_score=np.nan):
    """Evaluate metric(s) by cross-validation (reference ``_validation.py:47``)."""
    cv = check_cv(cv, y, classifier=is_classifier(estimator))
    if scoring is None or callable(scoring) or isinstance(scoring, str):
        scorers = {"score": get_scorer(scoring)}
    elif isinstance(scoring, dict):
        scorers = {k: get_scorer(v) for k, v in scoring.items()}
    else:
        scorers = {s: get_scorer(s) for s in scoring}
    # one task per fold: threads, one GPU per fold when several are visible
    # (parallel/tasks.py; the reference's joblib fan-out, _validation.py:267)
    results = Parallel(n_jobs=n_jobs)(
        delayed(_fit_and_score)(clone(estimator), X, y, train, test, scorers, fit_params or {},
                                return_train_score, error_score)
        for train, test in cv.split(X, y, groups))
    out = {"fit_time": np.array([r["fit_time"] for r in results]),
           "score_time": np.array([r["score_time"] for r in results])}
    if return_estimator:
        out["estimator"] = [r["estimator"] for r in results]
    for k in scorers:
        name = "test_score" if list(scorers) == ["score"] else f"test_{k}"
        out[name] = np.array([r["test"][k] for r in results])
        if return_train_score:
            tname = "train_score" if list(scorers) == ["score"] else f"train_{k}"
            out[tname] = np.array([r["train"][k] for r in results])
    return out


def cross_val_score(estimator, X, y=None, *, groups=None, scoring=None, cv=None, n_jobs=None,
                    verbose=0, fit_params=None, pre_dispatch="2*n_jobs", error_score=np.nan):
    r = cross_validate(estimator, X, y, groups=groups, scoring=scoring, cv=cv, n_jobs=n_jobs,
                       fit_params=fit_params, error_score=error_score)
    return r["test_score"]


def cross_val_predict(estimator, X, y=None, *, groups=None, cv=None, n_jobs=None, verbose=0,
                      fit_params=None, method="predict"):
    cv = check_cv(cv, y, classifier=is_classifier(estimator))
    n = len(X) if not hasattr(X, "shape") else X.shape[0]
    def fold(est, train, test):
        ytr = _safe_index(y, train)
        if ytr is not None:
            est.fit(_safe_index(X, train), ytr, **(fit_params or {}))
        else:
            est.fit(_safe_index(X, train), **(fit_params or {}))
        return test, np.asarray(getattr(est, method)(_safe_index(X, test)))

    parts = Parallel(n_jobs=n_jobs)(delayed(fold)(clone(estimator), train, test)
                                    for train, test in cv.split(X, y, groups))
    preds = None
    for test, p in parts:
        if preds is None:
            preds = np.empty((n,) + p.shape[1:], dtype=p.dtype)
        preds[test] = p
    return preds


def __getattr__(name):
    # the curves and the permutation test are defined with the searches
    # (_search.py); the reference exposes them from _validation.py
    if name in ("learning_curve", "validation_curve", "permutation_test_score"):
        from . import _search
        return getattr(_search, name)
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
