"""Model inspection (reference ``sklearn/inspection``):
``permutation_importance`` (``_permutation_importance.py:108``; one
RandomState(seed) per column, the same shuffles as the reference) and
``partial_dependence`` (``_partial_dependence.py:222``, brute-force
method: the grid is swept with one batched predict per grid point)."""

from itertools import product

import numpy as np
import scipy.sparse as sp
from scipy.stats.mstats import mquantiles

from .base import is_classifier, is_regressor
from .utils import Bunch
from .utils.metrics_extra import check_scoring
from .utils.validation import check_random_state


def _np(a):
    return a.detach().cpu().numpy() if hasattr(a, "detach") else np.asarray(a)


def _weights_scorer(scorer, est, X, y, sw):
    if sw is not None:
        return scorer(est, X, y, sample_weight=sw)
    return scorer(est, X, y)


def _permutation_scores(est, X, y, sw, col, seed, n_repeats, scorer, max_samples):
    rs = check_random_state(seed)
    if max_samples < X.shape[0]:
        rows = rs.choice(X.shape[0], max_samples, replace=False)
        X = X[rows]
        y = y[rows]
        sw = sw[rows] if sw is not None else None
    Xp = X.copy()
    idx = np.arange(Xp.shape[0])
    scores = []
    for _ in range(n_repeats):
        rs.shuffle(idx)
        if hasattr(Xp, "iloc"):
            c = Xp.iloc[idx, col]
            c.index = Xp.index
            Xp.iloc[:, col] = c
        else:
            Xp[:, col] = Xp[idx, col]
        scores.append(_weights_scorer(scorer, est, Xp, y, sw))
    return np.array(scores)


def permutation_importance(estimator, X, y, *, scoring=None, n_repeats=5, n_jobs=None,
                           random_state=None, sample_weight=None, max_samples=1.0):
    """Mean/std drop in score when each feature column is shuffled."""
    if not hasattr(X, "iloc"):
        X = np.asarray(X)
    y = np.asarray(y) if y is not None else None
    rs = check_random_state(random_state)
    seed = rs.randint(np.iinfo(np.int32).max + 1)
    if not isinstance(max_samples, (int, np.integer)):
        max_samples = int(max_samples * X.shape[0])
    elif not (0 < max_samples <= X.shape[0]):
        raise ValueError("max_samples must be in (0, n_samples]")
    scorer = check_scoring(estimator, scoring=scoring)
    base = _weights_scorer(scorer, estimator, X, y, sample_weight)
    scores = [_permutation_scores(estimator, X, y, sample_weight, c, seed, n_repeats, scorer,
                                  max_samples) for c in range(X.shape[1])]
    imp = base - np.array(scores)
    return Bunch(importances_mean=np.mean(imp, axis=1), importances_std=np.std(imp, axis=1),
                 importances=imp)


def _grid_from_X(X, percentiles, grid_resolution):
    if len(percentiles) != 2:
        raise ValueError("'percentiles' must be a sequence of 2 elements.")
    if not all(0 <= x <= 1 for x in percentiles):
        raise ValueError("'percentiles' values must be in [0, 1].")
    if percentiles[0] >= percentiles[1]:
        raise ValueError("percentiles[0] must be strictly less than percentiles[1].")
    if grid_resolution <= 1:
        raise ValueError("'grid_resolution' must be strictly greater than 1.")
    values = []
    for f in range(X.shape[1]):
        col = X[:, f]
        uniq = np.unique(col)
        if uniq.shape[0] < grid_resolution:
            axis = uniq
        else:
            emp = mquantiles(col, prob=percentiles, axis=0)
            if np.allclose(emp[0], emp[1]):
                raise ValueError("percentiles are too close to each other, unable to build the "
                                 "grid. Please choose percentiles that are further apart.")
            axis = np.linspace(emp[0], emp[1], num=grid_resolution, endpoint=True)
        values.append(axis)
    return np.asarray(list(product(*values))), values


def _response(est, X, method):
    if is_regressor(est):
        return _np(est.predict(X))
    if method == "auto":
        for m in ("predict_proba", "decision_function"):
            if hasattr(est, m):
                method = m
                break
    out = _np(getattr(est, method)(X))
    if out.ndim == 1:
        out = out[:, None]
    if method == "predict_proba" and out.shape[1] == 2:
        out = out[:, 1:]
    return out


def partial_dependence(estimator, X, features, *, response_method="auto",
                       percentiles=(0.05, 0.95), grid_resolution=100, method="auto",
                       kind="legacy"):
    """Averaged (and optionally individual) model response over a grid of
    values of ``features`` (brute method)."""
    if not (is_classifier(estimator) or is_regressor(estimator)):
        raise ValueError("'estimator' must be a fitted regressor or classifier.")
    if method not in ("auto", "brute"):
        raise ValueError("Only the 'brute' method is implemented (gradient-boosting recursion "
                         "falls back to brute force).")
    X = X.toarray() if sp.issparse(X) else np.asarray(X)
    features = np.atleast_1d(np.asarray(features)).ravel()
    if features.dtype == bool:
        features = np.flatnonzero(features)
    grid, values = _grid_from_X(X[:, features], percentiles, grid_resolution)
    Xe = X.copy()
    preds = []
    for point in grid:
        Xe[:, features] = point
        preds.append(_response(estimator, Xe, response_method))
    P = np.asarray(preds)
    if P.ndim == 2:
        P = P[:, :, None]
    # P: (n_points, n_samples, n_outputs) -> (n_outputs, n_samples, *grid_shape)
    P = P.transpose(2, 1, 0)
    shape = tuple(v.shape[0] for v in values)
    indiv = P.reshape(P.shape[0], P.shape[1], *shape)
    avg = indiv.mean(axis=1)
    if kind == "legacy":
        return avg, values
    if kind == "average":
        return Bunch(average=avg, values=values, grid_values=values)
    if kind == "individual":
        return Bunch(individual=indiv, values=values, grid_values=values)
    return Bunch(average=avg, individual=indiv, values=values, grid_values=values)


from ._inspection_plot import PartialDependenceDisplay, plot_partial_dependence  # noqa: E402

__all__ = ["permutation_importance", "partial_dependence", "PartialDependenceDisplay",
           "plot_partial_dependence"]

from .utils._aliases import alias_submodules  # noqa: E402
alias_submodules(__name__, "_partial_dependence")

from .utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
