"""Scoring metrics used by the estimators' ``score`` methods and the
evaluation pipelines (reference ``sklearn/metrics``: accuracy, r2,
confusion matrix, clustering agreement)."""

import numpy as np

from ..runtime.device import to_numpy


def accuracy_score(y_true, y_pred, *, normalize=True, sample_weight=None):
    y_true = np.asarray(to_numpy(y_true)).reshape(-1)
    y_pred = np.asarray(to_numpy(y_pred)).reshape(-1)
    if y_true.shape != y_pred.shape:
        raise ValueError("y_true and y_pred have different lengths")
    score = (y_true == y_pred).astype(np.float64)
    if sample_weight is not None:
        w = np.asarray(sample_weight, dtype=np.float64)
        return float(np.average(score, weights=w)) if normalize else float((score * w).sum())
    return float(score.mean()) if normalize else float(score.sum())


def r2_score(y_true, y_pred, *, sample_weight=None, multioutput="uniform_average"):
    """Coefficient of determination with the reference's target handling
    (``/root/reference/sklearn/metrics/_regression.py`` ``r2_score``, used by
    ``RegressorMixin.score`` at ``/root/reference/sklearn/base.py:564-566``):
    1-D targets become one output column, so ``(n,)`` and ``(n, 1)`` agree;
    per-output scores are combined by ``multioutput`` ('uniform_average' by
    default, 'raw_values', 'variance_weighted' or an array of weights); a
    constant output scores 1.0 when predicted exactly, else 0.0."""
    from .metrics_extra import r2_score_ext
    return r2_score_ext(to_numpy(y_true), to_numpy(y_pred), sample_weight=sample_weight,
                        multioutput=multioutput)


def confusion_matrix(y_true, y_pred, *, labels=None, sample_weight=None, normalize=None):
    """C[i, j] = (weighted) count of samples of true class labels[i]
    predicted as labels[j] (reference ``metrics/_classification.py:222``);
    ``normalize`` in {'true', 'pred', 'all'} divides by the row sums, the
    column sums or the total (0/0 -> 0).  One scatter-add, no Python loop."""
    y_true = np.asarray(to_numpy(y_true)).reshape(-1)
    y_pred = np.asarray(to_numpy(y_pred)).reshape(-1)
    if y_true.shape[0] != y_pred.shape[0]:
        raise ValueError("Found input variables with inconsistent numbers of samples: "
                         f"[{y_true.shape[0]}, {y_pred.shape[0]}]")
    if normalize not in ("true", "pred", "all", None):
        raise ValueError("normalize must be one of {'true', 'pred', 'all', None}")
    if labels is None:
        labels = np.unique(np.concatenate([y_true, y_pred]))
    else:
        labels = np.asarray(labels)
        if labels.size == 0:
            raise ValueError("'labels' should contains at least one label.")
        if y_true.size == 0:
            return np.zeros((labels.size, labels.size), dtype=int)
        if not np.isin(y_true, labels).any():
            raise ValueError("At least one label specified must be in y_true")
    n = labels.size
    if sample_weight is None:
        sw = np.ones(y_true.shape[0], dtype=np.int64)
    else:
        sw = np.asarray(sample_weight).reshape(-1)
        if sw.shape[0] != y_true.shape[0]:
            raise ValueError("Found input variables with inconsistent numbers of samples.")
    dtype = np.int64 if sw.dtype.kind in "iub" else np.float64
    # map labels to indices (labels need not be sorted); unknown -> dropped
    order = np.argsort(labels, kind="stable")
    sl = labels[order]

    def index(y):
        pos = np.clip(np.searchsorted(sl, y), 0, n - 1)
        ok = sl[pos] == y
        return order[pos], ok

    ti, tok = index(y_true)
    pi, pok = index(y_pred)
    keep = tok & pok
    cm = np.zeros((n, n), dtype=dtype)
    np.add.at(cm, (ti[keep], pi[keep]), sw[keep].astype(dtype))
    if normalize is not None:
        with np.errstate(all="ignore"):
            if normalize == "true":
                cm = cm / cm.sum(axis=1, keepdims=True)
            elif normalize == "pred":
                cm = cm / cm.sum(axis=0, keepdims=True)
            else:
                cm = cm / cm.sum()
        cm = np.nan_to_num(cm)
    return cm


def adjusted_rand_score(labels_true, labels_pred):
    """Adjusted Rand index (Hubert & Arabie)."""
    a = np.asarray(to_numpy(labels_true)).reshape(-1)
    b = np.asarray(to_numpy(labels_pred)).reshape(-1)
    _, ai = np.unique(a, return_inverse=True)
    _, bi = np.unique(b, return_inverse=True)
    cont = np.zeros((ai.max() + 1, bi.max() + 1), dtype=np.int64)
    np.add.at(cont, (ai, bi), 1)

    def c2(x):
        return (x * (x - 1) / 2.0).sum()
    n = a.size
    sum_comb = c2(cont)
    sa = c2(cont.sum(1))
    sb = c2(cont.sum(0))
    exp = sa * sb / (n * (n - 1) / 2.0) if n > 1 else 0.0
    mx = (sa + sb) / 2.0
    if mx == exp:
        return 1.0
    return float((sum_comb - exp) / (mx - exp))


def mean_squared_error(y_true, y_pred):
    y_true = np.asarray(to_numpy(y_true), dtype=np.float64)
    y_pred = np.asarray(to_numpy(y_pred), dtype=np.float64)
    return float(np.mean((y_true - y_pred) ** 2))
