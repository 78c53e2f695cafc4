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


def r2_score(y_true, y_pred, *, sample_weight=None):
    y_true = np.asarray(to_numpy(y_true), dtype=np.float64)
    y_pred = np.asarray(to_numpy(y_pred), dtype=np.float64)
    w = np.ones_like(y_true) if sample_weight is None else np.asarray(sample_weight, dtype=np.float64)
    num = (w * (y_true - y_pred) ** 2).sum()
    den = (w * (y_true - np.average(y_true, weights=w)) ** 2).sum()
    if den == 0:
        return 1.0 if num == 0 else 0.0
    return float(1 - num / den)


def confusion_matrix(y_true, y_pred, *, labels=None):
    y_true = np.asarray(to_numpy(y_true)).reshape(-1)
    y_pred = np.asarray(to_numpy(y_pred)).reshape(-1)
    if labels is None:
        labels = np.unique(np.concatenate([y_true, y_pred]))
    idx = {l: i for i, l in enumerate(labels)}
    cm = np.zeros((len(labels), len(labels)), dtype=np.int64)
    for t, p in zip(y_true, y_pred):
        if t in idx and p in idx:
            cm[idx[t], idx[p]] += 1
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
