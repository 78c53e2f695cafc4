"""Classification, regression and ranking metrics (reference
``metrics/_classification.py``, ``_regression.py``, ``_ranking.py``,
``_scorer.py``).  Host numpy: metrics are O(n) reductions over label /
score vectors that are already on the host after ``predict``."""

import warnings

import numpy as np
from scipy.special import xlogy

from ..exceptions import UndefinedMetricWarning
from ..runtime.device import to_numpy


def _arr(a, dtype=None):
    a = np.asarray(to_numpy(a))
    return a.astype(dtype) if dtype is not None else a


from .multiclass import type_of_target, unique_labels  # noqa: E402  (one definition)


def _check_targets(y_true, y_pred):
    y_true, y_pred = _arr(y_true), _arr(y_pred)
    if y_true.shape[0] != y_pred.shape[0]:
        raise ValueError("Found input variables with inconsistent numbers of samples: [%d, %d]"
                         % (y_true.shape[0], y_pred.shape[0]))
    tt, tp = type_of_target(y_true), type_of_target(y_pred)
    types = {tt, tp}
    if types == {"binary", "multiclass"}:
        types = {"multiclass"}
    if len(types) > 1:
        raise ValueError("Classification metrics can't handle a mix of {0} and {1} targets"
                         .format(tt, tp))
    t = types.pop()
    if t not in ("binary", "multiclass", "multilabel-indicator"):
        raise ValueError("{0} is not supported".format(t))
    if t == "binary" and len(unique_labels(y_true, y_pred)) > 2:
        t = "multiclass"
    return t, y_true, y_pred


# ------------------------------------------------------------ classification
def multilabel_confusion_matrix(y_true, y_pred, *, sample_weight=None, labels=None,
                                samplewise=False):
    t, y_true, y_pred = _check_targets(y_true, y_pred)
    sw = None if sample_weight is None else _arr(sample_weight, float)
    if t == "multilabel-indicator":
        if labels is not None:
            y_true, y_pred = y_true[:, labels], y_pred[:, labels]
        w = np.ones(y_true.shape[0]) if sw is None else sw
        axis = 1 if samplewise else 0
        tp = ((y_true == 1) & (y_pred == 1)) * w[:, None]
        tp_sum = tp.sum(axis)
        pred_sum = ((y_pred == 1) * w[:, None]).sum(axis)
        true_sum = ((y_true == 1) * w[:, None]).sum(axis)
        total = (w.sum() if not samplewise else np.full(y_true.shape[0], y_true.shape[1]) * w)
    else:
        present = unique_labels(y_true, y_pred)
        labels = present if labels is None else np.asarray(labels)
        w = np.ones(len(y_true)) if sw is None else sw
        tp_sum = np.array([np.sum(w[(y_true == c) & (y_pred == c)]) for c in labels])
        pred_sum = np.array([np.sum(w[y_pred == c]) for c in labels])
        true_sum = np.array([np.sum(w[y_true == c]) for c in labels])
        total = w.sum()
    fp = pred_sum - tp_sum
    fn = true_sum - tp_sum
    tn = total - tp_sum - fp - fn
    return np.array([tn, fp, fn, tp_sum]).T.reshape(-1, 2, 2)


def _prf_divide(num, den, metric, modifier, average, warn_for, zero_division="warn"):
    mask = den == 0.0
    den = den.copy()
    den[mask] = 1
    res = num / den
    if np.any(mask):
        zd = 0.0 if zero_division == "warn" else float(zero_division)
        res[mask] = zd
        if zero_division == "warn" and metric in warn_for:
            warnings.warn("{0} is ill-defined and being set to 0.0 in labels with no {1} "
                          "samples.".format(metric.capitalize(), modifier),
                          UndefinedMetricWarning, stacklevel=3)
    return res


def precision_recall_fscore_support(y_true, y_pred, *, beta=1.0, labels=None, pos_label=1,
                                    average=None, warn_for=("precision", "recall", "f-score"),
                                    sample_weight=None, zero_division="warn"):
    if beta < 0:
        raise ValueError("beta should be >=0 in the F-beta score")
    t, yt, yp = _check_targets(y_true, y_pred)
    if average == "binary":
        if t == "binary":
            present = unique_labels(yt, yp)
            if len(present) >= 2 and pos_label not in present:
                raise ValueError("pos_label=%r is not a valid label. It should be one of %s"
                                 % (pos_label, present))
            labels = [pos_label]
        else:
            raise ValueError("Target is %s but average='binary'. Please choose another average "
                             "setting, one of [None, 'micro', 'macro', 'weighted']." % t)
    samplewise = average == "samples"
    mcm = multilabel_confusion_matrix(yt, yp, sample_weight=sample_weight, labels=labels,
                                      samplewise=samplewise)
    tp_sum, pred_sum, true_sum = mcm[:, 1, 1], mcm[:, 1, 1] + mcm[:, 0, 1], \
        mcm[:, 1, 1] + mcm[:, 1, 0]
    if average == "micro":
        tp_sum, pred_sum, true_sum = (np.array([tp_sum.sum()]), np.array([pred_sum.sum()]),
                                      np.array([true_sum.sum()]))
    beta2 = beta ** 2
    precision = _prf_divide(tp_sum, pred_sum, "precision", "predicted", average, warn_for,
                            zero_division)
    recall = _prf_divide(tp_sum, true_sum, "recall", "true", average, warn_for, zero_division)
    if np.isposinf(beta):
        f = recall
    else:
        den = beta2 * precision + recall
        den[den == 0.0] = 1
        f = (1 + beta2) * precision * recall / den
    if average == "weighted":
        weights = true_sum
        if weights.sum() == 0:
            zd = 0.0 if zero_division == "warn" else float(zero_division)
            return zd, zd, zd, None
    elif average == "samples":
        weights = sample_weight
    else:
        weights = None
    if average is not None:
        precision = float(np.average(precision, weights=weights))
        recall = float(np.average(recall, weights=weights))
        f = float(np.average(f, weights=weights))
        true_sum = None
    return precision, recall, f, true_sum


def fbeta_score(y_true, y_pred, *, beta, labels=None, pos_label=1, average="binary",
                sample_weight=None, zero_division="warn"):
    return precision_recall_fscore_support(y_true, y_pred, beta=beta, labels=labels,
                                           pos_label=pos_label, average=average,
                                           warn_for=("f-score",), sample_weight=sample_weight,
                                           zero_division=zero_division)[2]


def f1_score(y_true, y_pred, *, labels=None, pos_label=1, average="binary", sample_weight=None,
             zero_division="warn"):
    return fbeta_score(y_true, y_pred, beta=1, labels=labels, pos_label=pos_label,
                       average=average, sample_weight=sample_weight, zero_division=zero_division)


def precision_score(y_true, y_pred, *, labels=None, pos_label=1, average="binary",
                    sample_weight=None, zero_division="warn"):
    return precision_recall_fscore_support(y_true, y_pred, labels=labels, pos_label=pos_label,
                                           average=average, warn_for=("precision",),
                                           sample_weight=sample_weight,
                                           zero_division=zero_division)[0]


def recall_score(y_true, y_pred, *, labels=None, pos_label=1, average="binary",
                 sample_weight=None, zero_division="warn"):
    return precision_recall_fscore_support(y_true, y_pred, labels=labels, pos_label=pos_label,
                                           average=average, warn_for=("recall",),
                                           sample_weight=sample_weight,
                                           zero_division=zero_division)[1]


def balanced_accuracy_score(y_true, y_pred, *, sample_weight=None, adjusted=False):
    from .metrics import confusion_matrix
    C = confusion_matrix(y_true, y_pred) if sample_weight is None else \
        _weighted_confusion(y_true, y_pred, sample_weight)
    with np.errstate(divide="ignore", invalid="ignore"):
        per_class = np.diag(C) / C.sum(axis=1)
    if np.any(np.isnan(per_class)):
        warnings.warn("y_pred contains classes not in y_true")
        per_class = per_class[~np.isnan(per_class)]
    score = np.mean(per_class)
    if adjusted:
        chance = 1 / len(per_class)
        score = (score - chance) / (1 - chance)
    return float(score)


def _weighted_confusion(y_true, y_pred, sample_weight, labels=None):
    yt, yp = _arr(y_true), _arr(y_pred)
    labels = unique_labels(yt, yp) if labels is None else np.asarray(labels)
    idx = {v: i for i, v in enumerate(labels.tolist())}
    C = np.zeros((len(labels), len(labels)))
    for a, b, w in zip(yt.tolist(), yp.tolist(), _arr(sample_weight, float)):
        if a in idx and b in idx:
            C[idx[a], idx[b]] += w
    return C


def cohen_kappa_score(y1, y2, *, labels=None, weights=None, sample_weight=None):
    C = _weighted_confusion(y1, y2, np.ones(len(_arr(y1))) if sample_weight is None
                            else sample_weight, labels)
    n = C.shape[0]
    expected = np.outer(C.sum(1), C.sum(0)) / C.sum()
    if weights is None:
        W = np.ones((n, n)) - np.eye(n)
    else:
        W = np.abs(np.subtract.outer(np.arange(n), np.arange(n))).astype(float)
        if weights == "quadratic":
            W = W ** 2
    return float(1 - np.sum(W * C) / np.sum(W * expected))


def matthews_corrcoef(y_true, y_pred, *, sample_weight=None):
    yt, yp = _arr(y_true), _arr(y_pred)
    C = _weighted_confusion(yt, yp, np.ones(len(yt)) if sample_weight is None else sample_weight)
    t_sum, p_sum = C.sum(1), C.sum(0)
    n_correct = np.trace(C)
    n = C.sum()
    cov_ytyp = n_correct * n - np.dot(t_sum, p_sum)
    cov_ypyp = n ** 2 - np.dot(p_sum, p_sum)
    cov_ytyt = n ** 2 - np.dot(t_sum, t_sum)
    if cov_ypyp * cov_ytyt == 0:
        return 0.0
    return float(cov_ytyp / np.sqrt(cov_ytyt * cov_ypyp))


def hamming_loss(y_true, y_pred, *, sample_weight=None):
    yt, yp = _arr(y_true), _arr(y_pred)
    w = 1.0 if sample_weight is None else _arr(sample_weight, float)
    if yt.ndim == 2:
        return float(np.average((yt != yp).mean(axis=1), weights=None if np.isscalar(w) else w))
    return float(np.average(yt != yp, weights=None if np.isscalar(w) else w))


def zero_one_loss(y_true, y_pred, *, normalize=True, sample_weight=None):
    from .metrics import accuracy_score
    yt, yp = _arr(y_true), _arr(y_pred)
    if yt.ndim == 2:
        score = np.all(yt == yp, axis=1).astype(float)
        s = np.average(score, weights=sample_weight) if normalize else \
            (score if sample_weight is None else score * _arr(sample_weight, float)).sum()
    else:
        s = accuracy_score(yt, yp, normalize=normalize, sample_weight=sample_weight)
    if normalize:
        return float(1 - s)
    n = len(yt) if sample_weight is None else float(np.sum(sample_weight))
    return float(n - s)


def jaccard_score(y_true, y_pred, *, labels=None, pos_label=1, average="binary",
                  sample_weight=None, zero_division="warn"):
    t, yt, yp = _check_targets(y_true, y_pred)
    if average == "binary":
        if t != "binary":
            raise ValueError("Target is %s but average='binary'." % t)
        labels = [pos_label]
    mcm = multilabel_confusion_matrix(yt, yp, sample_weight=sample_weight, labels=labels,
                                      samplewise=average == "samples")
    num = mcm[:, 1, 1]
    den = mcm[:, 1, 1] + mcm[:, 0, 1] + mcm[:, 1, 0]
    if average == "micro":
        num, den = np.array([num.sum()]), np.array([den.sum()])
    j = _prf_divide(num, den, "jaccard", "true or predicted", average, ("jaccard",),
                    zero_division)
    if average is None:
        return j
    w = (mcm[:, 1, 0] + mcm[:, 1, 1]) if average == "weighted" else \
        (sample_weight if average == "samples" else None)
    return float(np.average(j, weights=w))


def log_loss(y_true, y_pred, *, eps=1e-15, normalize=True, sample_weight=None, labels=None):
    yp = _arr(y_pred, float)
    yt = _arr(y_true)
    lab = np.unique(yt) if labels is None else np.asarray(labels)
    if len(lab) == 1:
        raise ValueError("y_true contains only one label ({0}). Please provide the true labels "
                         "explicitly through the labels argument.".format(lab[0]))
    Y = (yt[:, None] == lab[None, :]).astype(float)
    if Y.shape[1] == 2 and yp.ndim == 1:
        yp = np.c_[1 - yp, yp]
    if yp.ndim == 1:
        yp = yp[:, None]
    if yp.shape[1] == 1:
        yp = np.c_[1 - yp, yp]
    if Y.shape[1] == 1:
        Y = np.c_[1 - Y, Y]
    if yp.shape[1] != Y.shape[1]:
        raise ValueError("y_true and y_pred contain different number of classes")
    yp = np.clip(yp, eps, 1 - eps)
    yp = yp / yp.sum(axis=1, keepdims=True)
    loss = -(Y * np.log(yp)).sum(axis=1)
    if normalize:
        return float(np.average(loss, weights=sample_weight))
    return float(np.sum(loss if sample_weight is None else loss * sample_weight))


def hinge_loss(y_true, pred_decision, *, labels=None, sample_weight=None):
    yt = _arr(y_true)
    pd = _arr(pred_decision, float)
    lab = np.unique(yt if labels is None else labels)
    if pd.ndim == 1 or len(lab) <= 2:
        y = np.where(yt == lab[-1], 1.0, -1.0)
        margin = y * pd.ravel()
    else:
        mask = yt[:, None] == lab[None, :]
        margin = pd[mask] - np.max(np.where(mask, -np.inf, pd), axis=1)
    losses = np.maximum(1 - margin, 0)
    return float(np.average(losses, weights=sample_weight))


def brier_score_loss(y_true, y_prob, *, sample_weight=None, pos_label=None):
    yt, yp = _arr(y_true), _arr(y_prob, float)
    if pos_label is None:
        pos_label = 1 if set(np.unique(yt).tolist()) <= {0, 1, -1} else np.unique(yt)[-1]
    y = (yt == pos_label).astype(float)
    return float(np.average((y - yp) ** 2, weights=sample_weight))


def classification_report(y_true, y_pred, *, labels=None, target_names=None, sample_weight=None,
                          digits=2, output_dict=False, zero_division="warn"):
    yt, yp = _arr(y_true), _arr(y_pred)
    labels = unique_labels(yt, yp) if labels is None else np.asarray(labels)
    p, r, f, s = precision_recall_fscore_support(yt, yp, labels=labels, average=None,
                                                 sample_weight=sample_weight,
                                                 zero_division=zero_division)
    names = [str(t) for t in (target_names if target_names is not None else labels)]
    rep = {n: {"precision": p[i], "recall": r[i], "f1-score": f[i], "support": s[i]}
           for i, n in enumerate(names)}
    from .metrics import accuracy_score
    rep["accuracy"] = accuracy_score(yt, yp, sample_weight=sample_weight)
    for avg in ("macro", "weighted"):
        pa, ra, fa, _ = precision_recall_fscore_support(yt, yp, labels=labels, average=avg,
                                                        sample_weight=sample_weight,
                                                        zero_division=zero_division)
        rep[avg + " avg"] = {"precision": pa, "recall": ra, "f1-score": fa,
                             "support": float(np.sum(s))}
    if output_dict:
        return rep
    width = max(max(len(n) for n in names), len("weighted avg"), digits)
    head = "{:>{w}s} " + " {:>9}" * 4
    lines = [head.format("", "precision", "recall", "f1-score", "support", w=width), ""]
    row = "{:>{w}s} " + " {:>9.{d}f}" * 3 + " {:>9}"
    for n in names:
        v = rep[n]
        lines.append(row.format(n, v["precision"], v["recall"], v["f1-score"],
                                int(v["support"]), w=width, d=digits))
    lines.append("")
    lines.append(("{:>{w}s} " + " {:>9}" * 2 + " {:>9.{d}f} {:>9}").format(
        "accuracy", "", "", rep["accuracy"], int(np.sum(s)), w=width, d=digits))
    for avg in ("macro avg", "weighted avg"):
        v = rep[avg]
        lines.append(row.format(avg, v["precision"], v["recall"], v["f1-score"],
                                int(v["support"]), w=width, d=digits))
    return "\n".join(lines) + "\n"


# ---------------------------------------------------------------- ranking
def _binary_clf_curve(y_true, y_score, pos_label=None, sample_weight=None):
    yt, ys = _arr(y_true), _arr(y_score, float)
    if pos_label is None:
        pos_label = 1.0 if set(np.unique(yt).tolist()) <= {0, 1, -1} else np.unique(yt)[-1]
    y = (yt == pos_label)
    w = np.ones_like(ys) if sample_weight is None else _arr(sample_weight, float)
    order = np.argsort(ys, kind="mergesort")[::-1]
    ys, y, w = ys[order], y[order], w[order]
    distinct = np.where(np.diff(ys))[0]
    thr_idx = np.r_[distinct, y.size - 1]
    tps = np.cumsum(y * w)[thr_idx]
    fps = np.cumsum((1 - y) * w)[thr_idx] if sample_weight is not None else 1 + thr_idx - tps
    return fps, tps, ys[thr_idx]


def roc_curve(y_true, y_score, *, pos_label=None, sample_weight=None,
              drop_intermediate=True):
    fps, tps, thr = _binary_clf_curve(y_true, y_score, pos_label, sample_weight)
    if drop_intermediate and len(fps) > 2:
        opt = np.where(np.r_[True, np.logical_or(np.diff(fps, 2), np.diff(tps, 2)), True])[0]
        fps, tps, thr = fps[opt], tps[opt], thr[opt]
    tps = np.r_[0, tps]
    fps = np.r_[0, fps]
    thr = np.r_[np.inf, thr]
    fpr = fps / fps[-1] if fps[-1] > 0 else np.full(fps.shape, np.nan)
    tpr = tps / tps[-1] if tps[-1] > 0 else np.full(tps.shape, np.nan)
    return fpr, tpr, thr


def auc(x, y):
    x, y = _arr(x, float), _arr(y, float)
    direction = 1
    dx = np.diff(x)
    if np.any(dx < 0):
        if np.all(dx <= 0):
            direction = -1
        else:
            raise ValueError("x is neither increasing nor decreasing : {}.".format(x))
    return float(direction * np.trapezoid(y, x) if hasattr(np, "trapezoid")
                 else direction * np.trapz(y, x))


def precision_recall_curve(y_true, probas_pred, *, pos_label=None, sample_weight=None):
    fps, tps, thr = _binary_clf_curve(y_true, probas_pred, pos_label, sample_weight)
    ps = tps + fps
    precision = np.divide(tps, ps, out=np.ones_like(tps, dtype=float), where=ps != 0)
    recall = np.ones_like(tps, dtype=float) if tps[-1] == 0 else tps / tps[-1]
    last = tps.searchsorted(tps[-1])
    sl = slice(last, None, -1)
    return np.r_[precision[sl], 1], np.r_[recall[sl], 0], thr[sl]


def average_precision_score(y_true, y_score, *, average="macro", pos_label=1,
                            sample_weight=None):
    yt, ys = _arr(y_true), _arr(y_score, float)
    if yt.ndim == 2:
        scores = [average_precision_score(yt[:, k], ys[:, k], sample_weight=sample_weight)
                  for k in range(yt.shape[1])]
        return float(np.mean(scores)) if average == "macro" else np.asarray(scores)
    p, r, _ = precision_recall_curve(yt, ys, pos_label=pos_label, sample_weight=sample_weight)
    return float(-np.sum(np.diff(r) * np.array(p)[:-1]))


def roc_auc_score(y_true, y_score, *, average="macro", sample_weight=None, max_fpr=None,
                  multi_class="raise", labels=None):
    yt, ys = _arr(y_true), _arr(y_score, float)
    if yt.ndim == 1 and ys.ndim == 2 and ys.shape[1] > 2:
        if multi_class == "raise":
            raise ValueError("multi_class must be in ('ovo', 'ovr')")
        classes = np.unique(yt) if labels is None else np.asarray(labels)
        if multi_class == "ovr":
            Y = (yt[:, None] == classes[None, :]).astype(int)
            aucs = np.array([roc_auc_score(Y[:, k], ys[:, k], sample_weight=sample_weight)
                             for k in range(len(classes))])
            return float(np.average(aucs, weights=Y.sum(0) if average == "weighted" else None))
        scores = []
        for a in range(len(classes)):
            for b in range(a + 1, len(classes)):
                m = (yt == classes[a]) | (yt == classes[b])
                s_ab = roc_auc_score(yt[m] == classes[a], ys[m, a])
                s_ba = roc_auc_score(yt[m] == classes[b], ys[m, b])
                scores.append((s_ab + s_ba) / 2)
        return float(np.mean(scores))
    if ys.ndim == 2 and ys.shape[1] == 2 and yt.ndim == 1:
        ys = ys[:, 1]
    if yt.ndim == 2:
        aucs = np.array([roc_auc_score(yt[:, k], ys[:, k], sample_weight=sample_weight)
                         for k in range(yt.shape[1])])
        if average is None:
            return aucs
        if average == "micro":
            return roc_auc_score(yt.ravel(), ys.ravel())
        return float(np.average(aucs, weights=yt.sum(0) if average == "weighted" else None))
    if len(np.unique(yt)) != 2:
        raise ValueError("Only one class present in y_true. ROC AUC score is not defined in "
                         "that case.")
    fpr, tpr, _ = roc_curve(yt, ys, sample_weight=sample_weight)
    if max_fpr is None or max_fpr == 1:
        return auc(fpr, tpr)
    stop = np.searchsorted(fpr, max_fpr, "right")
    x_interp = [fpr[stop - 1], fpr[stop]]
    y_interp = [tpr[stop - 1], tpr[stop]]
    tpr = np.append(tpr[:stop], np.interp(max_fpr, x_interp, y_interp))
    fpr = np.append(fpr[:stop], max_fpr)
    partial = auc(fpr, tpr)
    min_area = 0.5 * max_fpr ** 2
    return float(0.5 * (1 + (partial - min_area) / (max_fpr - min_area)))


def det_curve(y_true, y_score, pos_label=None, sample_weight=None):
    """False positive / false negative rates per threshold (reference
    ``metrics/_ranking.py:235``): from the last threshold with no false
    positive beyond the first one, to the first one with no false negative,
    in order of decreasing false positive rate."""
    if len(np.unique(np.asarray(y_true))) != 2:
        raise ValueError("Only one class present in y_true. Detection error tradeoff curve is "
                         "not defined in that case.")
    fps, tps, thr = _binary_clf_curve(y_true, y_score, pos_label, sample_weight)
    fns = tps[-1] - tps
    p, n = tps[-1], fps[-1]
    first = fps.searchsorted(fps[0], side="right") - 1
    last = tps.searchsorted(tps[-1]) + 1
    sl = slice(max(first, 0), last)
    return fps[sl][::-1] / n, fns[sl][::-1] / p, thr[sl][::-1]


def top_k_accuracy_score(y_true, y_score, *, k=2, normalize=True, sample_weight=None,
                         labels=None):
    yt, ys = _arr(y_true), _arr(y_score, float)
    classes = np.unique(yt) if labels is None else np.asarray(labels)
    if ys.ndim == 1:
        hits = (ys >= 0.5).astype(int) == (yt == classes[-1]) if k == 1 else np.ones(len(yt), bool)
    else:
        top = np.argsort(ys, axis=1, kind="stable")[:, ::-1][:, :k]
        enc = np.searchsorted(classes, yt)
        hits = (top == enc[:, None]).any(axis=1)
    if normalize:
        return float(np.average(hits, weights=sample_weight))
    return float(np.sum(hits if sample_weight is None else hits * sample_weight))


def label_ranking_average_precision_score(y_true, y_score, *, sample_weight=None):
    yt, ys = _arr(y_true), _arr(y_score, float)
    out = np.zeros(yt.shape[0])
    for i in range(yt.shape[0]):
        rel = np.flatnonzero(yt[i])
        if len(rel) == 0 or len(rel) == yt.shape[1]:
            out[i] = 1.0
            continue
        s = ys[i]
        rank = np.array([np.sum(s >= s[j]) for j in rel], dtype=float)
        L = np.array([np.sum(s[rel] >= s[j]) for j in rel], dtype=float)
        out[i] = np.mean(L / rank)
    return float(np.average(out, weights=sample_weight))


def coverage_error(y_true, y_score, *, sample_weight=None):
    yt, ys = _arr(y_true), _arr(y_score, float)
    ymin = np.where(yt.astype(bool), ys, np.inf).min(axis=1, keepdims=True)
    cov = (ys >= ymin).sum(axis=1).astype(float)
    cov[~yt.astype(bool).any(axis=1)] = 0
    return float(np.average(cov, weights=sample_weight))


def label_ranking_loss(y_true, y_score, *, sample_weight=None):
    yt, ys = _arr(y_true).astype(bool), _arr(y_score, float)
    loss = np.zeros(yt.shape[0])
    for i in range(yt.shape[0]):
        pos, neg = ys[i][yt[i]], ys[i][~yt[i]]
        if len(pos) == 0 or len(neg) == 0:
            continue
        loss[i] = np.sum(pos[:, None] <= neg[None, :]) / (len(pos) * len(neg))
    return float(np.average(loss, weights=sample_weight))


def dcg_score(y_true, y_score, *, k=None, log_base=2, sample_weight=None, ignore_ties=False):
    yt, ys = _arr(y_true, float), _arr(y_score, float)
    disc = 1 / (np.log(np.arange(yt.shape[1]) + 2) / np.log(log_base))
    if k is not None:
        disc[k:] = 0
    gains = []
    for t, s in zip(yt, ys):
        order = np.argsort(s, kind="stable")[::-1]
        if ignore_ties:
            gains.append(np.sum(t[order] * disc))
        else:
            # tie-averaged gains (reference _tie_averaged_dcg)
            _, inv, counts = np.unique(-s, return_inverse=True, return_counts=True)
            ranked = np.zeros(len(counts))
            np.add.at(ranked, inv, t)
            ranked /= counts
            groups = np.cumsum(counts) - 1
            csum = np.r_[0, np.cumsum(disc)]
            disc_g = csum[groups + 1] - np.r_[0, csum[groups + 1][:-1]]
            gains.append(np.sum(ranked * disc_g))
    return float(np.average(gains, weights=sample_weight))


def ndcg_score(y_true, y_score, *, k=None, sample_weight=None, ignore_ties=False):
    yt = _arr(y_true, float)
    vals = []
    for i in range(yt.shape[0]):
        g = dcg_score(yt[i:i + 1], _arr(y_score, float)[i:i + 1], k=k, ignore_ties=ignore_ties)
        n = dcg_score(yt[i:i + 1], yt[i:i + 1], k=k, ignore_ties=True)
        vals.append(g / n if n > 0 else 0.0)
    return float(np.average(vals, weights=sample_weight))


# ---------------------------------------------------------------- regression
def _reg(y_true, y_pred):
    yt, yp = _arr(y_true, float), _arr(y_pred, float)
    if yt.ndim == 1:
        yt = yt.reshape(-1, 1)
    if yp.ndim == 1:
        yp = yp.reshape(-1, 1)
    if yt.shape[0] != yp.shape[0]:
        raise ValueError("Found input variables with inconsistent numbers of samples: "
                         f"[{yt.shape[0]}, {yp.shape[0]}]")
    if yt.shape != yp.shape:
        raise ValueError("y_true and y_pred have different number of output ({0}!={1})"
                         .format(yt.shape[1], yp.shape[1]))
    return yt, yp


def _agg(errors, multioutput):
    if isinstance(multioutput, str):
        if multioutput == "raw_values":
            return errors
        return float(np.average(errors))
    return float(np.average(errors, weights=multioutput))


def mean_absolute_error(y_true, y_pred, *, sample_weight=None, multioutput="uniform_average"):
    yt, yp = _reg(y_true, y_pred)
    return _agg(np.average(np.abs(yp - yt), weights=sample_weight, axis=0), multioutput)


def mean_squared_error_ext(y_true, y_pred, *, sample_weight=None, multioutput="uniform_average",
                           squared=True):
    yt, yp = _reg(y_true, y_pred)
    e = np.average((yt - yp) ** 2, axis=0, weights=sample_weight)
    if not squared:
        e = np.sqrt(e)
    return _agg(e, multioutput)


def mean_squared_log_error(y_true, y_pred, *, sample_weight=None, multioutput="uniform_average",
                           squared=True):
    yt, yp = _reg(y_true, y_pred)
    if (yt < 0).any() or (yp < 0).any():
        raise ValueError("Mean Squared Logarithmic Error cannot be used when targets contain "
                         "negative values.")
    return mean_squared_error_ext(np.log1p(yt), np.log1p(yp), sample_weight=sample_weight,
                                  multioutput=multioutput, squared=squared)


def median_absolute_error(y_true, y_pred, *, multioutput="uniform_average", sample_weight=None):
    yt, yp = _reg(y_true, y_pred)
    if sample_weight is None:
        e = np.median(np.abs(yp - yt), axis=0)
    else:
        from .stats import _weighted_percentile
        e = np.atleast_1d(_weighted_percentile(np.abs(yp - yt), sample_weight))
    return _agg(e, multioutput)


def mean_absolute_percentage_error(y_true, y_pred, *, sample_weight=None,
                                   multioutput="uniform_average"):
    yt, yp = _reg(y_true, y_pred)
    eps = np.finfo(np.float64).eps
    e = np.average(np.abs(yp - yt) / np.maximum(np.abs(yt), eps), weights=sample_weight, axis=0)
    return _agg(e, multioutput)


def explained_variance_score(y_true, y_pred, *, sample_weight=None,
                             multioutput="uniform_average"):
    yt, yp = _reg(y_true, y_pred)
    diff_avg = np.average(yt - yp, weights=sample_weight, axis=0)
    num = np.average((yt - yp - diff_avg) ** 2, weights=sample_weight, axis=0)
    ytm = np.average(yt, weights=sample_weight, axis=0)
    den = np.average((yt - ytm) ** 2, weights=sample_weight, axis=0)
    nz_num, nz_den = num != 0, den != 0
    valid = nz_num & nz_den
    out = np.ones(yt.shape[1])
    out[valid] = 1 - num[valid] / den[valid]
    out[nz_num & ~nz_den] = 0.0
    if isinstance(multioutput, str) and multioutput == "variance_weighted":
        return float(np.average(out, weights=den))
    return _agg(out, multioutput)


def r2_score_ext(y_true, y_pred, *, sample_weight=None, multioutput="uniform_average"):
    yt, yp = _reg(y_true, y_pred)
    w = np.ones(yt.shape[0]) if sample_weight is None else _arr(sample_weight, float)
    num = (w[:, None] * (yt - yp) ** 2).sum(axis=0)
    den = (w[:, None] * (yt - np.average(yt, axis=0, weights=w)) ** 2).sum(axis=0)
    nz_num, nz_den = num != 0, den != 0
    valid = nz_num & nz_den
    out = np.ones(yt.shape[1])
    out[valid] = 1 - num[valid] / den[valid]
    out[nz_num & ~nz_den] = 0.0
    if isinstance(multioutput, str) and multioutput == "variance_weighted":
        return float(np.average(out, weights=den)) if den.sum() else 1.0
    return _agg(out, multioutput)


def max_error(y_true, y_pred):
    yt, yp = _reg(y_true, y_pred)
    if yt.shape[1] > 1:
        raise ValueError("Multioutput not supported in max_error")
    return float(np.max(np.abs(yt - yp)))


def mean_tweedie_deviance(y_true, y_pred, *, sample_weight=None, power=0):
    yt, yp = _arr(y_true, float), _arr(y_pred, float)
    if power < 0:
        dev = 2 * (np.power(np.maximum(yt, 0), 2 - power) / ((1 - power) * (2 - power))
                   - yt * np.power(yp, 1 - power) / (1 - power)
                   + np.power(yp, 2 - power) / (2 - power))
    elif power == 0:
        dev = (yt - yp) ** 2
    elif power == 1:
        dev = 2 * (xlogy(yt, yt / yp) - yt + yp)
    elif power == 2:
        dev = 2 * (np.log(yp / yt) + yt / yp - 1)
    else:
        dev = 2 * (np.power(yt, 2 - power) / ((1 - power) * (2 - power))
                   - yt * np.power(yp, 1 - power) / (1 - power)
                   + np.power(yp, 2 - power) / (2 - power))
    return float(np.average(dev, weights=sample_weight))


def mean_poisson_deviance(y_true, y_pred, *, sample_weight=None):
    return mean_tweedie_deviance(y_true, y_pred, sample_weight=sample_weight, power=1)


def mean_gamma_deviance(y_true, y_pred, *, sample_weight=None):
    return mean_tweedie_deviance(y_true, y_pred, sample_weight=sample_weight, power=2)


def mean_pinball_loss(y_true, y_pred, *, sample_weight=None, alpha=0.5,
                      multioutput="uniform_average"):
    yt, yp = _reg(y_true, y_pred)
    diff = yt - yp
    sign = (diff >= 0).astype(diff.dtype)
    loss = alpha * sign * diff - (1 - alpha) * (1 - sign) * diff
    return _agg(np.average(loss, weights=sample_weight, axis=0), multioutput)


# ---------------------------------------------------------------- scorers
class _Scorer:
    def __init__(self, score_func, sign, kwargs, response):
        self._score_func, self._sign, self._kwargs, self._response = (score_func, sign, kwargs,
                                                                      response)

    def __call__(self, estimator, X, y_true, sample_weight=None):
        if self._response == "proba":
            y = estimator.predict_proba(X)
            if y.ndim == 2 and y.shape[1] == 2 and self._score_func is not log_loss:
                y = y[:, 1]
        elif self._response == "threshold":
            try:
                y = estimator.decision_function(X)
            except (AttributeError, NotImplementedError):
                y = estimator.predict_proba(X)
                if y.ndim == 2 and y.shape[1] == 2:
                    y = y[:, 1]
        else:
            y = estimator.predict(X)
        kw = dict(self._kwargs)
        if sample_weight is not None:
            kw["sample_weight"] = sample_weight
        return self._sign * self._score_func(y_true, y, **kw)

    def __repr__(self):
        return "make_scorer(%s)" % self._score_func.__name__


def make_scorer(score_func, *, greater_is_better=True, needs_proba=False, needs_threshold=False,
                **kwargs):
    resp = "proba" if needs_proba else ("threshold" if needs_threshold else "predict")
    return _Scorer(score_func, 1 if greater_is_better else -1, kwargs, resp)


def _scorers():
    from .metrics import accuracy_score, adjusted_rand_score, r2_score
    from .cluster_metrics import (adjusted_mutual_info_score, normalized_mutual_info_score,
                                  v_measure_score)
    return {
        "accuracy": make_scorer(accuracy_score),
        "balanced_accuracy": make_scorer(balanced_accuracy_score),
        "r2": make_scorer(r2_score),
        "explained_variance": make_scorer(explained_variance_score),
        "max_error": make_scorer(max_error, greater_is_better=False),
        "neg_mean_absolute_error": make_scorer(mean_absolute_error, greater_is_better=False),
        "neg_mean_squared_error": make_scorer(mean_squared_error_ext, greater_is_better=False),
        "neg_root_mean_squared_error": make_scorer(mean_squared_error_ext,
                                                   greater_is_better=False, squared=False),
        "neg_mean_squared_log_error": make_scorer(mean_squared_log_error,
                                                  greater_is_better=False),
        "neg_median_absolute_error": make_scorer(median_absolute_error, greater_is_better=False),
        "neg_mean_absolute_percentage_error": make_scorer(mean_absolute_percentage_error,
                                                          greater_is_better=False),
        "neg_mean_poisson_deviance": make_scorer(mean_poisson_deviance, greater_is_better=False),
        "neg_mean_gamma_deviance": make_scorer(mean_gamma_deviance, greater_is_better=False),
        "f1": make_scorer(f1_score), "f1_macro": make_scorer(f1_score, average="macro"),
        "f1_micro": make_scorer(f1_score, average="micro"),
        "f1_weighted": make_scorer(f1_score, average="weighted"),
        "precision": make_scorer(precision_score),
        "precision_macro": make_scorer(precision_score, average="macro"),
        "recall": make_scorer(recall_score),
        "recall_macro": make_scorer(recall_score, average="macro"),
        "jaccard": make_scorer(jaccard_score),
        "roc_auc": make_scorer(roc_auc_score, needs_threshold=True),
        "roc_auc_ovr": make_scorer(roc_auc_score, needs_proba=True, multi_class="ovr"),
        "roc_auc_ovo": make_scorer(roc_auc_score, needs_proba=True, multi_class="ovo"),
        "average_precision": make_scorer(average_precision_score, needs_threshold=True),
        "neg_log_loss": make_scorer(log_loss, greater_is_better=False, needs_proba=True),
        "neg_brier_score": make_scorer(brier_score_loss, greater_is_better=False,
                                       needs_proba=True),
        "adjusted_rand_score": make_scorer(adjusted_rand_score),
        "adjusted_mutual_info_score": make_scorer(adjusted_mutual_info_score),
        "normalized_mutual_info_score": make_scorer(normalized_mutual_info_score),
        "v_measure_score": make_scorer(v_measure_score),
    }


SCORERS = None


def get_scorer_ext(scoring):
    global SCORERS
    if callable(scoring):
        return scoring
    if SCORERS is None:
        SCORERS = _scorers()
    if scoring not in SCORERS:
        raise ValueError("%r is not a valid scoring value. Use sorted(SCORERS.keys()) to get "
                         "valid options." % scoring)
    return SCORERS[scoring]


def check_scoring(estimator, scoring=None, *, allow_none=False):
    if scoring is None:
        if hasattr(estimator, "score"):
            return lambda est, X, y=None, **kw: est.score(X, y) if y is not None else est.score(X)
        if allow_none:
            return None
        raise TypeError("If no scoring is specified, the estimator passed should have a 'score' "
                        "method. The estimator %r does not." % estimator)
    return get_scorer_ext(scoring)
