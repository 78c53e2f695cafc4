"""Visualisation API of the metrics (reference ``sklearn/metrics/_plot``):
``RocCurveDisplay`` (``roc_curve.py:10``), ``PrecisionRecallDisplay``
(``precision_recall_curve.py:10``), ``DetCurveDisplay`` (``det_curve.py:10``),
``ConfusionMatrixDisplay`` (``confusion_matrix.py:13``) and the deprecated
``plot_*`` helpers.

A display object holds the computed curve (arrays only, so it can be built
from any source and pickled), ``plot`` draws it with matplotlib (imported
lazily: the package does not need it unless something is drawn) and stores
the artists as ``line_`` / ``im_`` / ``text_`` plus ``ax_`` and
``figure_``.  ``from_estimator`` / ``from_predictions`` compute the curve
with this package's metric functions first (the reference adds them for the
confusion matrix; they are provided for every display here)."""

import warnings

import numpy as np

from ..base import is_classifier
from ..utils.metrics import confusion_matrix
from ..utils.metrics_extra import (auc, average_precision_score, det_curve,
                                   precision_recall_curve, roc_curve)


def _to_np(a):
    return a.detach().cpu().numpy() if hasattr(a, "detach") else np.asarray(a)


def _axes(ax):
    import matplotlib.pyplot as plt
    if ax is None:
        _, ax = plt.subplots()
    return ax


def _estimator_name(estimator, name):
    return name if name is not None else estimator.__class__.__name__


def _check_response_method(estimator, response_method):
    """The prediction method of a binary classifier to score with
    (reference ``metrics/_plot/base.py:6``): 'auto' tries predict_proba, then
    decision_function."""
    if response_method not in ("predict_proba", "decision_function", "auto"):
        raise ValueError("response_method must be 'predict_proba', 'decision_function' or "
                         "'auto'")
    order = (["predict_proba", "decision_function"] if response_method == "auto"
             else [response_method])
    for m in order:
        fn = getattr(estimator, m, None)
        if fn is not None:
            return fn
    raise ValueError("response method {} not defined in {}".format(
        " or ".join(order), estimator.__class__.__name__))


def _binary_response(X, estimator, response_method, pos_label=None):
    """(scores of the positive class, pos_label) of a fitted binary
    classifier (reference ``metrics/_plot/base.py:48``)."""
    name = estimator.__class__.__name__
    if not is_classifier(estimator):
        raise ValueError(f"Expected 'estimator' to be a binary classifier, but got {name}")
    classes = getattr(estimator, "classes_", None)
    if classes is None:
        raise ValueError(f"This {name} instance is not fitted yet. Call 'fit' with appropriate "
                         "arguments before using this estimator.")
    classes = _to_np(classes)
    if classes.shape[0] != 2:
        raise ValueError(f"{name} should be a binary classifier, got {classes.shape[0]} classes")
    fn = _check_response_method(estimator, response_method)
    y = _to_np(fn(X))
    if pos_label is not None and pos_label not in classes.tolist():
        raise ValueError(f"The class provided by 'pos_label' is unknown. Got {pos_label} "
                         f"instead of one of {classes.tolist()}")
    if fn.__name__ == "predict_proba":
        if y.ndim != 2 or y.shape[1] != 2:
            raise ValueError(f"{name} should be a binary classifier")
        if pos_label is None:
            pos_label = classes[1]
        y = y[:, int(np.flatnonzero(classes == pos_label)[0])]
    else:
        y = y.reshape(-1)
        if pos_label is None:
            pos_label = classes[1]
        elif pos_label == classes[0]:
            y = -y
    return y, pos_label


def _positive_suffix(pos_label):
    return "" if pos_label is None else f" (Positive label: {pos_label})"


class RocCurveDisplay:
    """ROC curve visualisation: ``fpr`` / ``tpr`` arrays, optional
    ``roc_auc`` (shown in the legend), ``estimator_name``, ``pos_label``."""

    def __init__(self, *, fpr, tpr, roc_auc=None, estimator_name=None, pos_label=None):
        self.fpr = fpr
        self.tpr = tpr
        self.roc_auc = roc_auc
        self.estimator_name = estimator_name
        self.pos_label = pos_label

    def plot(self, ax=None, *, name=None, **kwargs):
        ax = _axes(ax)
        name = self.estimator_name if name is None else name
        kw = {}
        if self.roc_auc is not None and name is not None:
            kw["label"] = f"{name} (AUC = {self.roc_auc:0.2f})"
        elif self.roc_auc is not None:
            kw["label"] = f"AUC = {self.roc_auc:0.2f}"
        elif name is not None:
            kw["label"] = name
        kw.update(kwargs)
        (self.line_,) = ax.plot(self.fpr, self.tpr, **kw)
        suffix = _positive_suffix(self.pos_label)
        ax.set(xlabel="False Positive Rate" + suffix, ylabel="True Positive Rate" + suffix)
        if "label" in kw:
            ax.legend(loc="lower right")
        self.ax_ = ax
        self.figure_ = ax.figure
        return self

    @classmethod
    def from_predictions(cls, y_true, y_pred, *, sample_weight=None, drop_intermediate=True,
                         pos_label=None, name=None, ax=None, **kwargs):
        fpr, tpr, _ = roc_curve(_to_np(y_true), _to_np(y_pred), pos_label=pos_label,
                                sample_weight=sample_weight,
                                drop_intermediate=drop_intermediate)
        if pos_label is None:
            classes = np.unique(_to_np(y_true))
            pos_label = classes[-1] if classes.size == 2 else 1
        disp = cls(fpr=fpr, tpr=tpr, roc_auc=auc(fpr, tpr),
                   estimator_name="Classifier" if name is None else name, pos_label=pos_label)
        return disp.plot(ax=ax, **kwargs)

    @classmethod
    def from_estimator(cls, estimator, X, y, *, sample_weight=None, drop_intermediate=True,
                       response_method="auto", pos_label=None, name=None, ax=None, **kwargs):
        y_score, pos_label = _binary_response(X, estimator, response_method, pos_label)
        return cls.from_predictions(y, y_score, sample_weight=sample_weight,
                                    drop_intermediate=drop_intermediate, pos_label=pos_label,
                                    name=_estimator_name(estimator, name), ax=ax, **kwargs)


class PrecisionRecallDisplay:
    """Precision-recall curve visualisation (step plot); ``average_precision``
    is shown in the legend."""

    def __init__(self, precision, recall, *, average_precision=None, estimator_name=None,
                 pos_label=None):
        self.precision = precision
        self.recall = recall
        self.average_precision = average_precision
        self.estimator_name = estimator_name
        self.pos_label = pos_label

    def plot(self, ax=None, *, name=None, **kwargs):
        ax = _axes(ax)
        name = self.estimator_name if name is None else name
        kw = {"drawstyle": "steps-post"}
        if self.average_precision is not None and name is not None:
            kw["label"] = f"{name} (AP = {self.average_precision:0.2f})"
        elif self.average_precision is not None:
            kw["label"] = f"AP = {self.average_precision:0.2f}"
        elif name is not None:
            kw["label"] = name
        kw.update(kwargs)
        (self.line_,) = ax.plot(self.recall, self.precision, **kw)
        suffix = _positive_suffix(self.pos_label)
        ax.set(xlabel="Recall" + suffix, ylabel="Precision" + suffix)
        if "label" in kw:
            ax.legend(loc="lower left")
        self.ax_ = ax
        self.figure_ = ax.figure
        return self

    @classmethod
    def from_predictions(cls, y_true, y_pred, *, sample_weight=None, pos_label=None, name=None,
                         ax=None, **kwargs):
        y_true, y_pred = _to_np(y_true), _to_np(y_pred)
        if pos_label is None:
            classes = np.unique(y_true)
            pos_label = classes[-1] if classes.size == 2 else 1
        precision, recall, _ = precision_recall_curve(y_true, y_pred, pos_label=pos_label,
                                                      sample_weight=sample_weight)
        ap = average_precision_score(y_true, y_pred, pos_label=pos_label,
                                     sample_weight=sample_weight)
        disp = cls(precision, recall, average_precision=ap,
                   estimator_name="Classifier" if name is None else name, pos_label=pos_label)
        return disp.plot(ax=ax, **kwargs)

    @classmethod
    def from_estimator(cls, estimator, X, y, *, sample_weight=None, pos_label=None,
                       response_method="auto", name=None, ax=None, **kwargs):
        y_score, pos_label = _binary_response(X, estimator, response_method, pos_label)
        return cls.from_predictions(y, y_score, sample_weight=sample_weight, pos_label=pos_label,
                                    name=_estimator_name(estimator, name), ax=ax, **kwargs)


# DET axes: normal-deviate scale, ticks at these error rates
_DET_TICKS = (0.001, 0.01, 0.05, 0.20, 0.5, 0.80, 0.95, 0.99, 0.999)


class DetCurveDisplay:
    """Detection error tradeoff curve on normal-deviate axes (false positive
    vs false negative rate through the probit transform)."""

    def __init__(self, *, fpr, fnr, estimator_name=None, pos_label=None):
        self.fpr = fpr
        self.fnr = fnr
        self.estimator_name = estimator_name
        self.pos_label = pos_label

    def plot(self, ax=None, *, name=None, **kwargs):
        from scipy.stats import norm
        ax = _axes(ax)
        name = self.estimator_name if name is None else name
        kw = {} if name is None else {"label": name}
        kw.update(kwargs)
        (self.line_,) = ax.plot(norm.ppf(self.fpr), norm.ppf(self.fnr), **kw)
        suffix = _positive_suffix(self.pos_label)
        ax.set(xlabel="False Positive Rate" + suffix, ylabel="False Negative Rate" + suffix)
        if "label" in kw:
            ax.legend(loc="lower right")
        loc = norm.ppf(_DET_TICKS)
        labels = [f"{t:.0%}" if round(100 * t, 6).is_integer() else f"{t:.1%}"
                  for t in _DET_TICKS]
        ax.set_xticks(loc)
        ax.set_xticklabels(labels)
        ax.set_xlim(-3, 3)
        ax.set_yticks(loc)
        ax.set_yticklabels(labels)
        ax.set_ylim(-3, 3)
        self.ax_ = ax
        self.figure_ = ax.figure
        return self

    @classmethod
    def from_predictions(cls, y_true, y_pred, *, sample_weight=None, pos_label=None, name=None,
                         ax=None, **kwargs):
        y_true, y_pred = _to_np(y_true), _to_np(y_pred)
        fpr, fnr, _ = det_curve(y_true, y_pred, pos_label=pos_label, sample_weight=sample_weight)
        if pos_label is None:
            classes = np.unique(y_true)
            pos_label = classes[-1] if classes.size == 2 else 1
        disp = cls(fpr=fpr, fnr=fnr, estimator_name="Classifier" if name is None else name,
                   pos_label=pos_label)
        return disp.plot(ax=ax, **kwargs)

    @classmethod
    def from_estimator(cls, estimator, X, y, *, sample_weight=None, response_method="auto",
                       pos_label=None, name=None, ax=None, **kwargs):
        y_score, pos_label = _binary_response(X, estimator, response_method, pos_label)
        return cls.from_predictions(y, y_score, sample_weight=sample_weight, pos_label=pos_label,
                                    name=_estimator_name(estimator, name), ax=ax, **kwargs)


class ConfusionMatrixDisplay:
    """Confusion matrix heat map with the cell values written in; the text
    colour flips at the midpoint of the colour map for contrast."""

    def __init__(self, confusion_matrix, *, display_labels=None):
        self.confusion_matrix = confusion_matrix
        self.display_labels = display_labels

    def plot(self, *, include_values=True, cmap="viridis", xticks_rotation="horizontal",
             values_format=None, ax=None, colorbar=True):
        ax = _axes(ax)
        fig = ax.figure
        cm = np.asarray(self.confusion_matrix)
        n = cm.shape[0]
        self.im_ = ax.imshow(cm, interpolation="nearest", cmap=cmap)
        self.text_ = None
        lo, hi = self.im_.cmap(0), self.im_.cmap(1.0)
        if include_values:
            self.text_ = np.empty_like(cm, dtype=object)
            thresh = (cm.max() + cm.min()) / 2.0
            for i in range(n):
                for j in range(n):
                    v = cm[i, j]
                    if values_format is not None:
                        txt = format(v, values_format)
                    else:   # 2 significant digits; integer counts as 'd' when shorter
                        txt = format(v, ".2g")
                        if cm.dtype.kind != "f" and len(format(v, "d")) < len(txt):
                            txt = format(v, "d")
                    self.text_[i, j] = ax.text(j, i, txt, ha="center", va="center",
                                               color=hi if v < thresh else lo)
        labels = np.arange(n) if self.display_labels is None else self.display_labels
        if colorbar:
            fig.colorbar(self.im_, ax=ax)
        ax.set(xticks=np.arange(n), yticks=np.arange(n), xticklabels=labels,
               yticklabels=labels, ylabel="True label", xlabel="Predicted label")
        ax.set_ylim((n - 0.5, -0.5))
        import matplotlib.pyplot as plt
        plt.setp(ax.get_xticklabels(), rotation=xticks_rotation)
        self.figure_ = fig
        self.ax_ = ax
        return self

    @classmethod
    def from_predictions(cls, y_true, y_pred, *, labels=None, sample_weight=None, normalize=None,
                         display_labels=None, include_values=True, xticks_rotation="horizontal",
                         values_format=None, cmap="viridis", ax=None, colorbar=True):
        y_true, y_pred = _to_np(y_true), _to_np(y_pred)
        cm = confusion_matrix(y_true, y_pred, labels=labels, sample_weight=sample_weight,
                              normalize=normalize)
        if display_labels is None:
            display_labels = (np.unique(np.concatenate([y_true, y_pred])) if labels is None
                              else labels)
        disp = cls(confusion_matrix=cm, display_labels=display_labels)
        return disp.plot(include_values=include_values, cmap=cmap, ax=ax,
                         xticks_rotation=xticks_rotation, values_format=values_format,
                         colorbar=colorbar)

    @classmethod
    def from_estimator(cls, estimator, X, y, *, labels=None, sample_weight=None, normalize=None,
                       display_labels=None, include_values=True, xticks_rotation="horizontal",
                       values_format=None, cmap="viridis", ax=None, colorbar=True):
        if not is_classifier(estimator):
            raise ValueError(f"{estimator.__class__.__name__} should be a classifier")
        return cls.from_predictions(y, _to_np(estimator.predict(X)), labels=labels,
                                    sample_weight=sample_weight, normalize=normalize,
                                    display_labels=display_labels,
                                    include_values=include_values,
                                    xticks_rotation=xticks_rotation,
                                    values_format=values_format, cmap=cmap, ax=ax,
                                    colorbar=colorbar)


def _deprecated(old, new):
    warnings.warn(f"Function {old} is deprecated; it will be removed in 1.2. Use {new} "
                  "instead.", FutureWarning, stacklevel=3)


def plot_roc_curve(estimator, X, y, *, sample_weight=None, drop_intermediate=True,
                   response_method="auto", name=None, ax=None, pos_label=None, **kwargs):
    """Deprecated form of ``RocCurveDisplay.from_estimator``."""
    _deprecated("plot_roc_curve", "RocCurveDisplay.from_estimator")
    return RocCurveDisplay.from_estimator(estimator, X, y, sample_weight=sample_weight,
                                          drop_intermediate=drop_intermediate,
                                          response_method=response_method, pos_label=pos_label,
                                          name=name, ax=ax, **kwargs)


def plot_precision_recall_curve(estimator, X, y, *, sample_weight=None, response_method="auto",
                                name=None, ax=None, pos_label=None, **kwargs):
    """Deprecated form of ``PrecisionRecallDisplay.from_estimator``."""
    _deprecated("plot_precision_recall_curve", "PrecisionRecallDisplay.from_estimator")
    return PrecisionRecallDisplay.from_estimator(estimator, X, y, sample_weight=sample_weight,
                                                 response_method=response_method,
                                                 pos_label=pos_label, name=name, ax=ax, **kwargs)


def plot_det_curve(estimator, X, y, *, sample_weight=None, response_method="auto", name=None,
                   ax=None, pos_label=None, **kwargs):
    """Deprecated form of ``DetCurveDisplay.from_estimator``."""
    _deprecated("plot_det_curve", "DetCurveDisplay.from_estimator")
    return DetCurveDisplay.from_estimator(estimator, X, y, sample_weight=sample_weight,
                                          response_method=response_method, pos_label=pos_label,
                                          name=name, ax=ax, **kwargs)


def plot_confusion_matrix(estimator, X, y_true, *, labels=None, sample_weight=None,
                          normalize=None, display_labels=None, include_values=True,
                          xticks_rotation="horizontal", values_format=None, cmap="viridis",
                          ax=None, colorbar=True):
    """Deprecated form of ``ConfusionMatrixDisplay.from_estimator``."""
    _deprecated("plot_confusion_matrix", "ConfusionMatrixDisplay.from_estimator")
    return ConfusionMatrixDisplay.from_estimator(
        estimator, X, y_true, labels=labels, sample_weight=sample_weight, normalize=normalize,
        display_labels=display_labels, include_values=include_values,
        xticks_rotation=xticks_rotation, values_format=values_format, cmap=cmap, ax=ax,
        colorbar=colorbar)


__all__ = ["RocCurveDisplay", "PrecisionRecallDisplay", "DetCurveDisplay",
           "ConfusionMatrixDisplay", "plot_roc_curve", "plot_precision_recall_curve",
           "plot_det_curve", "plot_confusion_matrix"]
