"""Class / sample weighting helpers (reference ``utils/class_weight.py``)."""

import numpy as np


def compute_class_weight(class_weight, *, classes, y):
    """Per-class weights: ``None`` (ones), ``'balanced'``
    (n_samples / (n_classes * bincount)) or a {class: weight} dict."""
    classes = np.asarray(classes)
    y = np.asarray(y)
    if set(np.unique(y)) - set(classes):
        raise ValueError("classes should include all valid labels that can be in y")
    if class_weight is None or len(class_weight) == 0:
        return np.ones(classes.shape[0], dtype=np.float64, order="C")
    if isinstance(class_weight, str):
        if class_weight != "balanced":
            raise ValueError("class_weight must be dict, 'balanced', or None, got: %r"
                             % class_weight)
        idx = np.searchsorted(classes, y)
        if not np.all(classes[idx] == y):
            raise ValueError("classes should have valid labels that are in y")
        counts = np.bincount(idx, minlength=len(classes)).astype(np.float64)
        return len(y) / (len(classes) * counts)
    if not isinstance(class_weight, dict):
        raise ValueError("class_weight must be dict, 'balanced', or None, got: %r" % class_weight)
    weight = np.ones(classes.shape[0], dtype=np.float64, order="C")
    for c, w in class_weight.items():
        i = np.searchsorted(classes, c)
        if i < len(classes) and classes[i] == c:
            weight[i] = w
    return weight


def compute_sample_weight(class_weight, y, *, indices=None):
    """Per-sample weights from a class weighting (multi-output: product over
    outputs; ``indices`` restricts the 'balanced' counts to a subsample)."""
    y = np.atleast_1d(np.asarray(y))
    if y.ndim == 1:
        y = y.reshape(-1, 1)
    n_outputs = y.shape[1]
    if isinstance(class_weight, str):
        if class_weight != "balanced":
            raise ValueError('The only valid preset for class_weight is "balanced". Given "%s".'
                             % class_weight)
    elif indices is not None:
        raise ValueError('The only valid class_weight for subsampling is "balanced". Given "%s".'
                         % class_weight)
    elif n_outputs > 1:
        if not hasattr(class_weight, "__iter__") or isinstance(class_weight, dict):
            raise ValueError("For multi-output, class_weight should be a list of dicts, or a "
                             "valid string.")
        if len(class_weight) != n_outputs:
            raise ValueError("For multi-output, number of elements in class_weight should match "
                             "number of outputs.")
    expanded = []
    for k in range(n_outputs):
        y_full = y[:, k]
        classes_full = np.unique(y_full)
        classes_missing = None
        cw = class_weight if (class_weight == "balanced" or n_outputs == 1) else class_weight[k]
        if indices is not None:
            y_sub = y[indices, k]
            classes_sub = np.unique(y_sub)
            weight_k = np.take(compute_class_weight(cw, classes=classes_sub, y=y_sub),
                               np.searchsorted(classes_sub, classes_full), mode="clip")
            classes_missing = set(classes_full) - set(classes_sub)
        else:
            weight_k = compute_class_weight(cw, classes=classes_full, y=y_full)
        weight_k = weight_k[np.searchsorted(classes_full, y_full)]
        if classes_missing:
            weight_k[np.isin(y_full, list(classes_missing))] = 0.0
        expanded.append(weight_k)
    return np.prod(expanded, axis=0, dtype=np.float64)
