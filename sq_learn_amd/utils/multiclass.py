"""Target-type introspection for classifiers (reference
``utils/multiclass.py``: ``unique_labels`` :43, ``is_multilabel`` :113,
``check_classification_targets`` :174, ``type_of_target`` :186,
``class_distribution`` :355, ``_ovr_decision_function`` :413).

Host-side NumPy: these inspect label arrays once per fit; device tensors are
moved to the host first.
"""

from itertools import chain

import numpy as np
import scipy.sparse as sp

from ..runtime.device import to_numpy

__all__ = ["type_of_target", "unique_labels", "is_multilabel", "check_classification_targets",
           "class_distribution"]


def _as_array(y):
    if hasattr(y, "detach"):
        return to_numpy(y)
    return y


def _is_integral_float(y):
    return y.dtype.kind == "f" and np.all(y.astype(int) == y)


def is_multilabel(y):
    """True for a 2-d label-indicator matrix (dense or sparse) whose entries
    take at most two values, zero being one of them when there are two."""
    y = _as_array(y)
    if hasattr(y, "__array__") or isinstance(y, (list, tuple)) or sp.issparse(y):
        if not sp.issparse(y):
            try:
                y = np.asarray(y)
            except ValueError:
                return False
    else:
        return False
    if not (hasattr(y, "shape") and y.ndim == 2 and y.shape[1] > 1):
        return False
    if sp.issparse(y):
        y = y.tocsr()
        vals = np.unique(y.data)
        return (len(y.data) == 0 or
                (vals.size == 1 and (y.dtype.kind in "biu" or _is_integral_float(vals))))
    labels = np.unique(y)
    return len(labels) < 3 and (y.dtype.kind in "biu" or _is_integral_float(labels))


def type_of_target(y):
    """The most specific of: 'continuous', 'continuous-multioutput',
    'binary', 'multiclass', 'multiclass-multioutput', 'multilabel-indicator',
    'unknown'."""
    y = _as_array(y)
    valid = ((isinstance(y, (list, tuple)) or hasattr(y, "__array__") or sp.issparse(y))
             and not isinstance(y, str))
    if not valid:
        raise ValueError("Expected array-like (array or non-string sequence), got %r" % (y,))
    if y.__class__.__name__ == "SparseSeries":
        raise ValueError("y cannot be class 'SparseSeries'.")
    if is_multilabel(y):
        return "multilabel-indicator"
    try:
        arr = np.asarray(y)
    except ValueError:
        return "unknown"    # ragged sequences
    # sequence-of-sequences targets are not supported
    try:
        if (not hasattr(arr[0], "__array__") and isinstance(arr[0], (list, tuple))
                and not isinstance(arr[0], str)):
            raise ValueError("You appear to be using a legacy multi-label data representation. "
                             "Sequence of sequences are no longer supported; use a binary "
                             "array or sparse matrix instead - the MultiLabelBinarizer "
                             "transformer can convert to this format.")
    except IndexError:
        pass
    if arr.ndim > 2 or (arr.dtype == object and len(arr) and not isinstance(arr.flat[0], str)):
        return "unknown"
    if arr.ndim == 2 and arr.shape[1] == 0:
        return "unknown"
    suffix = "-multioutput" if arr.ndim == 2 and arr.shape[1] > 1 else ""
    if arr.dtype.kind == "f" and np.any(arr != arr.astype(int)):
        if not np.all(np.isfinite(arr)):
            raise ValueError("Input contains NaN, infinity or a value too large for %r."
                             % arr.dtype)
        return "continuous" + suffix
    if len(np.unique(arr)) > 2 or (arr.ndim >= 2 and len(arr[0]) > 1):
        return "multiclass" + suffix
    return "binary"


def _unique_multiclass(y):
    if hasattr(y, "__array__"):
        return np.unique(np.asarray(y))
    return set(y)


def _unique_indicator(y):
    return np.arange(y.shape[1])


_UNIQUE = {"binary": _unique_multiclass, "multiclass": _unique_multiclass,
           "multilabel-indicator": _unique_indicator}


def unique_labels(*ys):
    """Sorted unique labels of one or more targets of a common kind
    (binary / multiclass mix, or multilabel indicators of one width);
    string and number labels cannot be mixed."""
    ys = [_as_array(y) for y in ys]
    if not ys:
        raise ValueError("No argument has been passed.")
    kinds = {type_of_target(y) for y in ys}
    if kinds == {"binary", "multiclass"}:
        kinds = {"multiclass"}
    if len(kinds) > 1:
        raise ValueError("Mix type of y not allowed, got types %s" % kinds)
    kind = kinds.pop()
    if kind == "multilabel-indicator":
        widths = {(y.shape[1] if sp.issparse(y) else np.asarray(y).shape[1]) for y in ys}
        if len(widths) > 1:
            raise ValueError("Multi-label binary indicator input with different numbers of "
                             "labels")
    fn = _UNIQUE.get(kind)
    if fn is None:
        raise ValueError("Unknown label type: %s" % repr(ys))
    labels = set(chain.from_iterable(fn(y) for y in ys))
    if len({isinstance(v, str) for v in labels}) > 1:
        raise ValueError("Mix of label input types (string and number)")
    return np.array(sorted(labels))


def check_classification_targets(y):
    """Raise unless y is a classification target (binary, multiclass,
    multiclass-multioutput, multilabel-indicator or multilabel-sequences)."""
    t = type_of_target(y)
    if t not in ("binary", "multiclass", "multiclass-multioutput", "multilabel-indicator",
                 "multilabel-sequences"):
        raise ValueError("Unknown label type: %r" % t)


def class_distribution(y, sample_weight=None):
    """Per output column: (classes, n_classes, class prior) lists; sparse
    columns count their implicit zeros."""
    y = _as_array(y)
    classes, n_classes, priors = [], [], []
    n = y.shape[0]
    sw = None if sample_weight is None else np.asarray(sample_weight, dtype=np.float64)
    if sp.issparse(y):
        y = y.tocsc()
        for k in range(y.shape[1]):
            lo, hi = y.indptr[k], y.indptr[k + 1]
            rows = y.indices[lo:hi]
            w_nz = sw[rows] if sw is not None else np.ones(hi - lo)
            cls, inv = np.unique(y.data[lo:hi], return_inverse=True)
            prior = np.bincount(inv, weights=w_nz)
            n_zero = n - (hi - lo)
            if n_zero > 0:
                zero_w = (sw.sum() - w_nz.sum()) if sw is not None else float(n_zero)
                if 0 not in cls:
                    cls = np.insert(cls, 0, 0)
                    prior = np.insert(prior, 0, zero_w)
                else:
                    prior[np.searchsorted(cls, 0)] += zero_w
            classes.append(cls)
            n_classes.append(cls.shape[0])
            priors.append(prior / prior.sum())
    else:
        y = np.asarray(y)
        y2 = y.reshape(-1, 1) if y.ndim == 1 else y
        for k in range(y2.shape[1]):
            cls, inv = np.unique(y2[:, k], return_inverse=True)
            prior = np.bincount(inv.ravel(), weights=sw)
            classes.append(cls)
            n_classes.append(cls.shape[0])
            priors.append(prior / prior.sum())
    return classes, n_classes, priors


def _check_partial_fit_first_call(clf, classes=None):
    """True on the first partial_fit call (sets ``classes_``); later calls
    must repeat the same classes or none."""
    if getattr(clf, "classes_", None) is None and classes is None:
        raise ValueError("classes must be passed on the first call to partial_fit.")
    if classes is not None:
        if getattr(clf, "classes_", None) is not None:
            if not np.array_equal(clf.classes_, unique_labels(classes)):
                raise ValueError("`classes=%r` is not the same as on last call to partial_fit, "
                                 "was: %r" % (classes, clf.classes_))
        else:
            clf.classes_ = unique_labels(classes)
            return True
    return False


def _ovr_decision_function(predictions, confidences, n_classes):
    """One-vs-one votes plus confidences squashed into (-1/3, 1/3): ties
    between vote counts are broken by the summed confidences."""
    n = predictions.shape[0]
    votes = np.zeros((n, n_classes))
    conf = np.zeros((n, n_classes))
    k = 0
    for i in range(n_classes):
        for j in range(i + 1, n_classes):
            conf[:, i] -= confidences[:, k]
            conf[:, j] += confidences[:, k]
            votes[predictions[:, k] == 0, i] += 1
            votes[predictions[:, k] == 1, j] += 1
            k += 1
    scaled = conf / (3 * (np.abs(conf) + 1))
    return votes + scaled
