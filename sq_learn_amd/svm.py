"""Reference-layout import path (``sklearn.svm``): libsvm / liblinear SVMs, LS-SVM and
quantum LS-SVM."""
from .models.svm import *  # noqa: F401,F403
from .models.svm import __all__  # noqa: F401


def l1_min_c(X, y, *, loss="squared_hinge", fit_intercept=True, intercept_scaling=1.0):
    """Lowest C for which an l1-penalised linear model is not empty
    (reference ``svm/_bounds.py``)."""
    import numpy as np

    from .preprocessing import LabelBinarizer
    if loss not in ("squared_hinge", "log"):
        raise ValueError('loss type not in ("squared_hinge", "log")')
    X = X.tocsc() if hasattr(X, "tocsc") else np.asarray(X, dtype=np.float64)
    Y = np.asarray(LabelBinarizer(neg_label=-1).fit_transform(y)).T
    den = np.max(np.abs(np.asarray(Y @ X if not hasattr(X, "tocsc") else (X.T @ Y.T).T)))
    if fit_intercept:
        bias = np.full((np.size(y), 1), intercept_scaling,
                       dtype=np.array(intercept_scaling).dtype)
        den = max(den, abs(np.dot(Y, bias)).max())
    if den == 0.0:
        raise ValueError("Ill-posed l1_min_c calculation: l1 will always select zero "
                         "coefficients for this data")
    return 0.5 / den if loss == "squared_hinge" else 2.0 / den

from .utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
