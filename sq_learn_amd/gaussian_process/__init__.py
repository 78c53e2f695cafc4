"""Reference-layout import path (``sklearn.gaussian_process``)."""
from ..models.gaussian_process import GaussianProcessClassifier, GaussianProcessRegressor  # noqa
from ..models.gaussian_process import kernels  # noqa: F401

__all__ = ["GaussianProcessRegressor", "GaussianProcessClassifier", "kernels"]

from ..utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
