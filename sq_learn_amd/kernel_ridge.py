"""Reference-layout import path (``sklearn.kernel_ridge``)."""
from .kernel_approximation import KernelRidge  # noqa: F401
