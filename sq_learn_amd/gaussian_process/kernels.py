"""Reference-layout import path (``sklearn.gaussian_process.kernels``)."""
from ..models.gaussian_process.kernels import *  # noqa: F401,F403
from ..models.gaussian_process.kernels import KernelOperator  # noqa: E402,F401
