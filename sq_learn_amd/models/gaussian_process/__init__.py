"""Gaussian processes (reference ``sklearn.gaussian_process``)."""
from . import kernels
from ._gp import GaussianProcessClassifier, GaussianProcessRegressor

__all__ = ["GaussianProcessRegressor", "GaussianProcessClassifier", "kernels"]
