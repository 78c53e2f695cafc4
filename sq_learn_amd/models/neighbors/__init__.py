"""Brute-force k-nearest neighbours (GEMM + top-k kernel)."""
from .knn import KNeighborsClassifier, KNeighborsRegressor, NearestNeighbors

__all__ = ["KNeighborsClassifier", "KNeighborsRegressor", "NearestNeighbors"]
