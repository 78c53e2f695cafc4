"""Nearest neighbours: GPU brute force (GEMM + top-k kernel) for the
euclidean path; host KD/ball trees (C++) and pairwise metrics otherwise."""
from .knn import KNeighborsClassifier, KNeighborsRegressor, NearestNeighbors
from ._extra import (VALID_METRICS, VALID_METRICS_SPARSE, BallTree, DistanceMetric, KDTree, KernelDensity,
                     KNeighborsTransformer, LocalOutlierFactor, NearestCentroid,
                     NeighborhoodComponentsAnalysis, RadiusNeighborsClassifier,
                     RadiusNeighborsRegressor, RadiusNeighborsTransformer, kneighbors_graph,
                     radius_neighbors_graph)

__all__ = ["KNeighborsClassifier", "KNeighborsRegressor", "NearestNeighbors", "KDTree",
           "BallTree", "DistanceMetric", "KernelDensity", "KNeighborsTransformer",
           "LocalOutlierFactor", "NearestCentroid", "NeighborhoodComponentsAnalysis",
           "RadiusNeighborsClassifier", "RadiusNeighborsRegressor", "RadiusNeighborsTransformer",
           "kneighbors_graph", "radius_neighbors_graph", "VALID_METRICS",
           "VALID_METRICS_SPARSE"]
