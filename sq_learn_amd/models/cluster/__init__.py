"""Clustering: q-means (``qMeans_``) and classical k-means."""
from .qmeans import QMeans, qMeans_
from .kmeans import KMeans, k_means, kmeans_plusplus
from ._lloyd import LloydEngine

__all__ = ["QMeans", "qMeans_", "KMeans", "k_means", "kmeans_plusplus", "LloydEngine"]
