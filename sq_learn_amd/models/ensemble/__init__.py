"""Ensembles (reference ``sklearn.ensemble``)."""
from ._forest import (ExtraTreesClassifier, ExtraTreesRegressor, RandomForestClassifier,
                      RandomForestRegressor, RandomTreesEmbedding)

__all__ = ["RandomForestClassifier", "RandomForestRegressor", "ExtraTreesClassifier",
           "ExtraTreesRegressor", "RandomTreesEmbedding"]
