"""Ensembles (reference ``sklearn.ensemble``)."""
from ._hist_gradient_boosting import (HistGradientBoostingClassifier,
                                      HistGradientBoostingRegressor)
from ._gb import GradientBoostingClassifier, GradientBoostingRegressor
from ._forest import (ExtraTreesClassifier, ExtraTreesRegressor, RandomForestClassifier,
                      RandomForestRegressor, RandomTreesEmbedding)

__all__ = ["RandomForestClassifier", "RandomForestRegressor", "ExtraTreesClassifier",
           "ExtraTreesRegressor", "RandomTreesEmbedding", "GradientBoostingClassifier",
           "GradientBoostingRegressor", "HistGradientBoostingClassifier",
           "HistGradientBoostingRegressor"]
from ._meta import (AdaBoostClassifier, AdaBoostRegressor, BaggingClassifier,  # noqa: E402
                    BaseEnsemble,
                    BaggingRegressor, IsolationForest, StackingClassifier, StackingRegressor,
                    VotingClassifier, VotingRegressor)

__all__ += ["BaggingClassifier", "BaggingRegressor", "IsolationForest", "AdaBoostClassifier",
            "AdaBoostRegressor", "VotingClassifier", "VotingRegressor", "StackingClassifier",
            "StackingRegressor", "BaseEnsemble"]
