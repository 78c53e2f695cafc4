"""Neural networks (reference ``sklearn.neural_network``)."""
from ._mlp import BernoulliRBM, MLPClassifier, MLPRegressor

__all__ = ["BernoulliRBM", "MLPClassifier", "MLPRegressor"]
