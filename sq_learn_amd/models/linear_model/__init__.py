"""Linear models (reference ``sklearn.linear_model``)."""
from ._base import LinearRegression
from ._bayes import ARDRegression, BayesianRidge
from ._coordinate_descent import (ElasticNet, ElasticNetCV, Lasso, LassoCV, enet_path,
                                  lasso_path)
from ._logistic import LogisticRegression
from ._stochastic_gradient import (PassiveAggressiveClassifier, PassiveAggressiveRegressor,
                                   Perceptron, SGDClassifier, SGDOneClassSVM, SGDRegressor)
from ._lm_extra import *  # noqa: F401,F403
from ._lm_extra import __all__ as _extra_all
from ._ridge import Ridge, RidgeClassifier, RidgeClassifierCV, RidgeCV, ridge_regression
from ._sgd_losses import Hinge, Huber, Log, ModifiedHuber, SquaredLoss

__all__ = ["LinearRegression", "ElasticNet", "ElasticNetCV", "Lasso", "LassoCV", "enet_path",
           "lasso_path", "Ridge", "RidgeClassifier", "RidgeClassifierCV", "RidgeCV",
           "ridge_regression", "LogisticRegression", "ARDRegression", "BayesianRidge", "SGDClassifier", "SGDRegressor",
           "SGDOneClassSVM", "Perceptron", "PassiveAggressiveClassifier",
           "PassiveAggressiveRegressor", "Hinge", "Huber", "Log", "ModifiedHuber", "SquaredLoss"]
__all__ = __all__ + list(_extra_all)
