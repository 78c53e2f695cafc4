"""Model selection: CV splitters, cross-validation and grid search
(reference ``sklearn/model_selection``)."""
from ._split import (KFold, ShuffleSplit, StratifiedKFold, StratifiedShuffleSplit, check_cv,
                     train_test_split)
from ._validation import (GridSearchCV, ParameterGrid, cross_val_predict, cross_val_score,
                          cross_validate, get_scorer)

__all__ = ["KFold", "StratifiedKFold", "ShuffleSplit", "StratifiedShuffleSplit", "check_cv",
           "train_test_split", "cross_validate", "cross_val_score", "cross_val_predict",
           "GridSearchCV", "ParameterGrid", "get_scorer"]
