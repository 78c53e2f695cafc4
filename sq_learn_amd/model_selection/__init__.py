"""Model selection: CV splitters, cross-validation, hyper-parameter search
and learning curves (reference ``sklearn/model_selection``)."""
from ._search import (GridSearchCV, HalvingGridSearchCV, HalvingRandomSearchCV, ParameterGrid,
                      ParameterSampler, RandomizedSearchCV, fit_grid_point, learning_curve,
                      permutation_test_score, validation_curve)
from ._split import (BaseCrossValidator, KFold, ShuffleSplit, StratifiedKFold, StratifiedShuffleSplit, check_cv,
                     train_test_split)
from ._split_extra import (GroupKFold, GroupShuffleSplit, LeaveOneGroupOut, LeaveOneOut,
                           LeavePGroupsOut, LeavePOut, PredefinedSplit, RepeatedKFold,
                           RepeatedStratifiedKFold, StratifiedGroupKFold, TimeSeriesSplit)
from ._validation import cross_val_predict, cross_val_score, cross_validate, get_scorer

__all__ = ["BaseCrossValidator", "fit_grid_point", "KFold", "StratifiedKFold", "ShuffleSplit", "StratifiedShuffleSplit", "check_cv",
           "train_test_split", "cross_validate", "cross_val_score", "cross_val_predict",
           "GridSearchCV", "RandomizedSearchCV", "HalvingGridSearchCV", "HalvingRandomSearchCV",
           "ParameterGrid", "ParameterSampler", "get_scorer", "learning_curve",
           "validation_curve", "permutation_test_score", "GroupKFold", "GroupShuffleSplit",
           "LeaveOneGroupOut", "LeaveOneOut", "LeavePGroupsOut", "LeavePOut", "PredefinedSplit",
           "RepeatedKFold", "RepeatedStratifiedKFold", "StratifiedGroupKFold", "TimeSeriesSplit"]

from ..utils._aliases import alias_submodules  # noqa: E402
alias_submodules(__name__, "_search_successive_halving", target="sq_learn_amd.model_selection._search")
