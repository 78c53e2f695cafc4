"""Decision-tree estimators (reference ``tree/_classes.py``:
``BaseDecisionTree.fit`` :145-412, ``predict`` :428, ``apply`` :480,
``decision_path`` :508, ``_prune_tree`` :533, ``cost_complexity_pruning_path``
:556, ``feature_importances_`` :596, ``DecisionTreeClassifier`` :622,
``DecisionTreeRegressor``, ``ExtraTreeClassifier``, ``ExtraTreeRegressor``).

Parameter resolution, class encoding, class weights and the splitter seed
(``random_state.randint(0, 2**31 - 1)``, the reference's ``Splitter.init``)
follow the reference so that a fitted tree is the reference's tree; growth
itself is the host-native builder (``csrc/host/tree.cpp``).
"""

from abc import ABCMeta, abstractmethod
import numbers
import warnings
from math import ceil

import numpy as np
import scipy.sparse as sp
import torch

from ...base import BaseEstimator, ClassifierMixin, RegressorMixin, clone, is_classifier
from ...utils.class_weight import compute_sample_weight
from ...utils.validation import check_is_fitted, check_random_state
from . import _tree
from ._tree import RAND_R_MAX, Tree

CRITERIA_CLF = ("gini", "entropy", "log_loss")
CRITERIA_REG = ("squared_error", "mse", "friedman_mse", "absolute_error", "mae", "poisson")


class Bunch(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:  # pragma: no cover
            raise AttributeError(k) from e


def _as_f32(X):
    if isinstance(X, torch.Tensor):
        X = X.detach().cpu().numpy()
    if sp.issparse(X):
        X = X.toarray()
    X = np.asarray(X)
    if X.ndim != 2:
        raise ValueError("Expected 2D array, got %dD array instead" % X.ndim)
    X = np.ascontiguousarray(X, dtype=np.float32)
    if not np.isfinite(X).all():
        raise ValueError("Input contains NaN, infinity or a value too large for dtype('float32').")
    return X


def resolve_max_features(max_features, n_features, is_clf):
    if isinstance(max_features, str):
        if max_features == "auto":
            return max(1, int(np.sqrt(n_features))) if is_clf else n_features
        if max_features == "sqrt":
            return max(1, int(np.sqrt(n_features)))
        if max_features == "log2":
            return max(1, int(np.log2(n_features)))
        raise ValueError("Invalid value for max_features. Allowed string values are 'auto', "
                         "'sqrt' or 'log2'.")
    if max_features is None:
        return n_features
    if isinstance(max_features, numbers.Integral):
        return int(max_features)
    return max(1, int(max_features * n_features)) if max_features > 0.0 else 0


class BaseDecisionTree(BaseEstimator, metaclass=ABCMeta):
    """Shared fit / predict machinery of the tree estimators (abstract, as
    the reference's ``tree/_classes.py:BaseDecisionTree``: the concrete
    classes define the constructor)."""

    @abstractmethod
    def __init__(self):
        pass

    def get_depth(self):
        check_is_fitted(self)
        return self.tree_.max_depth

    def get_n_leaves(self):
        check_is_fitted(self)
        return self.tree_.n_leaves

    # --------------------------------------------------------------- params
    def _resolve_params(self, n_samples, n_features, sample_weight):
        max_depth = np.iinfo(np.int32).max if self.max_depth is None else self.max_depth
        max_leaf_nodes = -1 if self.max_leaf_nodes is None else self.max_leaf_nodes
        if isinstance(self.min_samples_leaf, numbers.Integral):
            if not 1 <= self.min_samples_leaf:
                raise ValueError("min_samples_leaf must be at least 1 or in (0, 0.5], got %s"
                                 % self.min_samples_leaf)
            msl = self.min_samples_leaf
        else:
            if not 0.0 < self.min_samples_leaf <= 0.5:
                raise ValueError("min_samples_leaf must be at least 1 or in (0, 0.5], got %s"
                                 % self.min_samples_leaf)
            msl = int(ceil(self.min_samples_leaf * n_samples))
        if isinstance(self.min_samples_split, numbers.Integral):
            if not 2 <= self.min_samples_split:
                raise ValueError("min_samples_split must be an integer greater than 1 or a float "
                                 "in (0.0, 1.0]; got the integer %s" % self.min_samples_split)
            mss = self.min_samples_split
        else:
            if not 0.0 < self.min_samples_split <= 1.0:
                raise ValueError("min_samples_split must be an integer greater than 1 or a float "
                                 "in (0.0, 1.0]; got the float %s" % self.min_samples_split)
            mss = max(2, int(ceil(self.min_samples_split * n_samples)))
        mss = max(mss, 2 * msl)
        max_features = resolve_max_features(self.max_features, n_features, is_classifier(self))
        if not 0 <= self.min_weight_fraction_leaf <= 0.5:
            raise ValueError("min_weight_fraction_leaf must in [0, 0.5]")
        if max_depth <= 0:
            raise ValueError("max_depth must be greater than zero. ")
        if not 0 < max_features <= n_features:
            raise ValueError("max_features must be in (0, n_features]")
        if not isinstance(max_leaf_nodes, numbers.Integral):
            raise ValueError("max_leaf_nodes must be integral number but was %r" % max_leaf_nodes)
        if -1 < max_leaf_nodes < 2:
            raise ValueError(("max_leaf_nodes {0} must be either None or larger than 1")
                             .format(max_leaf_nodes))
        if self.min_impurity_decrease < 0.0:
            raise ValueError("min_impurity_decrease must be greater than or equal to 0")
        total_w = n_samples if sample_weight is None else float(np.sum(sample_weight))
        crit = self.criterion
        if crit in ("mse", "mae"):
            warnings.warn("Criterion '%s' was deprecated in v1.0; use '%s'." %
                          (crit, "squared_error" if crit == "mse" else "absolute_error"),
                          FutureWarning)
        valid = CRITERIA_CLF if is_classifier(self) else CRITERIA_REG
        if crit not in valid:
            raise ValueError("Unknown criterion %r" % crit)
        if self.splitter not in ("best", "random"):
            raise ValueError("Unknown splitter %r" % self.splitter)
        self.max_features_ = max_features
        return dict(criterion=crit, splitter=self.splitter, max_depth=max_depth,
                    min_samples_split=mss, min_samples_leaf=msl, max_features=max_features,
                    max_leaf_nodes=max_leaf_nodes,
                    min_weight_leaf=self.min_weight_fraction_leaf * total_w,
                    min_impurity_decrease=self.min_impurity_decrease)

    def _encode_y(self, y):
        y = np.atleast_1d(np.asarray(y))
        if y.ndim == 1:
            y = y.reshape(-1, 1)
        self.n_outputs_ = y.shape[1]
        expanded_class_weight = None
        if is_classifier(self):
            y_original = y.copy()
            self.classes_, self.n_classes_ = [], []
            enc = np.zeros(y.shape, dtype=np.intp)
            for k in range(self.n_outputs_):
                cls, enc[:, k] = np.unique(y[:, k], return_inverse=True)
                self.classes_.append(cls)
                self.n_classes_.append(cls.shape[0])
            y = enc
            if getattr(self, "class_weight", None) is not None:   # classifiers only
                expanded_class_weight = compute_sample_weight(self.class_weight, y_original)
            self.n_classes_ = np.array(self.n_classes_, dtype=np.intp)
        return np.ascontiguousarray(y, dtype=np.float64), expanded_class_weight

    def fit(self, X, y, sample_weight=None, check_input=True):
        random_state = check_random_state(self.random_state)
        if self.ccp_alpha < 0.0:
            raise ValueError("ccp_alpha must be greater than or equal to 0")
        X = _as_f32(X)
        n_samples, n_features = X.shape
        self.n_features_in_ = n_features
        y = np.asarray(y.detach().cpu().numpy() if isinstance(y, torch.Tensor) else y)
        if len(y) != n_samples:
            raise ValueError("Number of labels=%d does not match number of samples=%d"
                             % (len(y), n_samples))
        if self.criterion == "poisson":
            if np.any(y < 0):
                raise ValueError("Some value(s) of y are negative which is not allowed for "
                                 "Poisson regression.")
            if np.sum(y) <= 0:
                raise ValueError("Sum of y is not positive which is necessary for Poisson "
                                 "regression.")
        y, expanded_cw = self._encode_y(y)
        if sample_weight is not None:
            sample_weight = np.asarray(sample_weight, dtype=np.float64).reshape(-1)
            if sample_weight.shape[0] != n_samples:
                raise ValueError("sample_weight.shape == {}, expected {}!".format(
                    sample_weight.shape, (n_samples,)))
        if expanded_cw is not None:
            sample_weight = expanded_cw if sample_weight is None else sample_weight * expanded_cw
        params = self._resolve_params(n_samples, n_features, sample_weight)
        seed = random_state.randint(0, RAND_R_MAX)
        n_classes = self.n_classes_ if is_classifier(self) else np.ones(self.n_outputs_, np.intp)
        self.tree_ = _tree.build_trees(X, y, None if sample_weight is None else sample_weight[None],
                                       n_classes, params, [seed], n_threads=1)[0]
        if self.n_outputs_ == 1 and is_classifier(self):
            self.n_classes_ = self.n_classes_[0]
            self.classes_ = self.classes_[0]
        self._prune_tree()
        return self

    def _prune_tree(self):
        if self.ccp_alpha < 0.0:
            raise ValueError("ccp_alpha must be greater than or equal to 0")
        if self.ccp_alpha == 0.0:
            return
        self.tree_ = _tree.build_pruned_tree_ccp(self.tree_, self.ccp_alpha)

    def cost_complexity_pruning_path(self, X, y, sample_weight=None):
        est = clone(self).set_params(ccp_alpha=0.0)
        est.fit(X, y, sample_weight=sample_weight)
        return Bunch(**_tree.ccp_pruning_path(est.tree_))

    @property
    def feature_importances_(self):
        check_is_fitted(self)
        return self.tree_.compute_feature_importances()

    # ----------------------------------------------------------- prediction
    def _validate_X_predict(self, X, check_input=True):
        check_is_fitted(self)
        if isinstance(X, torch.Tensor) and X.is_cuda:
            Xp = X.float().contiguous()
        else:
            Xp = _as_f32(X)
        if Xp.shape[1] != self.n_features_in_:
            raise ValueError(f"X has {Xp.shape[1]} features, but {self.__class__.__name__} is "
                             f"expecting {self.n_features_in_} features as input.")
        return Xp

    def apply(self, X, check_input=True):
        return self.tree_.apply(self._validate_X_predict(X, check_input))

    def decision_path(self, X, check_input=True):
        return self.tree_.decision_path(self._validate_X_predict(X, check_input))

    def predict(self, X, check_input=True):
        proba = self.tree_.predict(self._validate_X_predict(X, check_input))
        n = proba.shape[0]
        if is_classifier(self):
            if self.n_outputs_ == 1:
                return self.classes_.take(np.argmax(proba[:, 0], axis=1), axis=0)
            out = np.zeros((n, self.n_outputs_), dtype=self.classes_[0].dtype)
            for k in range(self.n_outputs_):
                out[:, k] = self.classes_[k].take(np.argmax(proba[:, k], axis=1), axis=0)
            return out
        if self.n_outputs_ == 1:
            return proba[:, 0, 0]
        return proba[:, :, 0]


class DecisionTreeClassifier(ClassifierMixin, BaseDecisionTree):
    """CART classifier (gini / entropy)."""

    def __init__(self, *, criterion="gini", splitter="best", max_depth=None, min_samples_split=2,
                 min_samples_leaf=1, min_weight_fraction_leaf=0.0, max_features=None,
                 random_state=None, max_leaf_nodes=None, min_impurity_decrease=0.0,
                 class_weight=None, ccp_alpha=0.0):
        self.criterion = criterion
        self.splitter = splitter
        self.max_depth = max_depth
        self.min_samples_split = min_samples_split
        self.min_samples_leaf = min_samples_leaf
        self.min_weight_fraction_leaf = min_weight_fraction_leaf
        self.max_features = max_features
        self.random_state = random_state
        self.max_leaf_nodes = max_leaf_nodes
        self.min_impurity_decrease = min_impurity_decrease
        self.class_weight = class_weight
        self.ccp_alpha = ccp_alpha

    def predict_proba(self, X, check_input=True):
        proba = self.tree_.predict(self._validate_X_predict(X, check_input))
        if self.n_outputs_ == 1:
            p = proba[:, 0, :self.n_classes_]
            norm = p.sum(axis=1)
            norm[norm == 0.0] = 1.0
            return p / norm[:, None]
        out = []
        for k in range(self.n_outputs_):
            p = proba[:, k, :self.n_classes_[k]]
            norm = p.sum(axis=1)
            norm[norm == 0.0] = 1.0
            out.append(p / norm[:, None])
        return out

    def predict_log_proba(self, X):
        proba = self.predict_proba(X)
        if self.n_outputs_ == 1:
            return np.log(proba)
        return [np.log(p) for p in proba]


class DecisionTreeRegressor(RegressorMixin, BaseDecisionTree):
    """CART regressor (squared / Friedman / absolute error, Poisson)."""

    def __init__(self, *, criterion="squared_error", splitter="best", max_depth=None,
                 min_samples_split=2, min_samples_leaf=1, min_weight_fraction_leaf=0.0,
                 max_features=None, random_state=None, max_leaf_nodes=None,
                 min_impurity_decrease=0.0, ccp_alpha=0.0):
        self.criterion = criterion
        self.splitter = splitter
        self.max_depth = max_depth
        self.min_samples_split = min_samples_split
        self.min_samples_leaf = min_samples_leaf
        self.min_weight_fraction_leaf = min_weight_fraction_leaf
        self.max_features = max_features
        self.random_state = random_state
        self.max_leaf_nodes = max_leaf_nodes
        self.min_impurity_decrease = min_impurity_decrease
        self.ccp_alpha = ccp_alpha


class ExtraTreeClassifier(DecisionTreeClassifier):
    """Extremely randomized tree classifier (random thresholds)."""

    def __init__(self, *, criterion="gini", splitter="random", max_depth=None,
                 min_samples_split=2, min_samples_leaf=1, min_weight_fraction_leaf=0.0,
                 max_features="auto", random_state=None, max_leaf_nodes=None,
                 min_impurity_decrease=0.0, class_weight=None, ccp_alpha=0.0):
        super().__init__(criterion=criterion, splitter=splitter, max_depth=max_depth,
                         min_samples_split=min_samples_split, min_samples_leaf=min_samples_leaf,
                         min_weight_fraction_leaf=min_weight_fraction_leaf,
                         max_features=max_features, random_state=random_state,
                         max_leaf_nodes=max_leaf_nodes,
                         min_impurity_decrease=min_impurity_decrease, class_weight=class_weight,
                         ccp_alpha=ccp_alpha)


class ExtraTreeRegressor(DecisionTreeRegressor):
    """Extremely randomized tree regressor (random thresholds)."""

    def __init__(self, *, criterion="squared_error", splitter="random", max_depth=None,
                 min_samples_split=2, min_samples_leaf=1, min_weight_fraction_leaf=0.0,
                 max_features="auto", random_state=None, min_impurity_decrease=0.0,
                 max_leaf_nodes=None, ccp_alpha=0.0):
        super().__init__(criterion=criterion, splitter=splitter, max_depth=max_depth,
                         min_samples_split=min_samples_split, min_samples_leaf=min_samples_leaf,
                         min_weight_fraction_leaf=min_weight_fraction_leaf,
                         max_features=max_features, random_state=random_state,
                         max_leaf_nodes=max_leaf_nodes,
                         min_impurity_decrease=min_impurity_decrease, ccp_alpha=ccp_alpha)


__all__ = ["DecisionTreeClassifier", "DecisionTreeRegressor", "ExtraTreeClassifier",
           "ExtraTreeRegressor", "Tree"]
