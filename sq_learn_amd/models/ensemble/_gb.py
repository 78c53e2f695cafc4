"""Gradient tree boosting (reference ``ensemble/_gb.py``: ``_fit_stage``
:173-225, ``fit`` :371-530, ``_fit_stages`` :532-615, staged prediction,
``GradientBoostingClassifier`` / ``GradientBoostingRegressor``; losses of
``ensemble/_gb_losses.py``: least squares, least absolute deviation, Huber,
quantile, binomial / multinomial deviance, exponential).

Each stage grows K Friedman-MSE regression trees on the negative gradient
with the host-native builder (``csrc/host/tree.cpp``), then replaces the
leaf values by the loss's line-search / Newton step.  The boosting RNG is
the reference's: one ``RandomState`` shared by the subsample masks
(``_random_sample_mask``) and the per-tree splitter seeds.
"""

import numbers
import warnings

import numpy as np
from scipy.special import expit, logsumexp

from ...base import BaseEstimator, ClassifierMixin, RegressorMixin, is_classifier
from ...dummy import DummyClassifier, DummyRegressor
from ...utils.stats import _weighted_percentile
from ...utils.validation import check_is_fitted, check_random_state
from ..tree import DecisionTreeRegressor
from ..tree._classes import _as_f32, resolve_max_features
from ..tree._tree import RAND_R_MAX, TREE_LEAF, build_trees, forest_apply

# --------------------------------------------------------------------- losses


class LossFunction:
    is_multi_class = False

    def __init__(self, n_classes):
        self.K = n_classes

    def update_terminal_regions(self, tree, X, y, residual, raw, sample_weight, sample_mask,
                                learning_rate=0.1, k=0):
        terminal = tree.apply(X)
        masked = terminal.copy()
        masked[~sample_mask] = -1
        leaves = np.where(tree.children_left == TREE_LEAF)[0]
        # one pass grouping rows by leaf instead of a scan per leaf
        order = np.argsort(masked, kind="stable")
        sorted_leaf = masked[order]
        starts = np.searchsorted(sorted_leaf, leaves, side="left")
        ends = np.searchsorted(sorted_leaf, leaves, side="right")
        for leaf, s, e in zip(leaves, starts, ends):
            self._update_terminal_region(tree, order[s:e], leaf, y, residual, raw[:, k],
                                         sample_weight)
        raw[:, k] += learning_rate * tree.value[:, 0, 0].take(terminal, axis=0)


class LeastSquaresError(LossFunction):
    def __init__(self):
        super().__init__(1)

    def init_estimator(self):
        return DummyRegressor(strategy="mean")

    def __call__(self, y, raw, sample_weight=None):
        if sample_weight is None:
            return np.mean((y - raw.ravel()) ** 2)
        return 1 / sample_weight.sum() * np.sum(sample_weight * ((y - raw.ravel()) ** 2))

    def negative_gradient(self, y, raw, **kw):
        return y - raw.ravel()

    def update_terminal_regions(self, tree, X, y, residual, raw, sample_weight, sample_mask,
                                learning_rate=0.1, k=0):
        raw[:, k] += learning_rate * tree.predict(X).ravel()

    def get_init_raw_predictions(self, X, est):
        return est.predict(X).reshape(-1, 1).astype(np.float64)


class LeastAbsoluteError(LeastSquaresError):
    def init_estimator(self):
        return DummyRegressor(strategy="quantile", quantile=0.5)

    def __call__(self, y, raw, sample_weight=None):
        if sample_weight is None:
            return np.abs(y - raw.ravel()).mean()
        return 1 / sample_weight.sum() * np.sum(sample_weight * np.abs(y - raw.ravel()))

    def negative_gradient(self, y, raw, **kw):
        return 2 * (y - raw.ravel() > 0) - 1

    update_terminal_regions = LossFunction.update_terminal_regions

    def _update_terminal_region(self, tree, idx, leaf, y, residual, raw, sw):
        diff = y.take(idx) - raw.take(idx)
        tree.value[leaf, 0, 0] = _weighted_percentile(diff, sw.take(idx), percentile=50)


class HuberLossFunction(LeastSquaresError):
    def __init__(self, alpha=0.9):
        super().__init__()
        self.alpha = alpha
        self.gamma = None

    def init_estimator(self):
        return DummyRegressor(strategy="quantile", quantile=0.5)

    def __call__(self, y, raw, sample_weight=None):
        diff = y - raw.ravel()
        gamma = self.gamma
        if gamma is None:
            gamma = (np.percentile(np.abs(diff), self.alpha * 100) if sample_weight is None
                     else _weighted_percentile(np.abs(diff), sample_weight, self.alpha * 100))
        m = np.abs(diff) <= gamma
        if sample_weight is None:
            return (np.sum(0.5 * diff[m] ** 2) + np.sum(gamma * (np.abs(diff[~m]) - gamma / 2))
                    ) / y.shape[0]
        return (np.sum(0.5 * sample_weight[m] * diff[m] ** 2)
                + np.sum(gamma * sample_weight[~m] * (np.abs(diff[~m]) - gamma / 2))
                ) / sample_weight.sum()

    def negative_gradient(self, y, raw, sample_weight=None, **kw):
        diff = y - raw.ravel()
        gamma = (np.percentile(np.abs(diff), self.alpha * 100) if sample_weight is None
                 else _weighted_percentile(np.abs(diff), sample_weight, self.alpha * 100))
        m = np.abs(diff) <= gamma
        res = np.zeros(y.shape[0])
        res[m] = diff[m]
        res[~m] = gamma * np.sign(diff[~m])
        self.gamma = gamma
        return res

    update_terminal_regions = LossFunction.update_terminal_regions

    def _update_terminal_region(self, tree, idx, leaf, y, residual, raw, sw):
        diff = y.take(idx) - raw.take(idx)
        med = _weighted_percentile(diff, sw.take(idx), percentile=50)
        dm = diff - med
        tree.value[leaf, 0] = med + np.mean(np.sign(dm) * np.minimum(np.abs(dm), self.gamma))


class QuantileLossFunction(LeastSquaresError):
    def __init__(self, alpha=0.9):
        super().__init__()
        self.alpha = alpha
        self.percentile = alpha * 100

    def init_estimator(self):
        return DummyRegressor(strategy="quantile", quantile=self.alpha)

    def __call__(self, y, raw, sample_weight=None):
        raw = raw.ravel()
        diff = y - raw
        m = y > raw
        a = self.alpha
        if sample_weight is None:
            return (a * diff[m].sum() - (1 - a) * diff[~m].sum()) / y.shape[0]
        return ((a * np.sum(sample_weight[m] * diff[m])
                 - (1 - a) * np.sum(sample_weight[~m] * diff[~m])) / sample_weight.sum())

    def negative_gradient(self, y, raw, **kw):
        m = y > raw.ravel()
        return (self.alpha * m) - ((1 - self.alpha) * ~m)

    update_terminal_regions = LossFunction.update_terminal_regions

    def _update_terminal_region(self, tree, idx, leaf, y, residual, raw, sw):
        diff = y.take(idx) - raw.take(idx)
        tree.value[leaf, 0] = _weighted_percentile(diff, sw.take(idx), self.percentile)


class BinomialDeviance(LossFunction):
    def __init__(self, n_classes):
        if n_classes != 2:
            raise ValueError("{0:s} requires 2 classes; got {1:d} class(es)"
                             .format(self.__class__.__name__, n_classes))
        super().__init__(1)

    def init_estimator(self):
        return DummyClassifier(strategy="prior")

    def __call__(self, y, raw, sample_weight=None):
        raw = raw.ravel()
        if sample_weight is None:
            return -2 * np.mean((y * raw) - np.logaddexp(0, raw))
        return -2 / sample_weight.sum() * np.sum(sample_weight * ((y * raw)
                                                                   - np.logaddexp(0, raw)))

    def negative_gradient(self, y, raw, **kw):
        return y - expit(raw.ravel())

    def _update_terminal_region(self, tree, idx, leaf, y, residual, raw, sw):
        r, yy, w = residual.take(idx), y.take(idx), sw.take(idx)
        num = np.sum(w * r)
        den = np.sum(w * (yy - r) * (1 - yy + r))
        tree.value[leaf, 0, 0] = 0.0 if abs(den) < 1e-150 else num / den

    def _raw_prediction_to_proba(self, raw):
        p = np.ones((raw.shape[0], 2))
        p[:, 1] = expit(raw.ravel())
        p[:, 0] -= p[:, 1]
        return p

    def _raw_prediction_to_decision(self, raw):
        return np.argmax(self._raw_prediction_to_proba(raw), axis=1)

    def get_init_raw_predictions(self, X, est):
        p = np.clip(est.predict_proba(X)[:, 1], np.finfo(np.float32).eps,
                    1 - np.finfo(np.float32).eps)
        return np.log(p / (1 - p)).reshape(-1, 1).astype(np.float64)


class MultinomialDeviance(LossFunction):
    is_multi_class = True

    def __init__(self, n_classes):
        if n_classes < 3:
            raise ValueError("{0:s} requires more than 2 classes.".format(self.__class__.__name__))
        super().__init__(n_classes)

    def init_estimator(self):
        return DummyClassifier(strategy="prior")

    def __call__(self, y, raw, sample_weight=None):
        Y = np.zeros((y.shape[0], self.K))
        for k in range(self.K):
            Y[:, k] = y == k
        return np.average(-1 * (Y * raw).sum(axis=1) + logsumexp(raw, axis=1),
                          weights=sample_weight)

    def negative_gradient(self, y, raw, k=0, **kw):
        return y - np.nan_to_num(np.exp(raw[:, k] - logsumexp(raw, axis=1)))

    def _update_terminal_region(self, tree, idx, leaf, y, residual, raw, sw):
        r, yy, w = residual.take(idx), y.take(idx), sw.take(idx)
        num = np.sum(w * r) * (self.K - 1) / self.K
        den = np.sum(w * (yy - r) * (1 - yy + r))
        tree.value[leaf, 0, 0] = 0.0 if abs(den) < 1e-150 else num / den

    def _raw_prediction_to_proba(self, raw):
        return np.nan_to_num(np.exp(raw - logsumexp(raw, axis=1)[:, None]))

    def _raw_prediction_to_decision(self, raw):
        return np.argmax(self._raw_prediction_to_proba(raw), axis=1)

    def get_init_raw_predictions(self, X, est):
        p = np.clip(est.predict_proba(X), np.finfo(np.float32).eps, 1 - np.finfo(np.float32).eps)
        return np.log(p).astype(np.float64)


class ExponentialLoss(BinomialDeviance):
    def __call__(self, y, raw, sample_weight=None):
        raw = raw.ravel()
        if sample_weight is None:
            return np.mean(np.exp(-(2.0 * y - 1.0) * raw))
        return 1.0 / sample_weight.sum() * np.sum(sample_weight * np.exp(-(2 * y - 1) * raw))

    def negative_gradient(self, y, raw, **kw):
        y_ = -(2.0 * y - 1.0)
        return y_ * np.exp(y_ * raw.ravel())

    def _update_terminal_region(self, tree, idx, leaf, y, residual, raw, sw):
        rp, yy, w = raw.take(idx), y.take(idx), sw.take(idx)
        y_ = 2.0 * yy - 1.0
        num = np.sum(y_ * w * np.exp(-y_ * rp))
        den = np.sum(w * np.exp(-y_ * rp))
        tree.value[leaf, 0, 0] = 0.0 if abs(den) < 1e-150 else num / den

    def _raw_prediction_to_proba(self, raw):
        p = np.ones((raw.shape[0], 2))
        p[:, 1] = expit(2.0 * raw.ravel())
        p[:, 0] -= p[:, 1]
        return p

    def _raw_prediction_to_decision(self, raw):
        return (raw.ravel() >= 0).astype(int)

    def get_init_raw_predictions(self, X, est):
        p = np.clip(est.predict_proba(X)[:, 1], np.finfo(np.float32).eps,
                    1 - np.finfo(np.float32).eps)
        return (0.5 * np.log(p / (1 - p))).reshape(-1, 1).astype(np.float64)


LOSS_FUNCTIONS = {"squared_error": LeastSquaresError, "ls": LeastSquaresError,
                  "absolute_error": LeastAbsoluteError, "lad": LeastAbsoluteError,
                  "huber": HuberLossFunction, "quantile": QuantileLossFunction,
                  "deviance": None, "log_loss": None, "exponential": ExponentialLoss}


def _random_sample_mask(n_total, n_in_bag, random_state):
    """Reference ``_gradient_boosting.pyx:241``: exactly n_in_bag rows by
    sequential selection sampling over one ``rand(n)`` draw."""
    rand = random_state.rand(n_total)
    mask = np.zeros(n_total, dtype=bool)
    bagged = 0
    for i in range(n_total):
        if rand[i] * (n_total - i) < (n_in_bag - bagged):
            mask[i] = True
            bagged += 1
    return mask


# ------------------------------------------------------------------ boosting


class BaseGradientBoosting(BaseEstimator):
    _SUPPORTED_LOSS = ()

    def _check_params(self):
        if self.n_estimators <= 0:
            raise ValueError("n_estimators must be greater than 0 but was %r" % self.n_estimators)
        if self.learning_rate <= 0.0:
            raise ValueError("learning_rate must be greater than 0 but was %r"
                             % self.learning_rate)
        if self.loss not in self._SUPPORTED_LOSS:
            raise ValueError("Loss '{0:s}' not supported. ".format(self.loss))
        if self.loss in ("deviance", "log_loss"):
            cls = MultinomialDeviance if len(self.classes_) > 2 else BinomialDeviance
            self.loss_ = cls(self.n_classes_)
        elif is_classifier(self):
            self.loss_ = LOSS_FUNCTIONS[self.loss](self.n_classes_)
        elif self.loss in ("huber", "quantile"):
            self.loss_ = LOSS_FUNCTIONS[self.loss](self.alpha)
        else:
            self.loss_ = LOSS_FUNCTIONS[self.loss]()
        if not 0.0 < self.subsample <= 1.0:
            raise ValueError("subsample must be in (0,1] but was %r" % self.subsample)
        if self.init is not None and not (isinstance(self.init, str) and self.init == "zero"):
            if not hasattr(self.init, "fit"):
                raise ValueError("The init parameter must be an estimator or 'zero'. Got init={}"
                                 .format(self.init))
        if not 0.0 < self.alpha < 1.0:
            raise ValueError("alpha must be in (0.0, 1.0) but was %r" % self.alpha)
        self.max_features_ = resolve_max_features(self.max_features, self.n_features_in_,
                                                  is_classifier(self))

    def _tree_params(self, n, sample_weight):
        proto = DecisionTreeRegressor(criterion=self.criterion, max_depth=self.max_depth,
                                      min_samples_split=self.min_samples_split,
                                      min_samples_leaf=self.min_samples_leaf,
                                      min_weight_fraction_leaf=self.min_weight_fraction_leaf,
                                      min_impurity_decrease=self.min_impurity_decrease,
                                      max_features=self.max_features,
                                      max_leaf_nodes=self.max_leaf_nodes, ccp_alpha=self.ccp_alpha)
        return proto, proto._resolve_params(n, self.n_features_in_, sample_weight)

    def _fit_stage(self, i, X, y, raw, sample_weight, sample_mask, random_state):
        loss = self.loss_
        original_y = y
        raw_copy = raw.copy()
        n = X.shape[0]
        for k in range(loss.K):
            if loss.is_multi_class:
                y = np.array(original_y == k, dtype=np.float64)
            residual = loss.negative_gradient(y, raw_copy, k=k, sample_weight=sample_weight)
            proto, params = self._tree_params(n, None)
            sw = sample_weight * sample_mask.astype(np.float64) if self.subsample < 1.0 \
                else sample_weight
            params["min_weight_leaf"] = self.min_weight_fraction_leaf * float(np.sum(sw))
            seed = random_state.randint(0, RAND_R_MAX)
            tree_ = build_trees(X, residual.astype(np.float64), sw[None], [1], params, [seed],
                                n_threads=1)[0]
            tree = DecisionTreeRegressor(**proto.get_params())
            tree.tree_ = tree_
            tree.n_features_in_ = X.shape[1]
            tree.n_outputs_ = 1
            tree.max_features_ = params["max_features"]
            tree._prune_tree()
            loss.update_terminal_regions(tree.tree_, X, y, residual, raw, sample_weight,
                                         sample_mask, learning_rate=self.learning_rate, k=k)
            self.estimators_[i, k] = tree
        return raw

    def _init_state(self):
        self.init_ = self.init
        if self.init_ is None:
            self.init_ = self.loss_.init_estimator()
        self.estimators_ = np.empty((self.n_estimators, self.loss_.K), dtype=object)
        self.train_score_ = np.zeros((self.n_estimators,), dtype=np.float64)
        if self.subsample < 1.0:
            self.oob_improvement_ = np.zeros((self.n_estimators,), dtype=np.float64)

    def _clear_state(self):
        for a in ("estimators_", "train_score_", "oob_improvement_", "init_", "_rng"):
            if hasattr(self, a):
                delattr(self, a)

    def _resize_state(self):
        total = self.n_estimators
        if total < self.estimators_.shape[0]:
            raise ValueError("resize with smaller n_estimators %d < %d"
                             % (total, self.estimators_.shape[0]))
        self.estimators_ = np.resize(self.estimators_, (total, self.loss_.K))
        self.train_score_ = np.resize(self.train_score_, total)
        if self.subsample < 1 or hasattr(self, "oob_improvement_"):
            if hasattr(self, "oob_improvement_"):
                self.oob_improvement_ = np.resize(self.oob_improvement_, total)
            else:
                self.oob_improvement_ = np.zeros((total,), dtype=np.float64)

    def _is_initialized(self):
        return len(getattr(self, "estimators_", [])) > 0

    def fit(self, X, y, sample_weight=None, monitor=None):
        if not self.warm_start:
            self._clear_state()
        X = _as_f32(X)
        n_samples = X.shape[0]
        self.n_features_in_ = X.shape[1]
        y = np.asarray(y).reshape(-1)
        sw_none = sample_weight is None
        sample_weight = (np.ones(n_samples) if sample_weight is None
                         else np.asarray(sample_weight, dtype=np.float64).reshape(-1))
        y = self._validate_y(y, sample_weight)
        if self.n_iter_no_change is not None:
            from ...model_selection import train_test_split
            strat = y if is_classifier(self) else None
            X, X_val, y, y_val, sample_weight, sw_val = train_test_split(
                X, y, sample_weight, random_state=self.random_state,
                test_size=self.validation_fraction, stratify=strat)
            if is_classifier(self) and self._n_classes != np.unique(y).shape[0]:
                raise ValueError("The training data after the early stopping split is missing "
                                 "some classes. Try using another random seed.")
        else:
            X_val = y_val = sw_val = None
        self._check_params()
        if not self._is_initialized():
            self._init_state()
            if self.init_ == "zero":
                raw = np.zeros((X.shape[0], self.loss_.K))
            else:
                if sw_none:
                    self.init_.fit(X, y)
                else:
                    self.init_.fit(X, y, sample_weight=sample_weight)
                raw = self.loss_.get_init_raw_predictions(X, self.init_)
            begin = 0
            self._rng = check_random_state(self.random_state)
        else:
            if self.n_estimators < self.estimators_.shape[0]:
                raise ValueError("n_estimators=%d must be larger or equal to "
                                 "estimators_.shape[0]=%d when warm_start==True"
                                 % (self.n_estimators, self.estimators_.shape[0]))
            begin = self.estimators_.shape[0]
            raw = self._raw_predict(X)
            self._resize_state()
        n_stages = self._fit_stages(X, y, raw, sample_weight, self._rng, X_val, y_val, sw_val,
                                    begin, monitor)
        if n_stages != self.estimators_.shape[0]:
            self.estimators_ = self.estimators_[:n_stages]
            self.train_score_ = self.train_score_[:n_stages]
            if hasattr(self, "oob_improvement_"):
                self.oob_improvement_ = self.oob_improvement_[:n_stages]
        self.n_estimators_ = n_stages
        return self

    def _fit_stages(self, X, y, raw, sample_weight, rs, X_val, y_val, sw_val, begin, monitor):
        n = X.shape[0]
        do_oob = self.subsample < 1.0
        mask = np.ones(n, dtype=bool)
        n_inbag = max(1, int(self.subsample * n))
        loss = self.loss_
        if self.n_iter_no_change is not None:
            history = np.full(self.n_iter_no_change, np.inf)
            val_iter = self._staged_raw_predict(X_val)
        i = begin
        for i in range(begin, self.n_estimators):
            if do_oob:
                mask = _random_sample_mask(n, n_inbag, rs)
                old_oob = loss(y[~mask], raw[~mask], sample_weight[~mask])
            raw = self._fit_stage(i, X, y, raw, sample_weight, mask, rs)
            if do_oob:
                self.train_score_[i] = loss(y[mask], raw[mask], sample_weight[mask])
                self.oob_improvement_[i] = old_oob - loss(y[~mask], raw[~mask],
                                                          sample_weight[~mask])
            else:
                self.train_score_[i] = loss(y, raw, sample_weight)
            if self.verbose > 0:
                print("%10d %16.4f" % (i + 1, self.train_score_[i]))
            if monitor is not None and monitor(i, self, locals()):
                break
            if self.n_iter_no_change is not None:
                vl = loss(y_val, next(val_iter), sw_val)
                if np.any(vl + self.tol < history):
                    history[i % len(history)] = vl
                else:
                    break
        return i + 1

    # ----------------------------------------------------------- prediction
    def _raw_predict_init(self, X):
        check_is_fitted(self, "estimators_")
        if self.init_ == "zero":
            return np.zeros((X.shape[0], self.loss_.K))
        return self.loss_.get_init_raw_predictions(X, self.init_).astype(np.float64)

    def _leaf_values(self, X):
        """(n, n_stages, K) leaf values of every tree (one native traversal)."""
        trees = [e.tree_ for e in self.estimators_.ravel()]
        leaves = forest_apply(trees, X)
        vals = np.empty(leaves.shape)
        for j, t in enumerate(trees):
            vals[:, j] = t.value[:, 0, 0].take(leaves[:, j])
        return vals.reshape(X.shape[0], self.estimators_.shape[0], self.loss_.K)

    def _raw_predict(self, X):
        raw = self._raw_predict_init(X)
        if self.estimators_.size:
            raw += self.learning_rate * self._leaf_values(X).sum(axis=1)
        return raw

    def _staged_raw_predict(self, X):
        X = _as_f32(X)
        raw = self._raw_predict_init(X)
        for i in range(self.estimators_.shape[0]):
            for k in range(self.loss_.K):
                raw[:, k] += self.learning_rate * self.estimators_[i, k].tree_.predict(X)[:, 0, 0]
            yield raw.copy()

    def _validate_X(self, X):
        X = _as_f32(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError(f"X has {X.shape[1]} features, but {self.__class__.__name__} is "
                             f"expecting {self.n_features_in_} features as input.")
        return X

    @property
    def feature_importances_(self):
        check_is_fitted(self, "estimators_")
        rel = [np.mean([t.tree_.compute_feature_importances(normalize=False) for t in stage],
                       axis=0)
               for stage in self.estimators_ if any(t.tree_.node_count > 1 for t in stage)]
        if not rel:
            return np.zeros(self.n_features_in_, dtype=np.float64)
        avg = np.mean(rel, axis=0, dtype=np.float64)
        return avg / np.sum(avg)

    def apply(self, X):
        X = self._validate_X(X)
        trees = [e.tree_ for e in self.estimators_.ravel()]
        return forest_apply(trees, X).reshape(X.shape[0], *self.estimators_.shape)


class GradientBoostingClassifier(ClassifierMixin, BaseGradientBoosting):
    _SUPPORTED_LOSS = ("deviance", "log_loss", "exponential")

    def __init__(self, *, loss="deviance", learning_rate=0.1, n_estimators=100, subsample=1.0,
                 criterion="friedman_mse", min_samples_split=2, min_samples_leaf=1,
                 min_weight_fraction_leaf=0.0, max_depth=3, min_impurity_decrease=0.0, init=None,
                 random_state=None, max_features=None, verbose=0, max_leaf_nodes=None,
                 warm_start=False, validation_fraction=0.1, n_iter_no_change=None, tol=1e-4,
                 ccp_alpha=0.0):
        self.loss = loss
        self.learning_rate = learning_rate
        self.n_estimators = n_estimators
        self.subsample = subsample
        self.criterion = criterion
        self.min_samples_split = min_samples_split
        self.min_samples_leaf = min_samples_leaf
        self.min_weight_fraction_leaf = min_weight_fraction_leaf
        self.max_depth = max_depth
        self.min_impurity_decrease = min_impurity_decrease
        self.init = init
        self.random_state = random_state
        self.max_features = max_features
        self.verbose = verbose
        self.max_leaf_nodes = max_leaf_nodes
        self.warm_start = warm_start
        self.validation_fraction = validation_fraction
        self.n_iter_no_change = n_iter_no_change
        self.tol = tol
        self.ccp_alpha = ccp_alpha

    alpha = 0.9   # (regression-loss quantile; fixed for the classifier, not a parameter)

    def _validate_y(self, y, sample_weight):
        self.classes_, y = np.unique(y, return_inverse=True)
        n_trim = np.count_nonzero(np.bincount(y, sample_weight))
        if n_trim < 2:
            raise ValueError("y contains %d class after sample_weight trimmed classes with zero "
                             "weights, while a minimum of 2 classes are required." % n_trim)
        self._n_classes = len(self.classes_)
        self.n_classes_ = self._n_classes
        return y

    def decision_function(self, X):
        raw = self._raw_predict(self._validate_X(X))
        return raw.ravel() if raw.shape[1] == 1 else raw

    def staged_decision_function(self, X):
        for raw in self._staged_raw_predict(self._validate_X(X)):
            yield raw.ravel() if raw.shape[1] == 1 else raw

    def predict(self, X):
        raw = self._raw_predict(self._validate_X(X))
        return self.classes_.take(self.loss_._raw_prediction_to_decision(raw), axis=0)

    def staged_predict(self, X):
        for raw in self._staged_raw_predict(self._validate_X(X)):
            yield self.classes_.take(self.loss_._raw_prediction_to_decision(raw), axis=0)

    def predict_proba(self, X):
        return self.loss_._raw_prediction_to_proba(self._raw_predict(self._validate_X(X)))

    def predict_log_proba(self, X):
        return np.log(self.predict_proba(X))

    def staged_predict_proba(self, X):
        for raw in self._staged_raw_predict(self._validate_X(X)):
            yield self.loss_._raw_prediction_to_proba(raw)


class GradientBoostingRegressor(RegressorMixin, BaseGradientBoosting):
    _SUPPORTED_LOSS = ("squared_error", "ls", "absolute_error", "lad", "huber", "quantile")

    def __init__(self, *, loss="squared_error", learning_rate=0.1, n_estimators=100,
                 subsample=1.0, criterion="friedman_mse", min_samples_split=2,
                 min_samples_leaf=1, min_weight_fraction_leaf=0.0, max_depth=3,
                 min_impurity_decrease=0.0, init=None, random_state=None, max_features=None,
                 alpha=0.9, verbose=0, max_leaf_nodes=None, warm_start=False,
                 validation_fraction=0.1, n_iter_no_change=None, tol=1e-4, ccp_alpha=0.0):
        self.loss = loss
        self.learning_rate = learning_rate
        self.n_estimators = n_estimators
        self.subsample = subsample
        self.criterion = criterion
        self.min_samples_split = min_samples_split
        self.min_samples_leaf = min_samples_leaf
        self.min_weight_fraction_leaf = min_weight_fraction_leaf
        self.max_depth = max_depth
        self.min_impurity_decrease = min_impurity_decrease
        self.init = init
        self.random_state = random_state
        self.max_features = max_features
        self.alpha = alpha
        self.verbose = verbose
        self.max_leaf_nodes = max_leaf_nodes
        self.warm_start = warm_start
        self.validation_fraction = validation_fraction
        self.n_iter_no_change = n_iter_no_change
        self.tol = tol
        self.ccp_alpha = ccp_alpha

    def _validate_y(self, y, sample_weight=None):
        return np.asarray(y, dtype=np.float64)

    def predict(self, X):
        return self._raw_predict(self._validate_X(X)).ravel()

    def staged_predict(self, X):
        for raw in self._staged_raw_predict(self._validate_X(X)):
            yield raw.ravel()

    def apply(self, X):
        return super().apply(X)[:, :, 0]


__all__ = ["GradientBoostingClassifier", "GradientBoostingRegressor"]
