"""Forests of randomized trees (reference ``ensemble/_forest.py``:
``_generate_sample_indices`` :118, ``_parallel_build_trees`` :141,
``BaseForest.fit`` :300-427, OOB :441-500, ``feature_importances_`` :514,
``ForestClassifier`` :575, ``RandomForestClassifier``,
``RandomForestRegressor``, ``ExtraTreesClassifier``, ``ExtraTreesRegressor``,
``RandomTreesEmbedding``).

All trees of a fit are grown by ONE native call (``csrc/host/tree.cpp``,
OpenMP over trees) - the reference's joblib threading backend over Cython
builders, without per-tree Python work.  Per-tree seeds and bootstrap draws
reproduce the reference's streams: tree seed t = ``rs.randint(2**31 - 1)``,
bootstrap = ``RandomState(t).randint(0, n, n_bootstrap)``, splitter seed =
``RandomState(t).randint(0, 2**31 - 1)``.  Prediction on GPU rows runs the
HIP ``forest_predict`` kernel over device-resident node tables.
"""

import numbers
import threading
import warnings

import numpy as np
import scipy.sparse as sp
import torch

from ...base import BaseEstimator, ClassifierMixin, RegressorMixin, TransformerMixin
from ...exceptions import DataConversionWarning
from ...utils.class_weight import compute_sample_weight
from ...utils.validation import check_is_fitted, check_random_state
from ..tree import (DecisionTreeClassifier, DecisionTreeRegressor, ExtraTreeClassifier,
                    ExtraTreeRegressor)
from ..tree._classes import _as_f32, resolve_max_features
from ..tree._tree import RAND_R_MAX, build_trees, forest_apply, stack_trees

MAX_INT = np.iinfo(np.int32).max


def _get_n_samples_bootstrap(n_samples, max_samples):
    if max_samples is None:
        return n_samples
    if isinstance(max_samples, numbers.Integral):
        if not 1 <= max_samples <= n_samples:
            raise ValueError("`max_samples` must be in range 1 to {} but got value {}"
                             .format(n_samples, max_samples))
        return int(max_samples)
    if isinstance(max_samples, numbers.Real):
        if not 0 < max_samples < 1:
            raise ValueError("`max_samples` must be in range (0, 1) but got value {}"
                             .format(max_samples))
        return round(n_samples * max_samples)
    raise TypeError("`max_samples` should be int or float, but got type '{}'"
                    .format(type(max_samples)))


def _generate_sample_indices(random_state, n_samples, n_samples_bootstrap):
    return check_random_state(random_state).randint(0, n_samples, n_samples_bootstrap)


def _generate_unsampled_indices(random_state, n_samples, n_samples_bootstrap):
    idx = _generate_sample_indices(random_state, n_samples, n_samples_bootstrap)
    counts = np.bincount(idx, minlength=n_samples)
    return np.arange(n_samples)[counts == 0]


class BaseForest(BaseEstimator):
    """Shared forest machinery."""

    _tree_cls = None
    _tree_params = ("criterion", "max_depth", "min_samples_split", "min_samples_leaf",
                    "min_weight_fraction_leaf", "max_features", "max_leaf_nodes",
                    "min_impurity_decrease", "ccp_alpha")

    def _make_tree(self, seed):
        kw = {p: getattr(self, p) for p in self._tree_params if hasattr(self, p)}
        t = self._tree_cls(**kw)
        t.random_state = int(seed)
        return t

    def _validate_y_class_weight(self, y):
        return y, None

    def fit(self, X, y, sample_weight=None):
        if sp.issparse(y):
            raise ValueError("sparse multilabel-indicator for y is not supported.")
        X = _as_f32(X)
        n_samples, n_features = X.shape
        self.n_features_in_ = n_features
        y = np.atleast_1d(np.asarray(y.detach().cpu().numpy() if isinstance(y, torch.Tensor) else y))
        if y.ndim == 2 and y.shape[1] == 1:
            warnings.warn("A column-vector y was passed when a 1d array was expected. Please "
                          "change the shape of y to (n_samples,), for example using ravel().",
                          DataConversionWarning, stacklevel=2)
        if y.ndim == 1:
            y = y.reshape(-1, 1)
        if y.shape[0] != n_samples:
            raise ValueError("Found input variables with inconsistent numbers of samples: "
                             f"[{n_samples}, {y.shape[0]}]")
        self.n_outputs_ = y.shape[1]
        y, expanded_cw = self._validate_y_class_weight(y)
        y = np.ascontiguousarray(y, dtype=np.float64)
        if sample_weight is not None:
            sample_weight = np.asarray(sample_weight, dtype=np.float64).reshape(-1)
        if expanded_cw is not None:
            sample_weight = expanded_cw if sample_weight is None else sample_weight * expanded_cw
        n_boot = _get_n_samples_bootstrap(n_samples, self.max_samples)
        if not self.bootstrap and self.oob_score:
            raise ValueError("Out of bag estimation only available if bootstrap=True")
        if not isinstance(self.n_estimators, numbers.Integral) or self.n_estimators <= 0:
            raise ValueError("n_estimators must be greater than zero, got {0}."
                             .format(self.n_estimators))
        random_state = check_random_state(self.random_state)
        if not self.warm_start or not hasattr(self, "estimators_"):
            self.estimators_ = []
            self._device_tables = None
        n_more = self.n_estimators - len(self.estimators_)
        if n_more < 0:
            raise ValueError("n_estimators=%d must be larger or equal to len(estimators_)=%d "
                             "when warm_start==True" % (self.n_estimators, len(self.estimators_)))
        if n_more == 0:
            warnings.warn("Warm-start fitting without increasing n_estimators does not fit "
                          "new trees.")
        else:
            if self.warm_start and len(self.estimators_) > 0:
                random_state.randint(MAX_INT, size=len(self.estimators_))
            tree_seeds = [random_state.randint(MAX_INT) for _ in range(n_more)]
            self._grow(X, y, sample_weight, tree_seeds, n_boot)
            self._device_tables = None
        if self.oob_score:
            self._set_oob_score_and_attributes(X, y)
        if hasattr(self, "classes_") and self.n_outputs_ == 1:
            self.n_classes_ = self.n_classes_[0]
            self.classes_ = self.classes_[0]
        return self

    def _grow(self, X, y, sample_weight, tree_seeds, n_boot):
        n = X.shape[0]
        trees = [self._make_tree(s) for s in tree_seeds]
        proto = trees[0]
        params = proto._resolve_params(n, X.shape[1], sample_weight)
        if isinstance(self, ClassifierMixin):
            n_classes = np.asarray(self.n_classes_, dtype=np.intp)
        else:
            n_classes = np.ones(self.n_outputs_, dtype=np.intp)
        weights = None
        if self.bootstrap:
            weights = np.empty((len(trees), n))
            for j, s in enumerate(tree_seeds):
                w = np.ones(n) if sample_weight is None else sample_weight.copy()
                idx = _generate_sample_indices(s, n, n_boot)
                w *= np.bincount(idx, minlength=n)
                cw = getattr(self, "class_weight", None)
                if cw == "subsample":
                    w *= compute_sample_weight("balanced", y, indices=idx)
                elif cw == "balanced_subsample":
                    w *= compute_sample_weight("balanced", y, indices=idx)
                weights[j] = w
        elif sample_weight is not None:
            weights = np.tile(sample_weight, (len(trees), 1))
        if weights is not None:
            params["min_weight_leaf"] = None
            mwl = np.array([self.min_weight_fraction_leaf * w.sum() for w in weights])
        split_seeds = [check_random_state(s).randint(0, RAND_R_MAX) for s in tree_seeds]
        n_threads = 0 if self.n_jobs in (None, -1) else max(1, int(self.n_jobs))
        if weights is not None and np.any(mwl != mwl[0]):
            # per-tree leaf-weight floors: one native build per tree, fanned
            # out over the task layer (reference ``_forest.py:396``
            # ``Parallel(n_jobs, prefer="threads")``; the ctypes build releases
            # the GIL, so worker threads run the trees concurrently)
            from ...parallel.tasks import Parallel
            from ...utils.fixes import delayed

            def one(j):
                pj = dict(params, min_weight_leaf=mwl[j])
                return build_trees(X, y, weights[j:j + 1], n_classes, pj, split_seeds[j:j + 1],
                                   n_threads=1)[0]

            fitted = Parallel(n_jobs=self.n_jobs)(delayed(one)(j) for j in range(len(trees)))
        else:
            if weights is not None:
                params["min_weight_leaf"] = float(mwl[0])
            fitted = build_trees(X, y, weights, n_classes, params, split_seeds,
                                 n_threads=n_threads)
        for t, tr in zip(trees, fitted):
            t.tree_ = tr
            t.n_features_in_ = X.shape[1]
            t.n_outputs_ = self.n_outputs_
            t.max_features_ = params["max_features"]
            if isinstance(self, ClassifierMixin):
                if self.n_outputs_ == 1:
                    t.classes_ = np.arange(n_classes[0]).astype(np.float64)
                    t.n_classes_ = int(n_classes[0])
                else:
                    t.classes_ = [np.arange(c).astype(np.float64) for c in n_classes]
                    t.n_classes_ = n_classes.copy()
            t._prune_tree()
        self.estimators_.extend(trees)

    # ------------------------------------------------------------- queries
    def apply(self, X):
        check_is_fitted(self)
        X = self._validate_X_predict(X)
        return forest_apply([e.tree_ for e in self.estimators_], X)

    def decision_path(self, X):
        X = self._validate_X_predict(X)
        inds = [e.decision_path(X) for e in self.estimators_]
        n_nodes = [0] + [i.shape[1] for i in inds]
        return sp.hstack(inds).tocsr(), np.array(n_nodes).cumsum()

    def _validate_X_predict(self, X):
        check_is_fitted(self)
        if isinstance(X, torch.Tensor) and X.is_cuda:
            Xp = X.float().contiguous()
        else:
            Xp = _as_f32(X)
        if Xp.shape[1] != self.n_features_in_:
            raise ValueError(f"X has {Xp.shape[1]} features, but {self.__class__.__name__} is "
                             f"expecting {self.n_features_in_} features as input.")
        return Xp

    @property
    def feature_importances_(self):
        check_is_fitted(self)
        imps = [t.feature_importances_ for t in self.estimators_ if t.tree_.node_count > 1]
        if not imps:
            return np.zeros(self.n_features_in_, dtype=np.float64)
        m = np.mean(imps, axis=0, dtype=np.float64)
        return m / np.sum(m)

    def __len__(self):
        return len(self.estimators_)

    def __getitem__(self, i):
        return self.estimators_[i]

    def __iter__(self):
        return iter(self.estimators_)

    def _sum_leaf_values(self, X, normalize):
        """(n, n_outputs * S) sum over trees of (optionally per-output
        normalised) leaf values; device kernel for GPU rows."""
        trees = [e.tree_ for e in self.estimators_]
        if isinstance(X, torch.Tensor) and X.is_cuda:
            if getattr(self, "_device_tables", None) is None or \
                    self._device_tables.device != X.device:
                from ...ops.forest import ForestTables
                left, right, feat, thr, offs = stack_trees(trees)
                vals = np.concatenate([self._leaf_values(t, normalize) for t in trees])
                self._device_tables = ForestTables(left, right, feat, thr, offs, vals, X.device)
            return self._device_tables.predict_sum(X).cpu().numpy()
        leaves = forest_apply(trees, X)
        acc = None
        for j, t in enumerate(trees):
            v = self._leaf_values(t, normalize)[leaves[:, j]]
            acc = v if acc is None else acc + v
        return acc

    @staticmethod
    def _leaf_values(tree, normalize):
        v = tree.value
        if normalize:
            s = v.sum(axis=2, keepdims=True)
            s[s == 0.0] = 1.0
            v = v / s
        return v.reshape(v.shape[0], -1)


class ForestClassifier(ClassifierMixin, BaseForest):
    def _validate_y_class_weight(self, y):
        y = np.copy(y)
        expanded = None
        if self.class_weight is not None:
            y_original = np.copy(y)
        self.classes_, self.n_classes_ = [], []
        enc = np.zeros(y.shape, dtype=int)
        for k in range(self.n_outputs_):
            cls, enc[:, k] = np.unique(y[:, k], return_inverse=True)
            self.classes_.append(cls)
            self.n_classes_.append(cls.shape[0])
        y = enc
        if self.class_weight is not None:
            presets = ("balanced", "balanced_subsample")
            if isinstance(self.class_weight, str):
                if self.class_weight not in presets:
                    raise ValueError('Valid presets for class_weight include "balanced" and '
                                     '"balanced_subsample".Given "%s".' % self.class_weight)
                if self.warm_start:
                    warnings.warn('class_weight presets "balanced" or "balanced_subsample" are '
                                  'not recommended for warm_start if the fitted data differs '
                                  'from the full dataset.')
            if self.class_weight != "balanced_subsample" or not self.bootstrap:
                cw = "balanced" if self.class_weight == "balanced_subsample" else self.class_weight
                expanded = compute_sample_weight(cw, y_original)
        return y, expanded

    def predict_proba(self, X):
        X = self._validate_X_predict(X)
        T = len(self.estimators_)
        acc = self._sum_leaf_values(X, normalize=True) / T
        if self.n_outputs_ == 1:
            return acc[:, :self.n_classes_]
        S = acc.shape[1] // self.n_outputs_
        return [acc[:, k * S:k * S + self.n_classes_[k]] for k in range(self.n_outputs_)]

    def predict_log_proba(self, X):
        p = self.predict_proba(X)
        return np.log(p) if self.n_outputs_ == 1 else [np.log(q) for q in p]

    def predict(self, X):
        proba = self.predict_proba(X)
        if self.n_outputs_ == 1:
            return self.classes_.take(np.argmax(proba, axis=1), axis=0)
        n = proba[0].shape[0]
        out = np.empty((n, self.n_outputs_), dtype=self.classes_[0].dtype)
        for k in range(self.n_outputs_):
            out[:, k] = self.classes_[k].take(np.argmax(proba[k], axis=1), axis=0)
        return out

    def _set_oob_score_and_attributes(self, X, y):
        n = y.shape[0]
        ncls = np.atleast_1d(self.n_classes_)
        oob = np.zeros((n, ncls[0], self.n_outputs_))
        cnt = np.zeros((n, self.n_outputs_), dtype=np.int64)
        nb = _get_n_samples_bootstrap(n, self.max_samples)
        for e in self.estimators_:
            un = _generate_unsampled_indices(e.random_state, n, nb)
            p = e.predict_proba(X[un])
            if self.n_outputs_ == 1:
                p = p[..., None]
            else:
                p = np.stack(p, axis=2)
            oob[un] += p
            cnt[un] += 1
        if (cnt == 0).any():
            warnings.warn("Some inputs do not have OOB scores. This probably means too few "
                          "trees were used to compute any reliable OOB estimates.", UserWarning)
            cnt[cnt == 0] = 1
        oob /= cnt[:, None, :]
        if oob.shape[-1] == 1:
            oob = oob[..., 0]
        self.oob_decision_function_ = oob
        pred = np.argmax(oob, axis=1)
        yy = y if y.ndim == 2 and y.shape[1] > 1 else y.reshape(-1)
        self.oob_score_ = float(np.mean(np.all(pred.reshape(yy.shape) == yy, axis=-1)
                                        if yy.ndim == 2 else pred == yy))


class ForestRegressor(RegressorMixin, BaseForest):
    def predict(self, X):
        X = self._validate_X_predict(X)
        acc = self._sum_leaf_values(X, normalize=False) / len(self.estimators_)
        return acc[:, 0] if self.n_outputs_ == 1 else acc

    def _set_oob_score_and_attributes(self, X, y):
        n = y.shape[0]
        oob = np.zeros((n, self.n_outputs_))
        cnt = np.zeros((n, self.n_outputs_), dtype=np.int64)
        nb = _get_n_samples_bootstrap(n, self.max_samples)
        for e in self.estimators_:
            un = _generate_unsampled_indices(e.random_state, n, nb)
            p = e.predict(X[un])
            oob[un] += p.reshape(len(un), -1)
            cnt[un] += 1
        if (cnt == 0).any():
            warnings.warn("Some inputs do not have OOB scores. This probably means too few "
                          "trees were used to compute any reliable OOB estimates.", UserWarning)
            cnt[cnt == 0] = 1
        oob /= cnt
        self.oob_prediction_ = oob[:, 0] if self.n_outputs_ == 1 else oob
        from ...utils.metrics import r2_score
        self.oob_score_ = r2_score(y, self.oob_prediction_)


def _forest_init(self, n_estimators, criterion, max_depth, min_samples_split, min_samples_leaf,
                 min_weight_fraction_leaf, max_features, max_leaf_nodes, min_impurity_decrease,
                 bootstrap, oob_score, n_jobs, random_state, verbose, warm_start, ccp_alpha,
                 max_samples):
    self.n_estimators = n_estimators
    self.criterion = criterion
    self.max_depth = max_depth
    self.min_samples_split = min_samples_split
    self.min_samples_leaf = min_samples_leaf
    self.min_weight_fraction_leaf = min_weight_fraction_leaf
    self.max_features = max_features
    self.max_leaf_nodes = max_leaf_nodes
    self.min_impurity_decrease = min_impurity_decrease
    self.bootstrap = bootstrap
    self.oob_score = oob_score
    self.n_jobs = n_jobs
    self.random_state = random_state
    self.verbose = verbose
    self.warm_start = warm_start
    self.ccp_alpha = ccp_alpha
    self.max_samples = max_samples


class RandomForestClassifier(ForestClassifier):
    """Bootstrap-aggregated CART classifiers with feature subsampling."""
    _tree_cls = DecisionTreeClassifier

    def __init__(self, n_estimators=100, *, criterion="gini", max_depth=None,
                 min_samples_split=2, min_samples_leaf=1, min_weight_fraction_leaf=0.0,
                 max_features="auto", max_leaf_nodes=None, min_impurity_decrease=0.0,
                 bootstrap=True, oob_score=False, n_jobs=None, random_state=None, verbose=0,
                 warm_start=False, class_weight=None, ccp_alpha=0.0, max_samples=None):
        _forest_init(self, n_estimators, criterion, max_depth, min_samples_split,
                     min_samples_leaf, min_weight_fraction_leaf, max_features, max_leaf_nodes,
                     min_impurity_decrease, bootstrap, oob_score, n_jobs, random_state, verbose,
                     warm_start, ccp_alpha, max_samples)
        self.class_weight = class_weight


class RandomForestRegressor(ForestRegressor):
    """Bootstrap-aggregated CART regressors."""
    _tree_cls = DecisionTreeRegressor

    def __init__(self, n_estimators=100, *, criterion="squared_error", max_depth=None,
                 min_samples_split=2, min_samples_leaf=1, min_weight_fraction_leaf=0.0,
                 max_features="auto", max_leaf_nodes=None, min_impurity_decrease=0.0,
                 bootstrap=True, oob_score=False, n_jobs=None, random_state=None, verbose=0,
                 warm_start=False, ccp_alpha=0.0, max_samples=None):
        _forest_init(self, n_estimators, criterion, max_depth, min_samples_split,
                     min_samples_leaf, min_weight_fraction_leaf, max_features, max_leaf_nodes,
                     min_impurity_decrease, bootstrap, oob_score, n_jobs, random_state, verbose,
                     warm_start, ccp_alpha, max_samples)


class ExtraTreesClassifier(ForestClassifier):
    """Extremely randomized trees (random thresholds, no bootstrap by default)."""
    _tree_cls = ExtraTreeClassifier

    def __init__(self, n_estimators=100, *, criterion="gini", max_depth=None,
                 min_samples_split=2, min_samples_leaf=1, min_weight_fraction_leaf=0.0,
                 max_features="auto", max_leaf_nodes=None, min_impurity_decrease=0.0,
                 bootstrap=False, oob_score=False, n_jobs=None, random_state=None, verbose=0,
                 warm_start=False, class_weight=None, ccp_alpha=0.0, max_samples=None):
        _forest_init(self, n_estimators, criterion, max_depth, min_samples_split,
                     min_samples_leaf, min_weight_fraction_leaf, max_features, max_leaf_nodes,
                     min_impurity_decrease, bootstrap, oob_score, n_jobs, random_state, verbose,
                     warm_start, ccp_alpha, max_samples)
        self.class_weight = class_weight


class ExtraTreesRegressor(ForestRegressor):
    """Extremely randomized regression trees."""
    _tree_cls = ExtraTreeRegressor

    def __init__(self, n_estimators=100, *, criterion="squared_error", max_depth=None,
                 min_samples_split=2, min_samples_leaf=1, min_weight_fraction_leaf=0.0,
                 max_features="auto", max_leaf_nodes=None, min_impurity_decrease=0.0,
                 bootstrap=False, oob_score=False, n_jobs=None, random_state=None, verbose=0,
                 warm_start=False, ccp_alpha=0.0, max_samples=None):
        _forest_init(self, n_estimators, criterion, max_depth, min_samples_split,
                     min_samples_leaf, min_weight_fraction_leaf, max_features, max_leaf_nodes,
                     min_impurity_decrease, bootstrap, oob_score, n_jobs, random_state, verbose,
                     warm_start, ccp_alpha, max_samples)


class RandomTreesEmbedding(TransformerMixin, BaseForest):
    """Unsupervised one-hot leaf encoding by totally random trees
    (reference ``_forest.py: RandomTreesEmbedding``)."""
    _tree_cls = ExtraTreeRegressor
    criterion = "squared_error"
    max_features = 1

    def __init__(self, n_estimators=100, *, max_depth=5, min_samples_split=2,
                 min_samples_leaf=1, min_weight_fraction_leaf=0.0, max_leaf_nodes=None,
                 min_impurity_decrease=0.0, sparse_output=True, n_jobs=None, random_state=None,
                 verbose=0, warm_start=False):
        self.n_estimators = n_estimators
        self.max_depth = max_depth
        self.min_samples_split = min_samples_split
        self.min_samples_leaf = min_samples_leaf
        self.min_weight_fraction_leaf = min_weight_fraction_leaf
        self.max_leaf_nodes = max_leaf_nodes
        self.min_impurity_decrease = min_impurity_decrease
        self.sparse_output = sparse_output
        self.n_jobs = n_jobs
        self.random_state = random_state
        self.verbose = verbose
        self.warm_start = warm_start

    bootstrap = False
    oob_score = False
    max_samples = None
    ccp_alpha = 0.0

    def fit(self, X, y=None, sample_weight=None):
        self.fit_transform(X, y, sample_weight=sample_weight)
        return self

    def fit_transform(self, X, y=None, sample_weight=None):
        X = _as_f32(X)
        rnd = check_random_state(self.random_state)
        y = rnd.uniform(size=X.shape[0])
        BaseForest.fit(self, X, y, sample_weight=sample_weight)
        from ...preprocessing import OneHotEncoder
        self.one_hot_encoder_ = OneHotEncoder(sparse=self.sparse_output)
        return self.one_hot_encoder_.fit_transform(self.apply(X))

    def transform(self, X):
        check_is_fitted(self)
        return self.one_hot_encoder_.transform(self.apply(X))


__all__ = ["RandomForestClassifier", "RandomForestRegressor", "ExtraTreesClassifier",
           "ExtraTreesRegressor", "RandomTreesEmbedding"]
