"""Histogram-based gradient boosting (reference
``ensemble/_hist_gradient_boosting``: ``binning.py`` quantile bin mapper
:20-262, ``loss.py`` losses :147-427, ``gradient_boosting.py``
BaseHistGradientBoosting.fit :177-539 with early stopping, ``grower.py``,
``predictor.py``; estimators HistGradientBoostingRegressor /
HistGradientBoostingClassifier).

Binning and tree growth run host-native (``csrc/host/hgb.cpp``: OpenMP
histograms with the subtraction trick, the reference's split scans and
heap); gradients / hessians and raw-prediction updates are vectorised numpy
on the reference's float32 / float64 dtypes.
"""

import ctypes
import warnings

import numpy as np
from scipy.special import expit, logsumexp, xlogy

from ...base import BaseEstimator, ClassifierMixin, RegressorMixin, is_classifier
from ...ops import _host
from ...utils.stats import _weighted_percentile
from ...utils.validation import check_is_fitted, check_random_state

X_DTYPE = np.float64
G_H_DTYPE = np.float32
ALMOST_INF = 1e300


# ------------------------------------------------------------------ binning
def _find_binning_thresholds(col, max_bins):
    col = col[~np.isnan(col)]
    col = np.ascontiguousarray(col, dtype=X_DTYPE)
    distinct = np.unique(col)
    if len(distinct) <= max_bins:
        mids = distinct[:-1] + distinct[1:]
        mids *= 0.5
    else:
        pct = np.linspace(0, 100, num=max_bins + 1)[1:-1]
        mids = np.percentile(col, pct, method="midpoint").astype(X_DTYPE)
    np.clip(mids, a_min=None, a_max=ALMOST_INF, out=mids)
    return mids


class _BinMapper:
    """Quantile bin mapper; the last bin (n_bins - 1) holds missing values."""

    def __init__(self, n_bins=256, subsample=int(2e5), is_categorical=None,
                 known_categories=None, random_state=None):
        self.n_bins = n_bins
        self.subsample = subsample
        self.is_categorical = is_categorical
        self.known_categories = known_categories
        self.random_state = random_state

    def fit(self, X):
        if not 3 <= self.n_bins <= 256:
            raise ValueError("n_bins={} should be no smaller than 3 and no larger than 256."
                             .format(self.n_bins))
        max_bins = self.n_bins - 1
        rng = check_random_state(self.random_state)
        if self.subsample is not None and X.shape[0] > self.subsample:
            X = X.take(rng.choice(X.shape[0], self.subsample, replace=False), axis=0)
        self.missing_values_bin_idx_ = self.n_bins - 1
        # numpy's partition / unique release the GIL: features in parallel threads
        from concurrent.futures import ThreadPoolExecutor
        import os
        with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
            self.bin_thresholds_ = list(ex.map(lambda f: _find_binning_thresholds(X[:, f],
                                                                                  max_bins),
                                               range(X.shape[1])))
        self.n_bins_non_missing_ = np.array([t.shape[0] + 1 for t in self.bin_thresholds_],
                                            dtype=np.uint32)
        if self.is_categorical is not None:
            # categorical: the "thresholds" are the sorted categories, so a
            # known category maps to its rank
            for f in np.flatnonzero(self.is_categorical):
                cats = np.asarray(self.known_categories[f], dtype=X_DTYPE)
                self.bin_thresholds_[f] = cats
                self.n_bins_non_missing_[f] = cats.shape[0]
        self.is_categorical_ = (np.zeros(X.shape[1], dtype=np.uint8) if self.is_categorical
                                is None else np.asarray(self.is_categorical, dtype=np.uint8))
        return self

    def transform(self, X):
        X = np.ascontiguousarray(X, dtype=X_DTYPE)
        n, d = X.shape
        if d != self.n_bins_non_missing_.shape[0]:
            raise ValueError("This estimator was fitted with {} features but {} got passed to "
                             "transform()".format(self.n_bins_non_missing_.shape[0], d))
        thr = np.ascontiguousarray(np.concatenate(self.bin_thresholds_) if d else np.zeros(0),
                                   dtype=np.float64)
        offs = np.zeros(d + 1, dtype=np.int64)
        offs[1:] = np.cumsum([len(t) for t in self.bin_thresholds_])
        out = np.empty((d, n), dtype=np.uint8)
        _host.lib().sqh_hgb_map_bins(X.ctypes.data, n, d, thr.ctypes.data, offs.ctypes.data,
                                     int(self.missing_values_bin_idx_), out.ctypes.data)
        return out.T          # Fortran-ordered (n, d) view

    def fit_transform(self, X):
        return self.fit(X).transform(X)


# ------------------------------------------------------------------- losses
class BaseLoss:
    need_update_leaves_values = False

    def __init__(self, hessians_are_constant):
        self.hessians_are_constant = hessians_are_constant

    def __call__(self, y_true, raw, sample_weight):
        return np.average(self.pointwise_loss(y_true, raw), weights=sample_weight)

    def init_gradients_and_hessians(self, n_samples, prediction_dim, sample_weight):
        shape = (prediction_dim, n_samples)
        g = np.empty(shape, dtype=G_H_DTYPE)
        if self.hessians_are_constant:
            h = np.ones((1, 1), dtype=G_H_DTYPE)
        else:
            h = np.empty(shape, dtype=G_H_DTYPE)
        return g, h


class LeastSquares(BaseLoss):
    def __init__(self, sample_weight):
        super().__init__(hessians_are_constant=sample_weight is None)

    def pointwise_loss(self, y, raw):
        return 0.5 * np.power(y - raw.reshape(-1), 2)

    def get_baseline_prediction(self, y, sw, dim):
        return np.average(y, weights=sw)

    @staticmethod
    def inverse_link_function(raw):
        return raw

    def update_gradients_and_hessians(self, g, h, y, raw, sw):
        raw = raw.reshape(-1)
        if sw is None:
            g.reshape(-1)[:] = raw - y
        else:
            g.reshape(-1)[:] = (raw - y) * sw
            h.reshape(-1)[:] = sw


class LeastAbsoluteDeviation(BaseLoss):
    need_update_leaves_values = True

    def __init__(self, sample_weight):
        super().__init__(hessians_are_constant=sample_weight is None)

    def pointwise_loss(self, y, raw):
        return np.abs(y - raw.reshape(-1))

    def get_baseline_prediction(self, y, sw, dim):
        return np.median(y) if sw is None else _weighted_percentile(y, sw, 50)

    @staticmethod
    def inverse_link_function(raw):
        return raw

    def update_gradients_and_hessians(self, g, h, y, raw, sw):
        raw = raw.reshape(-1)
        s = 2 * (y - raw < 0) - 1
        if sw is None:
            g.reshape(-1)[:] = s
        else:
            g.reshape(-1)[:] = sw * s
            h.reshape(-1)[:] = sw

    def update_leaves_values(self, nodes, leaf_of_sample, y, raw, sw, shrinkage):
        leaves = np.where(nodes["is_leaf"])[0]
        order = np.argsort(leaf_of_sample, kind="stable")
        srt = leaf_of_sample[order]
        for leaf in leaves:
            s, e = np.searchsorted(srt, leaf), np.searchsorted(srt, leaf, side="right")
            idx = order[s:e]
            diff = y[idx] - raw[idx]
            med = np.median(diff) if sw is None else _weighted_percentile(diff, sw[idx], 50)
            nodes["value"][leaf] = shrinkage * med


class Poisson(BaseLoss):
    inverse_link_function = staticmethod(np.exp)

    def __init__(self, sample_weight):
        super().__init__(hessians_are_constant=False)

    def pointwise_loss(self, y, raw):
        raw = raw.reshape(-1)
        return xlogy(y, y) - y * (raw + 1) + np.exp(raw)

    def get_baseline_prediction(self, y, sw, dim):
        p = np.average(y, weights=sw)
        return np.log(np.clip(p, np.finfo(y.dtype).eps, None))

    def update_gradients_and_hessians(self, g, h, y, raw, sw):
        yp = np.exp(raw.reshape(-1))
        w = 1.0 if sw is None else sw
        g.reshape(-1)[:] = (yp - y) * w
        h.reshape(-1)[:] = yp * w


class BinaryCrossEntropy(BaseLoss):
    inverse_link_function = staticmethod(expit)

    def __init__(self, sample_weight):
        super().__init__(hessians_are_constant=False)

    def pointwise_loss(self, y, raw):
        raw = raw.reshape(-1)
        return np.logaddexp(0, raw) - y * raw

    def get_baseline_prediction(self, y, sw, dim):
        if dim > 2:
            raise ValueError("loss='binary_crossentropy' is not defined for multiclass "
                             "classification with n_classes=%d, use "
                             "loss='categorical_crossentropy' instead" % dim)
        p = np.clip(np.average(y, weights=sw), np.finfo(y.dtype).eps, 1 - np.finfo(y.dtype).eps)
        return np.log(p / (1 - p))

    def update_gradients_and_hessians(self, g, h, y, raw, sw):
        p = 1.0 / (1.0 + np.exp(-raw.reshape(-1)))
        w = 1.0 if sw is None else sw
        g.reshape(-1)[:] = (p - y) * w
        h.reshape(-1)[:] = p * (1.0 - p) * w

    def predict_proba(self, raw):
        raw = raw.reshape(-1)
        p = np.empty((raw.shape[0], 2))
        p[:, 1] = expit(raw)
        p[:, 0] = 1 - p[:, 1]
        return p


class CategoricalCrossEntropy(BaseLoss):
    def __init__(self, sample_weight):
        super().__init__(hessians_are_constant=False)

    def pointwise_loss(self, y, raw):
        one_hot = np.zeros_like(raw)
        for k in range(raw.shape[0]):
            one_hot[k, :] = y == k
        return logsumexp(raw, axis=0) - (one_hot * raw).sum(axis=0)

    def get_baseline_prediction(self, y, sw, dim):
        init = np.zeros((dim, 1))
        eps = np.finfo(y.dtype).eps
        for k in range(dim):
            init[k, :] += np.log(np.clip(np.average(y == k, weights=sw), eps, 1 - eps))
        return init

    def update_gradients_and_hessians(self, g, h, y, raw, sw):
        p = np.exp(raw - raw.max(axis=0, keepdims=True))
        p /= p.sum(axis=0, keepdims=True)
        w = 1.0 if sw is None else sw
        for k in range(raw.shape[0]):
            g[k] = (p[k] - (y == k)) * w
            h[k] = p[k] * (1.0 - p[k]) * w

    def predict_proba(self, raw):
        return np.exp(raw - logsumexp(raw, axis=0)[None, :]).T


_LOSSES = {"squared_error": LeastSquares, "least_squares": LeastSquares,
           "absolute_error": LeastAbsoluteDeviation,
           "least_absolute_deviation": LeastAbsoluteDeviation, "poisson": Poisson,
           "binary_crossentropy": BinaryCrossEntropy,
           "categorical_crossentropy": CategoricalCrossEntropy}

_NODE_FIELDS = [("value", np.float64), ("gain", np.float64), ("count", np.int32),
                ("feature_idx", np.int32), ("bin_threshold", np.int32), ("left", np.int32),
                ("right", np.int32), ("depth", np.int32), ("missing_go_to_left", np.uint8),
                ("is_leaf", np.uint8)]


class TreePredictor:
    """Predictor nodes of one fitted tree (reference ``predictor.py``)."""

    def __init__(self, nodes):
        self.nodes = nodes

    def get_n_leaf_nodes(self):
        return int(self.nodes["is_leaf"].sum())

    def get_max_depth(self):
        return int(self.nodes["depth"].max())


def _grow_tree(Xb, g, h, hess_const, nbnm, has_missing, mono, params, shrinkage, is_cat):
    lib = _host.lib()
    n, d = Xb.shape
    prm = np.array([params["max_leaf_nodes"], params["max_depth"], params["min_samples_leaf"],
                    0.0, params["l2_regularization"], 1e-3, shrinkage, params["n_bins"]],
                   dtype=np.float64)
    g = np.ascontiguousarray(g, dtype=np.float32)
    h = np.ascontiguousarray(h, dtype=np.float32).reshape(-1)
    handle = lib.sqh_hgb_grow(Xb.T.ctypes.data, n, d, g.ctypes.data, h.ctypes.data,
                              int(hess_const), nbnm.ctypes.data, has_missing.ctypes.data,
                              mono.ctypes.data, prm.ctypes.data, is_cat.ctypes.data)
    m = lib.sqh_hgb_size(handle)
    nodes = {name: np.empty(m, dtype=dt) for name, dt in _NODE_FIELDS}
    leaf_of_sample = np.empty(n, dtype=np.int32)
    lib.sqh_hgb_copy(handle, *(nodes[f].ctypes.data for f, _ in _NODE_FIELDS),
                     leaf_of_sample.ctypes.data, n)
    nodes["is_categorical"] = np.empty(m, dtype=np.uint8)
    nodes["left_cat_bitset"] = np.empty((m, 8), dtype=np.uint32)
    lib.sqh_hgb_copy_cat(handle, nodes["is_categorical"].ctypes.data,
                         nodes["left_cat_bitset"].ctypes.data)
    lib.sqh_hgb_free(handle)
    return nodes, leaf_of_sample


class BaseHistGradientBoosting(BaseEstimator):
    def _validate_parameters(self):
        if self.loss not in self._VALID_LOSSES and not isinstance(self.loss, BaseLoss):
            raise ValueError("Loss {} is not supported for {}. Accepted losses: {}."
                             .format(self.loss, self.__class__.__name__,
                                     ", ".join(self._VALID_LOSSES)))
        if self.learning_rate <= 0:
            raise ValueError("learning_rate={} must be strictly positive"
                             .format(self.learning_rate))
        if self.max_iter < 1:
            raise ValueError("max_iter={} must not be smaller than 1.".format(self.max_iter))
        if self.n_iter_no_change < 0:
            raise ValueError("n_iter_no_change={} must be positive."
                             .format(self.n_iter_no_change))
        if self.validation_fraction is not None and self.validation_fraction <= 0:
            raise ValueError("validation_fraction={} must be strictly positive, or None."
                             .format(self.validation_fraction))
        if self.tol < 0:
            raise ValueError("tol={} must not be smaller than 0.".format(self.tol))
        if not 2 <= self.max_bins <= 255:
            raise ValueError("max_bins={} should be no smaller than 2 and no larger than 255."
                             .format(self.max_bins))
        if self.max_leaf_nodes is not None and self.max_leaf_nodes <= 1:
            raise ValueError("max_leaf_nodes={} should not be smaller than 2"
                             .format(self.max_leaf_nodes))
        if self.max_depth is not None and self.max_depth < 1:
            raise ValueError("max_depth={} should not be smaller than 1".format(self.max_depth))
        if self.min_samples_leaf < 1:
            raise ValueError("min_samples_leaf={} should not be smaller than 1"
                             .format(self.min_samples_leaf))
        if self.l2_regularization < 0:
            raise ValueError("l2_regularization={} must be positive."
                             .format(self.l2_regularization))
        if self.monotonic_cst is not None and self.n_trees_per_iteration_ != 1:
            raise ValueError("monotonic constraints are not supported for multiclass "
                             "classification.")

    def _check_categories(self, X):
        """(is_categorical, known_categories) of X (reference
        ``gradient_boosting.py`` ``_check_categories``)."""
        cf = getattr(self, "categorical_features", None)
        if cf is None:
            return None, None
        cf = np.asarray(cf)
        if cf.size == 0:
            return None, None
        if cf.dtype.kind not in ("i", "b"):
            raise ValueError("categorical_features must be an array-like of bools or array-like "
                             "of ints.")
        d = X.shape[1]
        if cf.dtype.kind == "i":
            if np.max(cf) >= d or np.min(cf) < 0:
                raise ValueError("categorical_features set as integer indices must be in "
                                 "[0, n_features - 1]")
            is_cat = np.zeros(d, dtype=bool)
            is_cat[cf] = True
        else:
            if cf.shape[0] != d:
                raise ValueError("categorical_features set as a boolean mask must have shape "
                                 f"(n_features,), got: {cf.shape}")
            is_cat = cf
        if not np.any(is_cat):
            return None, None
        known = []
        for f in range(d):
            if not is_cat[f]:
                known.append(None)
                continue
            cats = np.unique(X[:, f])
            cats = cats[~np.isnan(cats)]
            if cats.size > self.max_bins:
                raise ValueError(f"Categorical feature at index {f} is expected to have a "
                                 f"cardinality <= {self.max_bins}")
            if (cats >= self.max_bins).any():
                raise ValueError(f"Categorical feature at index {f} is expected to be encoded "
                                 f"with values < {self.max_bins}")
            known.append(cats)
        return is_cat, known

    def fit(self, X, y, sample_weight=None):
        X = np.asarray(X.detach().cpu().numpy() if hasattr(X, "detach") else X, dtype=X_DTYPE)
        if X.ndim != 2:
            raise ValueError("Expected 2D array")
        if np.isinf(X).any():
            raise ValueError("Input contains infinity or a value too large for dtype('float64').")
        y = self._encode_y(np.asarray(y).reshape(-1))
        if sample_weight is not None:
            sample_weight = np.asarray(sample_weight, dtype=np.float64).reshape(-1)
        rng = check_random_state(self.random_state)
        if not (self.warm_start and self._is_fitted()):
            self._random_seed = rng.randint(np.iinfo(np.uint32).max, dtype="u8")
        self._validate_parameters()
        n_samples, self._n_features = X.shape
        self.n_features_in_ = self._n_features
        self.is_categorical_, known_categories = self._check_categories(X)
        if self.is_categorical_ is not None and self.monotonic_cst is not None and np.any(
                np.asarray(self.monotonic_cst)[self.is_categorical_] != 0):
            raise ValueError("Categorical features cannot have monotonic constraints.")
        self._loss = self._get_loss(sample_weight) if isinstance(self.loss, str) else self.loss
        self.do_early_stopping_ = (n_samples > 10000 if self.early_stopping == "auto"
                                   else bool(self.early_stopping))
        self._use_validation_data = self.validation_fraction is not None
        if self.do_early_stopping_ and self._use_validation_data:
            from ...model_selection import train_test_split
            strat = y if hasattr(self._loss, "predict_proba") else None
            if sample_weight is None:
                X_tr, X_val, y_tr, y_val = train_test_split(
                    X, y, test_size=self.validation_fraction, stratify=strat,
                    random_state=self._random_seed)
                sw_tr = sw_val = None
            else:
                X_tr, X_val, y_tr, y_val, sw_tr, sw_val = train_test_split(
                    X, y, sample_weight, test_size=self.validation_fraction, stratify=strat,
                    random_state=self._random_seed)
        else:
            X_tr, y_tr, sw_tr = X, y, sample_weight
            X_val = y_val = sw_val = None
        n_bins = self.max_bins + 1
        if not (self.warm_start and self._is_fitted()):
            self._bin_mapper = _BinMapper(n_bins=n_bins, is_categorical=self.is_categorical_,
                                          known_categories=known_categories,
                                          random_state=self._random_seed)
            Xb = self._bin_mapper.fit_transform(X_tr)
        else:
            Xb = self._bin_mapper.transform(X_tr)
        has_missing = (Xb == self._bin_mapper.missing_values_bin_idx_).any(axis=0).astype(np.uint8)
        n = Xb.shape[0]
        K = self.n_trees_per_iteration_
        if not (self._is_fitted() and self.warm_start):
            self._baseline_prediction = self._loss.get_baseline_prediction(y_tr, sw_tr, K)
            raw = np.zeros((K, n)) + self._baseline_prediction
            self._predictors = []
            self.train_score_, self.validation_score_ = [], []
            raw_val = None
            if self.do_early_stopping_:
                if self.scoring == "loss":
                    if self._use_validation_data:
                        raw_val = np.zeros((K, X_val.shape[0])) + self._baseline_prediction
                    self._check_early_stopping_loss(raw, y_tr, sw_tr, raw_val, y_val, sw_val)
                else:
                    self._check_early_stopping_scorer(X_tr, y_tr, sw_tr, X_val, y_val, sw_val)
            begin = 0
        else:
            if self.max_iter < self.n_iter_:
                raise ValueError("max_iter=%d must be larger than or equal to n_iter_=%d when "
                                 "warm_start==True" % (self.max_iter, self.n_iter_))
            self.train_score_ = list(self.train_score_)
            self.validation_score_ = list(self.validation_score_)
            raw = self._raw_predict(X_tr).reshape(K, n)
            raw_val = (self._raw_predict(X_val).reshape(K, -1)
                       if self.do_early_stopping_ and self._use_validation_data else None)
            begin = self.n_iter_
        g, h = self._loss.init_gradients_and_hessians(n, K, sw_tr)
        mono = (np.zeros(self._n_features, dtype=np.int8) if self.monotonic_cst is None
                else np.asarray(self.monotonic_cst, dtype=np.int8))
        if mono.shape[0] != self._n_features:
            raise ValueError("monotonic_cst has shape {} but the input data X has {} features."
                             .format(mono.shape[0], self._n_features))
        params = dict(max_leaf_nodes=self.max_leaf_nodes or 0, max_depth=self.max_depth or 0,
                      min_samples_leaf=self.min_samples_leaf,
                      l2_regularization=self.l2_regularization, n_bins=n_bins)
        nbnm = np.ascontiguousarray(self._bin_mapper.n_bins_non_missing_, dtype=np.uint32)
        is_cat = np.ascontiguousarray(self._bin_mapper.is_categorical_, dtype=np.uint8)
        self._known_cat_bitsets = np.zeros((self._n_features, 8), dtype=np.uint32)
        for f in np.flatnonzero(is_cat):
            for c in self._bin_mapper.bin_thresholds_[f].astype(int):
                self._known_cat_bitsets[f, c >> 5] |= np.uint32(1 << (c & 31))
        for it in range(begin, self.max_iter):
            self._loss.update_gradients_and_hessians(g, h, y_tr, raw, sw_tr)
            self._predictors.append([])
            for k in range(K):
                hk = h[0] if self._loss.hessians_are_constant else h[k]
                nodes, leaf_of = _grow_tree(Xb, g[k], hk, self._loss.hessians_are_constant,
                                            nbnm, has_missing, mono, params, self.learning_rate,
                                            is_cat)
                if self._loss.need_update_leaves_values:
                    self._loss.update_leaves_values(nodes, leaf_of, y_tr, raw[k], sw_tr,
                                                    self.learning_rate)
                self._finalize_thresholds(nodes)
                pred = TreePredictor(nodes)
                pred.known_cat_bitsets = self._known_cat_bitsets
                self._predictors[-1].append(pred)
                raw[k] += nodes["value"][leaf_of]
            stop = False
            if self.do_early_stopping_:
                if self.scoring == "loss":
                    if self._use_validation_data:
                        for k, p in enumerate(self._predictors[-1]):
                            raw_val[k] += _predict_trees([p], X_val)
                    stop = self._check_early_stopping_loss(raw, y_tr, sw_tr, raw_val, y_val,
                                                           sw_val)
                else:
                    stop = self._check_early_stopping_scorer(X_tr, y_tr, sw_tr, X_val, y_val,
                                                             sw_val)
            if self.verbose:
                print("[{}/{}] {} tree(s)".format(it + 1, self.max_iter, K))
            if stop:
                break
        self.train_score_ = np.asarray(self.train_score_)
        self.validation_score_ = np.asarray(self.validation_score_)
        return self

    def _finalize_thresholds(self, nodes):
        thr = np.zeros(len(nodes["value"]))
        raw = np.zeros((len(nodes["value"]), 8), dtype=np.uint32)
        for i in np.where(nodes["is_leaf"] == 0)[0]:
            f, b = nodes["feature_idx"][i], nodes["bin_threshold"][i]
            if nodes["is_categorical"][i]:
                # binned bitset -> raw category values
                cats = self._bin_mapper.bin_thresholds_[f]
                bits = nodes["left_cat_bitset"][i]
                for j, c in enumerate(cats):
                    if (bits[j >> 5] >> (j & 31)) & 1:
                        c = int(c)
                        raw[i, c >> 5] |= np.uint32(1 << (c & 31))
                continue
            if b == self._bin_mapper.n_bins_non_missing_[f] - 1:
                thr[i] = np.inf
            else:
                thr[i] = self._bin_mapper.bin_thresholds_[f][b]
        nodes["num_threshold"] = thr
        nodes["raw_left_cat_bitset"] = raw

    def _is_fitted(self):
        return len(getattr(self, "_predictors", [])) > 0

    @property
    def n_iter_(self):
        check_is_fitted(self, "_predictors")
        return len(self._predictors)

    def _should_stop(self, scores):
        ref = self.n_iter_no_change + 1
        if len(scores) < ref:
            return False
        ref_score = scores[-ref] + self.tol
        return not any(s > ref_score for s in scores[-ref + 1:])

    def _check_early_stopping_loss(self, raw, y_tr, sw_tr, raw_val, y_val, sw_val):
        self.train_score_.append(-self._loss(y_tr, raw, sw_tr))
        if self._use_validation_data:
            self.validation_score_.append(-self._loss(y_val, raw_val, sw_val))
            return self._should_stop(self.validation_score_)
        return self._should_stop(self.train_score_)

    def _check_early_stopping_scorer(self, X_tr, y_tr, sw_tr, X_val, y_val, sw_val):
        if self.scoring is not None and not callable(self.scoring):
            raise ValueError("only scoring='loss', None or a callable(est, X, y) are supported")
        score = (lambda est, X_, y_: est.score(X_, y_)) if self.scoring is None else self.scoring
        yt = self.classes_[y_tr.astype(int)] if is_classifier(self) else y_tr
        self.train_score_.append(score(self, X_tr, yt))
        if self._use_validation_data:
            yv = self.classes_[y_val.astype(int)] if is_classifier(self) else y_val
            self.validation_score_.append(score(self, X_val, yv))
            return self._should_stop(self.validation_score_)
        return self._should_stop(self.train_score_)

    def _raw_predict(self, X):
        X = np.asarray(X.detach().cpu().numpy() if hasattr(X, "detach") else X, dtype=X_DTYPE)
        check_is_fitted(self, "_predictors")
        if X.shape[1] != self._n_features:
            raise ValueError("X has {} features but this estimator was trained with {} features."
                             .format(X.shape[1], self._n_features))
        K = self.n_trees_per_iteration_
        raw = np.zeros((K, X.shape[0])) + self._baseline_prediction
        for k in range(K):
            raw[k] += _predict_trees([it[k] for it in self._predictors], X)
        return raw

    def _staged_raw_predict(self, X):
        X = np.asarray(X, dtype=X_DTYPE)
        K = self.n_trees_per_iteration_
        raw = np.zeros((K, X.shape[0])) + self._baseline_prediction
        for it in self._predictors:
            for k in range(K):
                raw[k] += _predict_trees([it[k]], X)
            yield raw.copy()


def _predict_trees(preds, X):
    X = np.ascontiguousarray(X, dtype=X_DTYPE)
    n, d = X.shape
    if not preds:
        return np.zeros(n)
    cat = lambda k, dt: np.ascontiguousarray(np.concatenate([p.nodes[k] for p in preds]), dtype=dt)  # noqa
    offs = np.zeros(len(preds), dtype=np.int64)
    offs[1:] = np.cumsum([len(p.nodes["value"]) for p in preds])[:-1]
    out = np.empty(n)
    arrs = [cat("feature_idx", np.int32), cat("num_threshold", np.float64),
            cat("missing_go_to_left", np.uint8), cat("left", np.int32), cat("right", np.int32),
            cat("is_leaf", np.uint8), cat("value", np.float64)]
    known = getattr(preds[0], "known_cat_bitsets", None)
    if known is not None and any(p.nodes.get("is_categorical", np.zeros(1)).any() for p in preds):
        ic = cat("is_categorical", np.uint8)
        rb = np.ascontiguousarray(np.concatenate([p.nodes["raw_left_cat_bitset"] for p in preds]),
                                  dtype=np.uint32)
        kb = np.ascontiguousarray(known, dtype=np.uint32)
        _host.lib().sqh_hgb_predict_cat(X.ctypes.data, n, d, *(a.ctypes.data for a in arrs),
                                        ic.ctypes.data, rb.ctypes.data, kb.ctypes.data,
                                        offs.ctypes.data, len(preds), out.ctypes.data)
        return out
    _host.lib().sqh_hgb_predict(X.ctypes.data, n, d, *(a.ctypes.data for a in arrs),
                                offs.ctypes.data, len(preds), out.ctypes.data)
    return out


class HistGradientBoostingRegressor(RegressorMixin, BaseHistGradientBoosting):

    def _more_tags(self):
        return {"allow_nan": True}

    _VALID_LOSSES = ("squared_error", "least_squares", "absolute_error",
                     "least_absolute_deviation", "poisson")

    def __init__(self, loss="squared_error", *, learning_rate=0.1, max_iter=100,
                 max_leaf_nodes=31, max_depth=None, min_samples_leaf=20, l2_regularization=0.0,
                 max_bins=255, categorical_features=None, monotonic_cst=None, warm_start=False,
                 early_stopping="auto", scoring="loss", validation_fraction=0.1,
                 n_iter_no_change=10, tol=1e-7, verbose=0, random_state=None):
        self.loss = loss
        self.learning_rate = learning_rate
        self.max_iter = max_iter
        self.max_leaf_nodes = max_leaf_nodes
        self.max_depth = max_depth
        self.min_samples_leaf = min_samples_leaf
        self.l2_regularization = l2_regularization
        self.max_bins = max_bins
        self.categorical_features = categorical_features
        self.monotonic_cst = monotonic_cst
        self.warm_start = warm_start
        self.early_stopping = early_stopping
        self.scoring = scoring
        self.validation_fraction = validation_fraction
        self.n_iter_no_change = n_iter_no_change
        self.tol = tol
        self.verbose = verbose
        self.random_state = random_state

    n_trees_per_iteration_ = 1

    def _encode_y(self, y):
        y = y.astype(X_DTYPE, copy=False)
        if self.loss == "poisson":
            if not (np.all(y >= 0) and np.sum(y) > 0):
                raise ValueError("loss='poisson' requires non-negative y and sum(y) > 0.")
        return y

    def _get_loss(self, sample_weight):
        return _LOSSES[self.loss](sample_weight=sample_weight)

    def predict(self, X):
        return self._loss.inverse_link_function(self._raw_predict(X).ravel())

    def staged_predict(self, X):
        for raw in self._staged_raw_predict(X):
            yield self._loss.inverse_link_function(raw.ravel())


class HistGradientBoostingClassifier(ClassifierMixin, BaseHistGradientBoosting):

    def _more_tags(self):
        return {"allow_nan": True}

    _VALID_LOSSES = ("binary_crossentropy", "categorical_crossentropy", "log_loss", "auto")

    def __init__(self, loss="auto", *, learning_rate=0.1, max_iter=100, max_leaf_nodes=31,
                 max_depth=None, min_samples_leaf=20, l2_regularization=0.0, max_bins=255,
                 categorical_features=None, monotonic_cst=None, warm_start=False,
                 early_stopping="auto", scoring="loss", validation_fraction=0.1,
                 n_iter_no_change=10, tol=1e-7, verbose=0, random_state=None):
        self.loss = loss
        self.learning_rate = learning_rate
        self.max_iter = max_iter
        self.max_leaf_nodes = max_leaf_nodes
        self.max_depth = max_depth
        self.min_samples_leaf = min_samples_leaf
        self.l2_regularization = l2_regularization
        self.max_bins = max_bins
        self.categorical_features = categorical_features
        self.monotonic_cst = monotonic_cst
        self.warm_start = warm_start
        self.early_stopping = early_stopping
        self.scoring = scoring
        self.validation_fraction = validation_fraction
        self.n_iter_no_change = n_iter_no_change
        self.tol = tol
        self.verbose = verbose
        self.random_state = random_state

    def _encode_y(self, y):
        self.classes_, enc = np.unique(y, return_inverse=True)
        n_classes = self.classes_.shape[0]
        self.n_trees_per_iteration_ = 1 if n_classes <= 2 else n_classes
        return enc.astype(X_DTYPE, copy=False)

    def _get_loss(self, sample_weight):
        if self.loss == "categorical_crossentropy" and self.n_trees_per_iteration_ == 1:
            raise ValueError("'categorical_crossentropy' is not suitable for a binary "
                             "classification problem. Please use 'auto' or "
                             "'binary_crossentropy' instead.")
        if self.loss in ("auto", "log_loss"):
            cls = BinaryCrossEntropy if self.n_trees_per_iteration_ == 1 else \
                CategoricalCrossEntropy
            return cls(sample_weight=sample_weight)
        return _LOSSES[self.loss](sample_weight=sample_weight)

    def decision_function(self, X):
        raw = self._raw_predict(X)
        return raw.ravel() if raw.shape[0] == 1 else raw.T

    def staged_decision_function(self, X):
        for raw in self._staged_raw_predict(X):
            yield raw.ravel() if raw.shape[0] == 1 else raw.T

    def predict_proba(self, X):
        return self._loss.predict_proba(self._raw_predict(X))

    def predict(self, X):
        return self.classes_[np.argmax(self.predict_proba(X), axis=1)]

    def staged_predict_proba(self, X):
        for raw in self._staged_raw_predict(X):
            yield self._loss.predict_proba(raw)

    def staged_predict(self, X):
        for p in self.staged_predict_proba(X):
            yield self.classes_[np.argmax(p, axis=1)]


__all__ = ["HistGradientBoostingClassifier", "HistGradientBoostingRegressor"]
