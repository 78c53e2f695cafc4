"""Ensemble meta-estimators (reference ``sklearn/ensemble``):
``BaggingClassifier`` / ``BaggingRegressor`` (``_bagging.py``),
``IsolationForest`` (``_iforest.py``), ``AdaBoostClassifier`` (SAMME /
SAMME.R) / ``AdaBoostRegressor`` (AdaBoost.R2) (``_weight_boosting.py``),
``VotingClassifier`` / ``VotingRegressor`` (``_voting.py``) and
``StackingClassifier`` / ``StackingRegressor`` (``_stacking.py``).

RNG streams follow the reference: bagging draws one seed per member from
``random_state``; each member's own ``random_state`` and its bootstrap /
feature indices derive independently from that seed, so the trees (built
by the native CART of ``csrc/host/tree.cpp``) match the reference's.
"""

import numbers
from abc import ABCMeta, abstractmethod
from copy import deepcopy

from ...parallel.tasks import Parallel
from ...utils.fixes import delayed
import numpy as np

from ...base import (BaseEstimator, ClassifierMixin, MetaEstimatorMixin, OutlierMixin,
                     RegressorMixin, TransformerMixin, clone, is_classifier)
from ...utils.metaestimators import _BaseComposition
from ...utils.random import sample_without_replacement
from ...utils.validation import check_is_fitted, check_random_state

MAX_INT = np.iinfo(np.int32).max



def _fit_member(est, X, y, sample_weight):
    """One ensemble member's fit (a task of the task layer)."""
    if sample_weight is None:
        return est.fit(X, y)
    return est.fit(X, y, sample_weight=sample_weight)

def _np(a):
    return a.detach().cpu().numpy() if hasattr(a, "detach") else np.asarray(a)


def _dense(X):
    import scipy.sparse as sp
    if sp.issparse(X):
        return X.toarray().astype(np.float64)
    return np.asarray(_np(X), dtype=np.float64)


def _set_random_states(est, random_state):
    rs = check_random_state(random_state)
    to_set = {}
    for key in sorted(est.get_params(deep=True)):
        if key == "random_state" or key.endswith("__random_state"):
            to_set[key] = rs.randint(MAX_INT)
    if to_set:
        est.set_params(**to_set)


def _gen_indices(rs, bootstrap, n_pop, n):
    if bootstrap:
        return rs.randint(0, n_pop, n)
    return sample_without_replacement(n_pop, n, random_state=rs)


def _accepts_sample_weight(est):
    import inspect
    return "sample_weight" in inspect.signature(est.fit).parameters


# ------------------------------------------------------------------ Bagging
class BaseEnsemble(MetaEstimatorMixin, BaseEstimator, metaclass=ABCMeta):
    """Base of homogeneous ensembles (reference ``ensemble/_base.py``):
    validates ``base_estimator`` and stamps out configured clones."""

    @abstractmethod
    def __init__(self, base_estimator=None, *, n_estimators=10, estimator_params=tuple()):
        self.base_estimator = base_estimator
        self.n_estimators = n_estimators
        self.estimator_params = estimator_params

    def _validate_estimator(self, default=None):
        if not isinstance(self.n_estimators, numbers.Integral):
            raise ValueError("n_estimators must be an integer, got {0}."
                             .format(type(self.n_estimators)))
        if self.n_estimators <= 0:
            raise ValueError("n_estimators must be greater than zero, got {0}."
                             .format(self.n_estimators))
        self.base_estimator_ = self.base_estimator if self.base_estimator is not None \
            else default
        if self.base_estimator_ is None:
            raise ValueError("base_estimator cannot be None")

    def _make_estimator(self, append=True, random_state=None):
        est = clone(self.base_estimator_)
        est.set_params(**{p: getattr(self, p) for p in self.estimator_params})
        if random_state is not None:
            _set_random_states(est, random_state)
        if append:
            self.estimators_.append(est)
        return est

    def __len__(self):
        return len(self.estimators_)

    def __getitem__(self, index):
        return self.estimators_[index]

    def __iter__(self):
        return iter(self.estimators_)


class BaseBagging(MetaEstimatorMixin, BaseEstimator):
    def _default_base(self):
        raise NotImplementedError

    def _resolve(self, n, d, max_samples=None):
        ms = self.max_samples if max_samples is None else max_samples
        if not isinstance(ms, numbers.Integral):
            ms = int(ms * n)
        if not (0 < ms <= n):
            raise ValueError("max_samples must be in (0, n_samples]")
        mf = self.max_features
        if isinstance(mf, numbers.Integral):
            pass
        elif isinstance(mf, float):
            mf = mf * d
        else:
            raise ValueError("max_features must be int or float")
        mf = max(1, int(mf))
        if not (0 < mf <= d):
            raise ValueError("max_features must be in (0, n_features]")
        return ms, mf

    def _fit(self, X, y, max_samples=None, max_depth=None, sample_weight=None):
        rs = check_random_state(self.random_state)
        n, d = X.shape
        self.n_features_in_ = d
        self._n_samples = n
        base = clone(self.base_estimator) if self.base_estimator is not None \
            else self._default_base()
        if max_depth is not None:
            base.max_depth = max_depth
        self.base_estimator_ = base
        ms, mf = self._resolve(n, d, max_samples)
        self._max_samples, self._max_features = ms, mf
        if not self.bootstrap and self.oob_score:
            raise ValueError("Out of bag estimation only available if bootstrap=True")
        if self.warm_start and self.oob_score:
            raise ValueError("Out of bag estimate only available if warm_start=False")
        if not self.warm_start or not hasattr(self, "estimators_"):
            self.estimators_, self.estimators_features_, self._seeds = [], [], np.zeros(0, int)
        n_more = self.n_estimators - len(self.estimators_)
        if n_more < 0:
            raise ValueError("n_estimators=%d must be larger or equal to len(estimators_)=%d "
                             "when warm_start==True" % (self.n_estimators, len(self.estimators_)))
        if n_more == 0:
            return self
        if self.warm_start and len(self.estimators_) > 0:
            rs.randint(MAX_INT, size=len(self.estimators_))
        seeds = rs.randint(MAX_INT, size=n_more)
        self._seeds = np.concatenate([self._seeds, seeds])
        sw_ok = _accepts_sample_weight(base)

        def fit_one(seed):
            est = clone(base)
            _set_random_states(est, seed)
            r = check_random_state(seed)
            feats = _gen_indices(r, self.bootstrap_features, d, mf)
            idx = _gen_indices(r, self.bootstrap, n, ms)
            if sw_ok:
                w = np.ones(n) if sample_weight is None else np.array(sample_weight, float)
                if self.bootstrap:
                    w *= np.bincount(idx, minlength=n)
                else:
                    m = np.zeros(n, dtype=bool)
                    m[idx] = True
                    w[~m] = 0
                est.fit(X[:, feats], y, sample_weight=w)
            else:
                est.fit(X[idx][:, feats], y[idx])
            return est, feats

        # members are independent (seeded per member): the task layer fans
        # them out over n_jobs threads / the node's GPUs (reference
        # ensemble/_bagging.py:382 Parallel(n_jobs))
        for est, feats in Parallel(n_jobs=self.n_jobs)(delayed(fit_one)(sd) for sd in seeds):
            self.estimators_.append(est)
            self.estimators_features_.append(feats)
        if self.oob_score:
            self._set_oob_score(X, y)
        return self

    def _get_estimators_indices(self):
        for seed in self._seeds:
            r = check_random_state(seed)
            feats = _gen_indices(r, self.bootstrap_features, self.n_features_in_,
                                 self._max_features)
            idx = _gen_indices(r, self.bootstrap, self._n_samples, self._max_samples)
            yield feats, idx

    @property
    def estimators_samples_(self):
        return [idx for _, idx in self._get_estimators_indices()]

    def fit(self, X, y, sample_weight=None):
        X = _dense(X)
        y = self._validate_y(np.asarray(_np(y)))
        return self._fit(X, y, sample_weight=sample_weight)


class BaggingClassifier(ClassifierMixin, BaseBagging):
    def __init__(self, base_estimator=None, n_estimators=10, *, max_samples=1.0,
                 max_features=1.0, bootstrap=True, bootstrap_features=False, oob_score=False,
                 warm_start=False, n_jobs=None, random_state=None, verbose=0):
        self.base_estimator = base_estimator
        self.n_estimators = n_estimators
        self.max_samples = max_samples
        self.max_features = max_features
        self.bootstrap = bootstrap
        self.bootstrap_features = bootstrap_features
        self.oob_score = oob_score
        self.warm_start = warm_start
        self.n_jobs = n_jobs
        self.random_state = random_state
        self.verbose = verbose

    def _default_base(self):
        from ..tree import DecisionTreeClassifier
        return DecisionTreeClassifier()

    def _validate_y(self, y):
        self.classes_, y = np.unique(y.ravel(), return_inverse=True)
        self.n_classes_ = len(self.classes_)
        return y

    def _member_proba(self, est, Xf):
        nc = self.n_classes_
        if hasattr(est, "predict_proba"):
            p = _np(est.predict_proba(Xf))
            if p.shape[1] == nc:
                return p
            out = np.zeros((Xf.shape[0], nc))
            out[:, est.classes_] = p
            return out
        pred = _np(est.predict(Xf)).astype(int)
        out = np.zeros((Xf.shape[0], nc))
        out[np.arange(Xf.shape[0]), pred] = 1
        return out

    def predict_proba(self, X):
        check_is_fitted(self, "estimators_")
        X = _dense(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError("Number of features of the model must match the input. Model "
                             "n_features_in_ is {0} and input n_features is {1}."
                             .format(self.n_features_in_, X.shape[1]))
        P = sum(self._member_proba(e, X[:, f])
                for e, f in zip(self.estimators_, self.estimators_features_))
        return P / self.n_estimators

    def predict_log_proba(self, X):
        return np.log(self.predict_proba(X))

    def predict(self, X):
        return self.classes_.take(np.argmax(self.predict_proba(X), axis=1), axis=0)

    def decision_function(self, X):
        check_is_fitted(self, "estimators_")
        X = _dense(X)
        return sum(_np(e.decision_function(X[:, f]))
                   for e, f in zip(self.estimators_, self.estimators_features_)) / \
            self.n_estimators

    def _set_oob_score(self, X, y):
        n = y.shape[0]
        pred = np.zeros((n, self.n_classes_))
        for e, (f, idx) in zip(self.estimators_, self._get_estimators_indices()):
            mask = np.ones(n, dtype=bool)
            mask[idx] = False
            pred[mask] += self._member_proba(e, X[mask][:, f])
        den = pred.sum(axis=1)[:, np.newaxis]
        with np.errstate(invalid="ignore", divide="ignore"):
            oob = pred / den
        self.oob_decision_function_ = oob
        self.oob_score_ = np.mean(y == np.argmax(pred, axis=1))


class BaggingRegressor(RegressorMixin, BaseBagging):
    def __init__(self, base_estimator=None, n_estimators=10, *, max_samples=1.0,
                 max_features=1.0, bootstrap=True, bootstrap_features=False, oob_score=False,
                 warm_start=False, n_jobs=None, random_state=None, verbose=0):
        self.base_estimator = base_estimator
        self.n_estimators = n_estimators
        self.max_samples = max_samples
        self.max_features = max_features
        self.bootstrap = bootstrap
        self.bootstrap_features = bootstrap_features
        self.oob_score = oob_score
        self.warm_start = warm_start
        self.n_jobs = n_jobs
        self.random_state = random_state
        self.verbose = verbose

    def _default_base(self):
        from ..tree import DecisionTreeRegressor
        return DecisionTreeRegressor()

    def _validate_y(self, y):
        return y.astype(np.float64)

    def predict(self, X):
        check_is_fitted(self, "estimators_")
        X = _dense(X)
        return sum(_np(e.predict(X[:, f]))
                   for e, f in zip(self.estimators_, self.estimators_features_)) / \
            self.n_estimators

    def _set_oob_score(self, X, y):
        n = y.shape[0]
        pred = np.zeros(n)
        cnt = np.zeros(n)
        for e, (f, idx) in zip(self.estimators_, self._get_estimators_indices()):
            mask = np.ones(n, dtype=bool)
            mask[idx] = False
            pred[mask] += _np(e.predict(X[mask][:, f]))
            cnt[mask] += 1
        cnt[cnt == 0] = 1
        pred /= cnt
        from ...metrics import r2_score
        self.oob_prediction_ = pred
        self.oob_score_ = r2_score(y, pred)


# --------------------------------------------------------- IsolationForest
def _average_path_length(n):
    n = np.asarray(n, dtype=np.float64)
    shape = n.shape
    n = n.reshape((1, -1))
    out = np.zeros(n.shape)
    m1, m2 = n <= 1, n == 2
    nm = ~(m1 | m2)
    out[m2] = 1.0
    out[nm] = 2.0 * (np.log(n[nm] - 1.0) + np.euler_gamma) - 2.0 * (n[nm] - 1.0) / n[nm]
    return out.reshape(shape)


class IsolationForest(OutlierMixin, BaseBagging):
    # fixed bagging settings of the shared BaseBagging machinery (class
    # attributes: not constructor parameters)
    base_estimator = None
    bootstrap_features = False
    oob_score = False

    """Isolation forest: random-split trees; anomaly score from the mean
    isolation depth."""

    def __init__(self, *, n_estimators=100, max_samples="auto", contamination="auto",
                 max_features=1.0, bootstrap=False, n_jobs=None, random_state=None, verbose=0,
                 warm_start=False):
        self.n_estimators = n_estimators
        self.max_samples = max_samples
        self.contamination = contamination
        self.max_features = max_features
        self.bootstrap = bootstrap
        self.n_jobs = n_jobs
        self.random_state = random_state
        self.verbose = verbose
        self.warm_start = warm_start

    def get_params(self, deep=True):
        p = super().get_params(deep)
        return p

    def _default_base(self):
        from ..tree import ExtraTreeRegressor
        return ExtraTreeRegressor(max_features=1, splitter="random")

    def fit(self, X, y=None, sample_weight=None):
        X = _dense(X)
        rnd = check_random_state(self.random_state)
        y = rnd.uniform(size=X.shape[0])
        n = X.shape[0]
        if isinstance(self.max_samples, str):
            if self.max_samples != "auto":
                raise ValueError("max_samples (%s) is not supported.Valid choices are: \"auto\", "
                                 "int orfloat" % self.max_samples)
            ms = min(256, n)
        elif isinstance(self.max_samples, numbers.Integral):
            ms = min(self.max_samples, n)
        else:
            if not 0.0 < self.max_samples <= 1.0:
                raise ValueError("max_samples must be in (0, 1], got %r" % self.max_samples)
            ms = int(self.max_samples * n)
        self.max_samples_ = ms
        self._fit(X, y, max_samples=ms, max_depth=int(np.ceil(np.log2(max(ms, 2)))),
                  sample_weight=sample_weight)
        if self.contamination == "auto":
            self.offset_ = -0.5
        else:
            self.offset_ = np.percentile(self.score_samples(X), 100.0 * self.contamination)
        return self

    def score_samples(self, X):
        check_is_fitted(self, "estimators_")
        X = _dense(X)
        if X.ndim != 2:
            raise ValueError(f"Expected 2D array, got {X.ndim}D array instead. Reshape your data "
                             "either using array.reshape(-1, 1) or array.reshape(1, -1).")
        if X.shape[1] != self.n_features_in_:
            raise ValueError("X has %d features, but IsolationForest is expecting %d features "
                             "as input." % (X.shape[1], self.n_features_in_))
        depths = np.zeros(X.shape[0])
        sub = self._max_features != X.shape[1]
        for t, f in zip(self.estimators_, self.estimators_features_):
            Xs = X[:, f] if sub else X
            leaves = t.apply(Xs)
            path = t.decision_path(Xs)
            nl = t.tree_.n_node_samples[leaves]
            depths += np.ravel(path.sum(axis=1)) + _average_path_length(nl) - 1.0
        den = len(self.estimators_) * _average_path_length([self.max_samples_])
        return -(2 ** (-np.divide(depths, den, out=np.ones_like(depths), where=den != 0)))

    def decision_function(self, X):
        return self.score_samples(X) - self.offset_

    def predict(self, X):
        dec = self.decision_function(X)
        out = np.ones(dec.shape[0], dtype=int)
        out[dec < 0] = -1
        return out


# ----------------------------------------------------------------- AdaBoost
def _softmax(Z):
    Z = Z - Z.max(axis=1, keepdims=True)
    E = np.exp(Z)
    return E / E.sum(axis=1, keepdims=True)


def _samme_proba(est, nc, X):
    p = np.clip(_np(est.predict_proba(X)), np.finfo(np.float64).eps, None)
    lp = np.log(p)
    return (nc - 1) * (lp - (1.0 / nc) * lp.sum(axis=1)[:, np.newaxis])


class BaseWeightBoosting(MetaEstimatorMixin, BaseEstimator):
    def fit(self, X, y, sample_weight=None):
        X = _dense(X)
        y = np.asarray(_np(y))
        if self.learning_rate <= 0:
            raise ValueError("learning_rate must be greater than zero")
        self.n_features_in_ = X.shape[1]
        sw = np.ones(X.shape[0]) if sample_weight is None else \
            np.array(sample_weight, dtype=np.float64)
        sw = sw / sw.sum()
        if np.any(sw < 0):
            raise ValueError("sample_weight cannot contain negative weights")
        self.base_estimator_ = clone(self.base_estimator) if self.base_estimator is not None \
            else self._default_base()
        self.estimators_ = []
        self.estimator_weights_ = np.zeros(self.n_estimators)
        self.estimator_errors_ = np.ones(self.n_estimators)
        rs = check_random_state(self.random_state)
        for it in range(self.n_estimators):
            sw, w, err = self._boost(it, X, y, sw, rs)
            if sw is None:
                break
            self.estimator_weights_[it] = w
            self.estimator_errors_[it] = err
            if err == 0:
                break
            s = np.sum(sw)
            if s <= 0:
                break
            if it < self.n_estimators - 1:
                sw /= s
        return self

    def _make(self, rs):
        est = clone(self.base_estimator_)
        _set_random_states(est, rs)
        self.estimators_.append(est)
        return est

    @property
    def feature_importances_(self):
        norm = self.estimator_weights_.sum()
        return sum(w * e.feature_importances_
                   for w, e in zip(self.estimator_weights_, self.estimators_)) / norm


class AdaBoostClassifier(ClassifierMixin, BaseWeightBoosting):
    def __init__(self, base_estimator=None, *, n_estimators=50, learning_rate=1.0,
                 algorithm="SAMME.R", random_state=None):
        self.base_estimator = base_estimator
        self.n_estimators = n_estimators
        self.learning_rate = learning_rate
        self.algorithm = algorithm
        self.random_state = random_state

    def _default_base(self):
        from ..tree import DecisionTreeClassifier
        return DecisionTreeClassifier(max_depth=1)

    def fit(self, X, y, sample_weight=None):
        if self.algorithm not in ("SAMME", "SAMME.R"):
            raise ValueError("algorithm %s is not supported" % self.algorithm)
        return super().fit(X, y, sample_weight)

    def _boost(self, it, X, y, sw, rs):
        est = self._make(rs)
        est.fit(X, y, sample_weight=sw)
        if it == 0:
            self.classes_ = est.classes_
            self.n_classes_ = len(self.classes_)
        nc, classes = self.n_classes_, self.classes_
        if self.algorithm == "SAMME.R":
            P = _np(est.predict_proba(X))
            pred = classes.take(np.argmax(P, axis=1), axis=0)
            err = np.mean(np.average(pred != y, weights=sw, axis=0))
            if err <= 0:
                return sw, 1.0, 0.0
            codes = np.array([-1.0 / (nc - 1), 1.0])
            coding = codes.take(classes == y[:, np.newaxis])
            P = np.clip(P, np.finfo(P.dtype).eps, None)
            from scipy.special import xlogy
            w = -1.0 * self.learning_rate * ((nc - 1.0) / nc) * xlogy(coding, P).sum(axis=1)
            if it != self.n_estimators - 1:
                sw = sw * np.exp(w * ((sw > 0) | (w < 0)))
            return sw, 1.0, err
        pred = _np(est.predict(X))
        wrong = pred != y
        err = np.mean(np.average(wrong, weights=sw, axis=0))
        if err <= 0:
            return sw, 1.0, 0.0
        if err >= 1.0 - 1.0 / nc:
            self.estimators_.pop(-1)
            if not self.estimators_:
                raise ValueError("BaseClassifier in AdaBoostClassifier ensemble is worse than "
                                 "random, ensemble can not be fit.")
            return None, None, None
        w = self.learning_rate * (np.log((1.0 - err) / err) + np.log(nc - 1.0))
        if it != self.n_estimators - 1:
            sw = np.exp(np.log(sw) + w * wrong * (sw > 0))
        return sw, w, err

    def decision_function(self, X):
        check_is_fitted(self, "estimators_")
        X = _dense(X)
        nc = self.n_classes_
        classes = self.classes_[:, np.newaxis]
        if self.algorithm == "SAMME.R":
            pred = sum(_samme_proba(e, nc, X) for e in self.estimators_)
        else:
            pred = sum((_np(e.predict(X)) == classes).T * w
                       for e, w in zip(self.estimators_, self.estimator_weights_))
        pred = pred / self.estimator_weights_.sum()
        if nc == 2:
            pred[:, 0] *= -1
            return pred.sum(axis=1)
        return pred

    def predict(self, X):
        d = self.decision_function(X)
        if self.n_classes_ == 2:
            return self.classes_.take(d > 0, axis=0)
        return self.classes_.take(np.argmax(d, axis=1), axis=0)

    def predict_proba(self, X):
        d = self.decision_function(X)
        nc = self.n_classes_
        if nc == 1:
            return np.ones((np.asarray(X).shape[0], 1))
        d = np.vstack([-d, d]).T / 2 if nc == 2 else d / (nc - 1)
        return _softmax(d)

    def predict_log_proba(self, X):
        return np.log(self.predict_proba(X))

    def staged_predict(self, X):
        X = _dense(X)
        nc = self.n_classes_
        pred, norm = None, 0.0
        for e, w in zip(self.estimators_, self.estimator_weights_):
            norm += w
            cur = _samme_proba(e, nc, X) if self.algorithm == "SAMME.R" else \
                (_np(e.predict(X)) == self.classes_[:, np.newaxis]).T * w
            pred = cur if pred is None else pred + cur
            d = pred / norm
            if nc == 2:
                dd = d.copy()
                dd[:, 0] *= -1
                yield self.classes_.take(dd.sum(axis=1) > 0, axis=0)
            else:
                yield self.classes_.take(np.argmax(d, axis=1), axis=0)


class AdaBoostRegressor(RegressorMixin, BaseWeightBoosting):
    def __init__(self, base_estimator=None, *, n_estimators=50, learning_rate=1.0,
                 loss="linear", random_state=None):
        self.base_estimator = base_estimator
        self.n_estimators = n_estimators
        self.learning_rate = learning_rate
        self.loss = loss
        self.random_state = random_state

    def _default_base(self):
        from ..tree import DecisionTreeRegressor
        return DecisionTreeRegressor(max_depth=3)

    def fit(self, X, y, sample_weight=None):
        if self.loss not in ("linear", "square", "exponential"):
            raise ValueError("loss must be 'linear', 'square', or 'exponential'")
        return super().fit(X, np.asarray(_np(y), dtype=np.float64), sample_weight)

    def _boost(self, it, X, y, sw, rs):
        est = self._make(rs)
        n = X.shape[0]
        bi = rs.choice(np.arange(n), size=n, replace=True, p=sw)
        est.fit(X[bi], y[bi])
        err_v = np.abs(_np(est.predict(X)) - y)
        mask = sw > 0
        msw, me = sw[mask], err_v[mask]
        emax = me.max()
        if emax != 0:
            me = me / emax
        if self.loss == "square":
            me = me ** 2
        elif self.loss == "exponential":
            me = 1.0 - np.exp(-me)
        err = (msw * me).sum()
        if err <= 0:
            return sw, 1.0, 0.0
        if err >= 0.5:
            if len(self.estimators_) > 1:
                self.estimators_.pop(-1)
            return None, None, None
        beta = err / (1.0 - err)
        w = self.learning_rate * np.log(1.0 / beta)
        if it != self.n_estimators - 1:
            sw = sw.copy()
            sw[mask] *= np.power(beta, (1.0 - me) * self.learning_rate)
        return sw, w, err

    def _median_predict(self, X, limit):
        P = np.array([_np(e.predict(X)) for e in self.estimators_[:limit]]).T
        order = np.argsort(P, axis=1)
        cdf = np.cumsum(self.estimator_weights_[order], axis=1)
        above = cdf >= 0.5 * cdf[:, -1][:, np.newaxis]
        mi = above.argmax(axis=1)
        r = np.arange(X.shape[0])
        return P[r, order[r, mi]]

    def predict(self, X):
        check_is_fitted(self, "estimators_")
        X = _dense(X)
        return self._median_predict(X, len(self.estimators_))

    def staged_predict(self, X):
        X = _dense(X)
        for i in range(1, len(self.estimators_) + 1):
            yield self._median_predict(X, i)


# ------------------------------------------------------------------- Voting
class _BaseVoting(TransformerMixin, MetaEstimatorMixin, _BaseComposition):
    def get_params(self, deep=True):
        return self._get_params("estimators", deep=deep)

    def set_params(self, **params):
        self._set_params("estimators", **params)
        return self

    def _validate_names(self, names):
        if len(set(names)) != len(names):
            raise ValueError("Names provided are not unique: {0!r}".format(list(names)))

    @property
    def _weights_not_none(self):
        if self.weights is None:
            return None
        return [w for (_, e), w in zip(self.estimators, self.weights) if e != "drop"]

    def _fit_members(self, X, y, sample_weight):
        names = [n for n, _ in self.estimators]
        self._validate_names(names)
        if self.weights is not None and len(self.weights) != len(self.estimators):
            raise ValueError("Number of `estimators` and weights must be equal; got %d weights, "
                             "%d estimators" % (len(self.weights), len(self.estimators)))
        self.estimators_ = []
        self.named_estimators_ = {}
        live = [(n, e) for n, e in self.estimators if e != "drop"]
        fitted = Parallel(n_jobs=self.n_jobs)(
            delayed(_fit_member)(clone(e), X, y, sample_weight) for _, e in live)
        for (n, _), c in zip(live, fitted):
            self.estimators_.append(c)
            self.named_estimators_[n] = c
        if hasattr(self.estimators_[0], "n_features_in_"):
            self.n_features_in_ = self.estimators_[0].n_features_in_
        return self

    def _predict(self, X):
        return np.asarray([_np(e.predict(X)) for e in self.estimators_]).T


class VotingClassifier(ClassifierMixin, _BaseVoting):
    def __init__(self, estimators, *, voting="hard", weights=None, n_jobs=None,
                 flatten_transform=True, verbose=False):
        self.estimators = estimators
        self.voting = voting
        self.weights = weights
        self.n_jobs = n_jobs
        self.flatten_transform = flatten_transform
        self.verbose = verbose

    def fit(self, X, y, sample_weight=None):
        from ...preprocessing import LabelEncoder
        if self.voting not in ("soft", "hard"):
            raise ValueError("Voting must be 'soft' or 'hard'; got (voting=%r)" % self.voting)
        y = np.asarray(_np(y))
        if y.ndim > 1 and y.shape[1] > 1:
            raise NotImplementedError("Multilabel and multi-output classification is not "
                                      "supported.")
        self.le_ = LabelEncoder().fit(y)
        self.classes_ = self.le_.classes_
        return self._fit_members(X, self.le_.transform(y), sample_weight)

    def _collect_probas(self, X):
        return np.asarray([_np(e.predict_proba(X)) for e in self.estimators_])

    def predict_proba(self, X):
        if self.voting == "hard":
            raise AttributeError("predict_proba is not available when voting=%r" % self.voting)
        check_is_fitted(self, "estimators_")
        return np.average(self._collect_probas(X), axis=0, weights=self._weights_not_none)

    def predict(self, X):
        check_is_fitted(self, "estimators_")
        if self.voting == "soft":
            maj = np.argmax(self.predict_proba(X), axis=1)
        else:
            P = self._predict(X).astype(int)
            maj = np.apply_along_axis(
                lambda x: np.argmax(np.bincount(x, weights=self._weights_not_none)), axis=1,
                arr=P)
        return self.le_.inverse_transform(maj)

    def transform(self, X):
        check_is_fitted(self, "estimators_")
        if self.voting == "soft":
            P = self._collect_probas(X)
            return np.hstack(P) if self.flatten_transform else P
        return self._predict(X)


class VotingRegressor(RegressorMixin, _BaseVoting):
    def __init__(self, estimators, *, weights=None, n_jobs=None, verbose=False):
        self.estimators = estimators
        self.weights = weights
        self.n_jobs = n_jobs
        self.verbose = verbose

    def fit(self, X, y, sample_weight=None):
        return self._fit_members(X, np.asarray(_np(y), dtype=np.float64), sample_weight)

    def predict(self, X):
        check_is_fitted(self, "estimators_")
        return np.average(self._predict(X), axis=1, weights=self._weights_not_none)

    def transform(self, X):
        check_is_fitted(self, "estimators_")
        return self._predict(X)


# ----------------------------------------------------------------- Stacking
class _BaseStacking(TransformerMixin, MetaEstimatorMixin, _BaseComposition):
    def get_params(self, deep=True):
        return self._get_params("estimators", deep=deep)

    def set_params(self, **params):
        self._set_params("estimators", **params)
        return self

    def _method_name(self, est, method):
        if est == "drop":
            return None
        if method == "auto":
            for m in ("predict_proba", "decision_function", "predict"):
                if hasattr(est, m):
                    return m
        if not hasattr(est, method):
            raise ValueError("Underlying estimator %s does not implement the method %s."
                             % (type(est).__name__, method))
        return method

    def _concat(self, X, preds):
        meta = []
        for i, p in enumerate(preds):
            p = np.asarray(p)
            if p.ndim == 1:
                meta.append(p.reshape(-1, 1))
            elif self.stack_method_[i] == "predict_proba" and len(getattr(self, "classes_", [])) \
                    == 2:
                meta.append(p[:, 1:])
            else:
                meta.append(p)
        if self.passthrough:
            meta.append(_dense(X))
        return np.hstack(meta)

    def _fit_stack(self, X, y, sample_weight):
        from ...model_selection import check_cv, cross_val_predict
        names = [n for n, _ in self.estimators]
        if len(set(names)) != len(names):
            raise ValueError("Names provided are not unique: {0!r}".format(names))
        ests = [e for _, e in self.estimators]
        if all(e == "drop" for e in ests):
            raise ValueError("All estimators are dropped. At least one is required to be an "
                             "estimator.")
        self.final_estimator_ = clone(self.final_estimator) if self.final_estimator is not None \
            else self._default_final()
        self.estimators_ = []
        self.named_estimators_ = {}
        live_named = [(n, e) for n, e in self.estimators if e != "drop"]
        fitted = Parallel(n_jobs=self.n_jobs)(
            delayed(_fit_member)(clone(e), X, y, sample_weight) for _, e in live_named)
        for (n, _), c in zip(live_named, fitted):
            self.estimators_.append(c)
            self.named_estimators_[n] = c
        meth = self.stack_method if isinstance(self.stack_method, str) else None
        self.stack_method_ = [self._method_name(e, meth or "auto") for e in ests]
        self.stack_method_ = [m for m in self.stack_method_ if m is not None]
        if self.cv == "prefit":
            preds = [getattr(e, m)(X) for e, m in zip(self.estimators_, self.stack_method_)]
        else:
            cv = check_cv(self.cv, y=y, classifier=is_classifier(self))
            if hasattr(cv, "random_state") and cv.random_state is None and \
                    getattr(cv, "shuffle", False):
                cv.random_state = np.random.RandomState()
            fp = {} if sample_weight is None else {"sample_weight": sample_weight}
            live = [e for e in ests if e != "drop"]
            preds = [cross_val_predict(clone(e), X, y, cv=deepcopy(cv), method=m, fit_params=fp)
                     for e, m in zip(live, self.stack_method_)]
        Xm = self._concat(X, preds)
        self.final_estimator_.fit(Xm, y) if sample_weight is None else \
            self.final_estimator_.fit(Xm, y, sample_weight=sample_weight)
        if hasattr(self.estimators_[0], "n_features_in_"):
            self.n_features_in_ = self.estimators_[0].n_features_in_
        return self

    def transform(self, X):
        check_is_fitted(self, "estimators_")
        preds = [getattr(e, m)(X) for e, m in zip(self.estimators_, self.stack_method_)]
        return self._concat(X, preds)


class StackingClassifier(ClassifierMixin, _BaseStacking):
    def __init__(self, estimators, final_estimator=None, *, cv=None, stack_method="auto",
                 n_jobs=None, passthrough=False, verbose=0):
        self.estimators = estimators
        self.final_estimator = final_estimator
        self.cv = cv
        self.stack_method = stack_method
        self.n_jobs = n_jobs
        self.passthrough = passthrough
        self.verbose = verbose

    def _default_final(self):
        from ..linear_model import LogisticRegression
        return LogisticRegression()

    def fit(self, X, y, sample_weight=None):
        from ...preprocessing import LabelEncoder
        self._le = LabelEncoder().fit(np.asarray(_np(y)))
        self.classes_ = self._le.classes_
        return self._fit_stack(X, self._le.transform(np.asarray(_np(y))), sample_weight)

    def predict(self, X):
        return self._le.inverse_transform(
            np.asarray(self.final_estimator_.predict(self.transform(X))).astype(int))

    def predict_proba(self, X):
        return self.final_estimator_.predict_proba(self.transform(X))

    def decision_function(self, X):
        return self.final_estimator_.decision_function(self.transform(X))


class StackingRegressor(RegressorMixin, _BaseStacking):
    stack_method = "predict"   # fixed for regressors (not a parameter)

    def __init__(self, estimators, final_estimator=None, *, cv=None, n_jobs=None,
                 passthrough=False, verbose=0):
        self.estimators = estimators
        self.final_estimator = final_estimator
        self.cv = cv

        self.n_jobs = n_jobs
        self.passthrough = passthrough
        self.verbose = verbose

    def _default_final(self):
        from ..linear_model import RidgeCV
        return RidgeCV()

    def fit(self, X, y, sample_weight=None):
        return self._fit_stack(X, np.asarray(_np(y), dtype=np.float64), sample_weight)

    def predict(self, X):
        return self.final_estimator_.predict(self.transform(X))


__all__ = ["BaggingClassifier", "BaggingRegressor", "IsolationForest", "AdaBoostClassifier",
           "AdaBoostRegressor", "VotingClassifier", "VotingRegressor", "StackingClassifier",
           "StackingRegressor"]
