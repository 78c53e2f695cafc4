"""Stochastic-gradient linear models (reference
``linear_model/_stochastic_gradient.py``, ``_perceptron.py``,
``_passive_aggressive.py``).

The per-sample loop is the host-native ``sqh_sgd_plain``
(``csrc/host/sgd.cpp``) - SGD is inherently sequential over samples, so
it runs as tight C++ on one core while one-vs-rest subproblems of a
multiclass fit run concurrently on a thread pool (ctypes drops the GIL).
RNG consumption follows the reference exactly:

* binary / OvR subproblem (reference _stochastic_gradient.py:fit_binary):
  ``make_dataset`` draws ``randint(1, 2**31-1)`` then the shuffle seed is
  ``randint(MAX_INT)`` from the same RandomState;
* multiclass: ``seeds = rs.randint(MAX_INT, size=n_classes)`` first, each
  subproblem seeded with its own RandomState(seed);
* regressor / one-class: dataset seed from the global RNG, shuffle seed
  ``randint(0, 2**31-1)`` from ``check_random_state(random_state)``.
"""

import ctypes
import numbers
import warnings
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import scipy.sparse as sp

from ...base import BaseEstimator, ClassifierMixin, OutlierMixin, RegressorMixin
from ...exceptions import ConvergenceWarning
from ...ops import _host
from ...utils.class_weight import compute_class_weight
from ...utils.validation import check_array, check_is_fitted, check_random_state
from ._base import LinearClassifierMixin, SparseCoefMixin
from ._sgd_losses import make_loss

MAX_INT = np.iinfo(np.int32).max
DEFAULT_EPSILON = 0.1
_LOSS_KIND = {"hinge": 0, "squared_hinge": 1, "log": 2, "log_loss": 2, "modified_huber": 3,
              "squared_error": 4, "squared_loss": 4, "huber": 5, "epsilon_insensitive": 6,
              "squared_epsilon_insensitive": 7, "perceptron": 0}
LEARNING_RATE_TYPES = {"constant": 1, "optimal": 2, "invscaling": 3, "adaptive": 4,
                       "pa1": 5, "pa2": 6}
PENALTY_TYPES = {"none": 0, "l2": 2, "l1": 1, "elasticnet": 3}


def _c(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def _as_sgd_X(X):
    if sp.issparse(X):
        X = sp.csr_matrix(X, dtype=np.float64)
        X.sort_indices()
        return X
    return check_array(X, dtype=np.float64, order="C")


def _plain_sgd(coef, intercept, average_coef, average_intercept, loss, loss_param, penalty_type,
               alpha, C, l1_ratio, X, y, sample_weight, validation_mask, early_stopping,
               score_type, n_iter_no_change, max_iter, tol, fit_intercept, shuffle, seed,
               weight_pos, weight_neg, learning_rate, eta0, power_t, one_class, t, average):
    """Runs the native loop in place on ``coef`` / ``average_coef``;
    returns (intercept, average_intercept, n_iter)."""
    n, d = X.shape
    if sp.issparse(X):
        data, indptr, indices = X.data, X.indptr.astype(np.int32), X.indices.astype(np.int32)
        decay = 0.01
    else:
        data, indptr, indices = X, None, None
        decay = 1.0
    assert coef.dtype == np.float64 and coef.flags.c_contiguous and coef.shape == (d,)
    aw = average_coef if average_coef is not None else None
    if aw is not None:
        assert aw.flags.c_contiguous and aw.shape == (d,)
    io = np.array([intercept, average_intercept, 0.0])
    iprm = np.array([_LOSS_KIND[loss], penalty_type, LEARNING_RATE_TYPES[learning_rate],
                     n_iter_no_change, max_iter, int(fit_intercept), int(shuffle), int(one_class),
                     int(early_stopping), score_type], dtype=np.int32)
    dprm = np.array([loss_param, alpha, C, l1_ratio, tol if tol is not None else -np.inf,
                     weight_pos, weight_neg, eta0, power_t, t, decay, float(average)],
                    dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    sw = np.ascontiguousarray(sample_weight, dtype=np.float64)
    vm = np.ascontiguousarray(validation_mask, dtype=np.uint8)
    index = np.arange(n, dtype=np.int32)
    rc = _host.lib().sqh_sgd_plain(_c(coef), _c(aw), _c(io), _c(data), _c(indptr), _c(indices),
                                   _c(y), _c(sw), n, d, _c(vm), _c(iprm), _c(dprm),
                                   int(seed) & 0xFFFFFFFF, _c(index))
    if rc < 0:
        raise ValueError(("Floating-point under-/overflow occurred at epoch #%d. Scaling input "
                          "data with StandardScaler or MinMaxScaler might help.") % (-rc))
    return float(io[0]), float(io[1]), int(rc)


def _dataset_seed(random_state):
    """The reference's make_dataset draw (reference linear_model/_base.py:194)."""
    check_random_state(random_state).randint(1, MAX_INT)


class BaseSGD(SparseCoefMixin, BaseEstimator):
    """Shared parameters/validation (reference _stochastic_gradient.py:73-320)."""

    loss_functions = {}

    def _validate_params(self, for_partial_fit=False):
        if not isinstance(self.shuffle, bool):
            raise ValueError("shuffle must be either True or False")
        if not isinstance(self.early_stopping, bool):
            raise ValueError("early_stopping must be either True or False")
        if self.early_stopping and for_partial_fit:
            raise ValueError("early_stopping should be False with partial_fit")
        if self.max_iter is not None and self.max_iter <= 0:
            raise ValueError("max_iter must be > zero. Got %f" % self.max_iter)
        if not (0.0 <= self.l1_ratio <= 1.0):
            raise ValueError("l1_ratio must be in [0, 1]")
        if not isinstance(self, SGDOneClassSVM) and self.alpha < 0.0:
            raise ValueError("alpha must be >= 0")
        if self.n_iter_no_change < 1:
            raise ValueError("n_iter_no_change must be >= 1")
        if not (0.0 < self.validation_fraction < 1.0):
            raise ValueError("validation_fraction must be in range (0, 1)")
        if self.learning_rate in ("constant", "invscaling", "adaptive") and self.eta0 <= 0.0:
            raise ValueError("eta0 must be > 0")
        if self.learning_rate == "optimal" and self.alpha == 0:
            raise ValueError("alpha must be > 0 since learning_rate is 'optimal'. alpha is used "
                             "to compute the optimal learning rate.")
        self._get_penalty_type(self.penalty)
        if self.learning_rate not in LEARNING_RATE_TYPES:
            raise ValueError("learning rate %s is not supported. " % self.learning_rate)
        if self.loss not in self.loss_functions:
            raise ValueError("The loss %s is not supported. " % self.loss)

    def _loss_param(self, loss):
        if loss in ("huber", "epsilon_insensitive", "squared_epsilon_insensitive"):
            return self.epsilon
        if loss in ("hinge", "squared_hinge"):
            return 1.0
        return 0.0

    def _get_penalty_type(self, penalty):
        key = str(penalty).lower()
        if key not in PENALTY_TYPES:
            raise ValueError("Penalty %s is not supported. " % penalty)
        return PENALTY_TYPES[key]

    def _allocate_parameter_mem(self, n_classes, n_features, coef_init=None,
                                intercept_init=None, one_class=0):
        if n_classes > 2:
            if coef_init is not None:
                coef_init = np.array(coef_init, dtype=np.float64, order="C")
                if coef_init.shape != (n_classes, n_features):
                    raise ValueError("Provided ``coef_`` does not match dataset. ")
                self.coef_ = coef_init
            else:
                self.coef_ = np.zeros((n_classes, n_features), dtype=np.float64, order="C")
            if intercept_init is not None:
                intercept_init = np.array(intercept_init, dtype=np.float64, order="C")
                if intercept_init.shape != (n_classes,):
                    raise ValueError("Provided intercept_init does not match dataset.")
                self.intercept_ = intercept_init
            else:
                self.intercept_ = np.zeros(n_classes, dtype=np.float64, order="C")
        else:
            if coef_init is not None:
                coef_init = np.array(coef_init, dtype=np.float64, order="C").ravel()
                if coef_init.shape != (n_features,):
                    raise ValueError("Provided coef_init does not match dataset.")
                self.coef_ = coef_init
            else:
                self.coef_ = np.zeros(n_features, dtype=np.float64, order="C")
            if intercept_init is not None:
                intercept_init = np.asarray(intercept_init, dtype=np.float64)
                if intercept_init.shape not in ((1,), ()):
                    raise ValueError("Provided intercept_init does not match dataset.")
                if one_class:
                    self.offset_ = intercept_init.reshape(1,)
                else:
                    self.intercept_ = intercept_init.reshape(1,)
            else:
                if one_class:
                    self.offset_ = np.zeros(1, dtype=np.float64)
                else:
                    self.intercept_ = np.zeros(1, dtype=np.float64)
        if self.average > 0:
            self._standard_coef = self.coef_
            self._average_coef = np.zeros(self.coef_.shape, dtype=np.float64, order="C")
            self._standard_intercept = 1 - self.offset_ if one_class else self.intercept_
            self._average_intercept = np.zeros(self._standard_intercept.shape, dtype=np.float64)

    def _make_validation_split(self, y):
        from ...model_selection import ShuffleSplit, StratifiedShuffleSplit
        n = y.shape[0]
        mask = np.zeros(n, dtype=np.uint8)
        if not self.early_stopping:
            return mask
        splitter = StratifiedShuffleSplit if isinstance(self, ClassifierMixin) else ShuffleSplit
        cv = splitter(test_size=self.validation_fraction, random_state=self.random_state)
        idx_train, idx_val = next(cv.split(np.zeros((n, 1)), y))
        if idx_train.shape[0] == 0 or idx_val.shape[0] == 0:
            raise ValueError(
                "Splitting %d samples into a train set and a validation set with "
                "validation_fraction=%r led to an empty set (%d and %d samples). Please either "
                "change validation_fraction, increase number of samples, or disable "
                "early_stopping." % (n, self.validation_fraction, idx_train.shape[0],
                                     idx_val.shape[0]))
        mask[idx_val] = 1
        return mask

    def _check_X_predict(self, X):
        check_is_fitted(self)
        X = X.tocsr() if sp.issparse(X) else check_array(X, dtype=np.float64)
        d = np.atleast_2d(self.coef_).shape[-1]
        if X.shape[1] != d:
            raise ValueError("X has %d features, but %s is expecting %d features as input."
                             % (X.shape[1], type(self).__name__, d))
        return X

    def _sample_weight(self, sample_weight, n):
        if sample_weight is None:
            return np.ones(n, dtype=np.float64)
        if isinstance(sample_weight, numbers.Number):
            return np.full(n, float(sample_weight))
        sw = np.asarray(sample_weight, dtype=np.float64)
        if sw.shape != (n,):
            raise ValueError("sample_weight.shape == {}, expected {}!".format(sw.shape, (n,)))
        return sw


def _fit_binary(est, i, X, y, alpha, C, learning_rate, max_iter, pos_weight, neg_weight,
                sample_weight, validation_mask=None, random_state=None, loss=None):
    """Reference _stochastic_gradient.py:fit_binary."""
    y_i = np.ones(y.shape, dtype=np.float64)
    y_i[y != est.classes_[i]] = -1.0
    average_intercept = 0.0
    average_coef = None
    if len(est.classes_) == 2:
        if not est.average:
            coef, intercept = est.coef_.ravel(), est.intercept_[0]
        else:
            coef, intercept = est._standard_coef.ravel(), est._standard_intercept[0]
            average_coef, average_intercept = est._average_coef.ravel(), est._average_intercept[0]
    else:
        if not est.average:
            coef, intercept = est.coef_[i], est.intercept_[i]
        else:
            coef, intercept = est._standard_coef[i], est._standard_intercept[i]
            average_coef, average_intercept = est._average_coef[i], est._average_intercept[i]
    rs = check_random_state(random_state)
    _dataset_seed(rs)
    if validation_mask is None:
        validation_mask = est._make_validation_split(y_i)
    seed = rs.randint(MAX_INT)
    loss = loss if loss is not None else est.loss
    intercept, average_intercept, n_iter = _plain_sgd(
        coef, intercept, average_coef, average_intercept, loss, est._loss_param(loss),
        est._get_penalty_type(est.penalty), alpha, C, est.l1_ratio, X, y_i, sample_weight,
        validation_mask, est.early_stopping, 0, int(est.n_iter_no_change), max_iter, est.tol,
        est.fit_intercept, est.shuffle, seed, pos_weight, neg_weight, learning_rate, est.eta0,
        est.power_t, 0, est.t_, est.average)
    if est.average:
        if len(est.classes_) == 2:
            est._average_intercept[0] = average_intercept
        else:
            est._average_intercept[i] = average_intercept
    return coef, intercept, n_iter


class BaseSGDClassifier(LinearClassifierMixin, BaseSGD):
    """OvR SGD classifier core (reference _stochastic_gradient.py:474-790)."""

    loss_functions = {k: None for k in ("hinge", "squared_hinge", "perceptron", "log", "log_loss",
                                        "modified_huber", "squared_error", "squared_loss",
                                        "huber", "epsilon_insensitive",
                                        "squared_epsilon_insensitive")}

    def _partial_fit(self, X, y, alpha, C, loss, learning_rate, max_iter, classes,
                     sample_weight, coef_init, intercept_init):
        first_call = not hasattr(self, "classes_") or self.classes_ is None
        X = _as_sgd_X(X)
        y = np.asarray(y)
        if y.ndim == 2 and y.shape[1] == 1:
            y = y.ravel()
        n, d = X.shape
        if X.shape[0] != y.shape[0]:
            raise ValueError("Found input variables with inconsistent numbers of samples: "
                             "[%d, %d]" % (X.shape[0], y.shape[0]))
        if first_call:
            if classes is None:
                raise ValueError("classes must be passed on the first call to partial_fit.")
            self.classes_ = np.unique(classes)
            self.n_features_in_ = d
        elif classes is not None and not np.array_equal(self.classes_, np.unique(classes)):
            raise ValueError("`classes=%r` is not the same as on last call to partial_fit, "
                             "was: %r" % (classes, self.classes_))
        n_classes = self.classes_.shape[0]
        self._expanded_class_weight = compute_class_weight(self.class_weight,
                                                           classes=self.classes_, y=y)
        sample_weight = self._sample_weight(sample_weight, n)
        if getattr(self, "coef_", None) is None or coef_init is not None:
            self._allocate_parameter_mem(n_classes, d, coef_init, intercept_init)
        elif d != self.coef_.shape[-1]:
            raise ValueError("Number of features %d does not match previous data %d."
                             % (d, self.coef_.shape[-1]))
        self.loss_function_ = make_loss(loss, self._loss_param(loss))
        self._fit_loss = loss
        if not hasattr(self, "t_"):
            self.t_ = 1.0
        if n_classes > 2:
            self._fit_multiclass(X, y, alpha, C, learning_rate, sample_weight, max_iter)
        elif n_classes == 2:
            self._fit_binary(X, y, alpha, C, learning_rate, sample_weight, max_iter)
        else:
            raise ValueError("The number of classes has to be greater than one; got %d class"
                             % n_classes)
        return self

    def _fit(self, X, y, alpha, C, loss, learning_rate, coef_init=None, intercept_init=None,
             sample_weight=None):
        self._validate_params()
        if hasattr(self, "classes_"):
            self.classes_ = None
        classes = np.unique(np.asarray(y))
        if self.warm_start and getattr(self, "coef_", None) is not None:
            if coef_init is None:
                coef_init = self.coef_
            if intercept_init is None:
                intercept_init = self.intercept_
        else:
            self.coef_ = None
            self.intercept_ = None
        if self.average > 0:
            self._standard_coef = self.coef_
            self._standard_intercept = self.intercept_
            self._average_coef = None
            self._average_intercept = None
        self.t_ = 1.0
        self._partial_fit(X, y, alpha, C, loss, learning_rate, self.max_iter, classes,
                          sample_weight, coef_init, intercept_init)
        if self.tol is not None and self.tol > -np.inf and self.n_iter_ == self.max_iter:
            warnings.warn("Maximum number of iteration reached before convergence. Consider "
                          "increasing max_iter to improve the fit.", ConvergenceWarning)
        return self

    def _fit_binary(self, X, y, alpha, C, learning_rate, sample_weight, max_iter):
        coef, intercept, n_iter = _fit_binary(
            self, 1, X, y, alpha, C, learning_rate, max_iter, self._expanded_class_weight[1],
            self._expanded_class_weight[0], sample_weight, random_state=self.random_state,
            loss=self._fit_loss)
        self.t_ += n_iter * X.shape[0]
        self.n_iter_ = n_iter
        if self.average > 0:
            if self.average <= self.t_ - 1:
                self.coef_ = self._average_coef.reshape(1, -1)
                self.intercept_ = self._average_intercept
            else:
                self.coef_ = self._standard_coef.reshape(1, -1)
                self._standard_intercept = np.atleast_1d(intercept)
                self.intercept_ = self._standard_intercept
        else:
            self.coef_ = coef.reshape(1, -1)
            self.intercept_ = np.atleast_1d(intercept)

    def _fit_multiclass(self, X, y, alpha, C, learning_rate, sample_weight, max_iter):
        validation_mask = self._make_validation_split(y)
        rs = check_random_state(self.random_state)
        seeds = rs.randint(MAX_INT, size=len(self.classes_))

        def job(i):
            return _fit_binary(self, i, X, y, alpha, C, learning_rate, max_iter,
                               self._expanded_class_weight[i], 1., sample_weight,
                               validation_mask=validation_mask, random_state=seeds[i],
                               loss=self._fit_loss)

        n_jobs = self.n_jobs if getattr(self, "n_jobs", None) not in (None, 0) else 1
        if n_jobs < 0:
            import os
            n_jobs = os.cpu_count() or 1
        if n_jobs > 1:
            with ThreadPoolExecutor(min(n_jobs, len(seeds))) as ex:
                result = list(ex.map(job, range(len(seeds))))
        else:
            result = [job(i) for i in range(len(seeds))]
        n_iter = 0.
        for i, (_, intercept, n_iter_i) in enumerate(result):
            self.intercept_[i] = intercept
            n_iter = max(n_iter, n_iter_i)
        self.t_ += n_iter * X.shape[0]
        self.n_iter_ = n_iter
        if self.average > 0:
            if self.average <= self.t_ - 1.0:
                self.coef_ = self._average_coef
                self.intercept_ = self._average_intercept
            else:
                self.coef_ = self._standard_coef
                self._standard_intercept = np.atleast_1d(self.intercept_)
                self.intercept_ = self._standard_intercept

    def partial_fit(self, X, y, classes=None, sample_weight=None):
        self._validate_params(for_partial_fit=True)
        if self.class_weight in ["balanced"]:
            raise ValueError("class_weight 'balanced' is not supported for partial_fit. In order "
                             "to use 'balanced' weights, use compute_class_weight('balanced', "
                             "classes=classes, y=y).")
        return self._partial_fit(X, y, alpha=self.alpha, C=1.0, loss=self.loss,
                                 learning_rate=self.learning_rate, max_iter=1, classes=classes,
                                 sample_weight=sample_weight, coef_init=None,
                                 intercept_init=None)

    def fit(self, X, y, coef_init=None, intercept_init=None, sample_weight=None):
        return self._fit(X, y, alpha=self.alpha, C=1.0, loss=self.loss,
                         learning_rate=self.learning_rate, coef_init=coef_init,
                         intercept_init=intercept_init, sample_weight=sample_weight)

    def decision_function(self, X):
        X = self._check_X_predict(X)
        coef = self.coef_.toarray() if sp.issparse(self.coef_) else self.coef_
        scores = np.asarray(X @ coef.T) + self.intercept_
        return scores.ravel() if scores.shape[1] == 1 else scores


class SGDClassifier(BaseSGDClassifier):
    """Linear classifiers trained by SGD (reference _stochastic_gradient.py:792)."""

    def __init__(self, loss="hinge", *, penalty="l2", alpha=0.0001, l1_ratio=0.15,
                 fit_intercept=True, max_iter=1000, tol=1e-3, shuffle=True, verbose=0,
                 epsilon=DEFAULT_EPSILON, n_jobs=None, random_state=None, learning_rate="optimal",
                 eta0=0.0, power_t=0.5, early_stopping=False, validation_fraction=0.1,
                 n_iter_no_change=5, class_weight=None, warm_start=False, average=False):
        self.loss = loss
        self.penalty = penalty
        self.alpha = alpha
        self.l1_ratio = l1_ratio
        self.fit_intercept = fit_intercept
        self.max_iter = max_iter
        self.tol = tol
        self.shuffle = shuffle
        self.verbose = verbose
        self.epsilon = epsilon
        self.n_jobs = n_jobs
        self.random_state = random_state
        self.learning_rate = learning_rate
        self.eta0 = eta0
        self.power_t = power_t
        self.early_stopping = early_stopping
        self.validation_fraction = validation_fraction
        self.n_iter_no_change = n_iter_no_change
        self.class_weight = class_weight
        self.warm_start = warm_start
        self.average = average

    def _check_proba(self):
        if self.loss not in ("log", "log_loss", "modified_huber"):
            raise AttributeError("probability estimates are not available for loss=%r"
                                 % self.loss)
        return True

    @property
    def predict_proba(self):
        self._check_proba()
        return self._predict_proba

    def _predict_proba(self, X):
        check_is_fitted(self)
        if self.loss in ("log", "log_loss"):
            return self._predict_proba_lr(X)
        binary = len(self.classes_) == 2
        scores = self.decision_function(X)
        if binary:
            prob2 = np.ones((scores.shape[0], 2))
            prob = prob2[:, 1]
        else:
            prob = scores
        np.clip(scores, -1, 1, prob)
        prob += 1.
        prob /= 2.
        if binary:
            prob2[:, 0] -= prob
            return prob2
        prob_sum = prob.sum(axis=1)
        all_zero = prob_sum == 0
        if np.any(all_zero):
            prob[all_zero, :] = 1
            prob_sum[all_zero] = len(self.classes_)
        prob /= prob_sum.reshape((prob.shape[0], -1))
        return prob

    @property
    def predict_log_proba(self):
        self._check_proba()
        return lambda X: np.log(self._predict_proba(X))


class Perceptron(BaseSGDClassifier):
    """Perceptron == SGDClassifier(loss='perceptron', eta0=1,
    learning_rate='constant', penalty=None) (reference _perceptron.py:134)."""

    def __init__(self, *, penalty=None, alpha=0.0001, l1_ratio=0.15, fit_intercept=True,
                 max_iter=1000, tol=1e-3, shuffle=True, verbose=0, eta0=1.0, n_jobs=None,
                 random_state=0, early_stopping=False, validation_fraction=0.1,
                 n_iter_no_change=5, class_weight=None, warm_start=False):
        self.penalty = penalty
        self.alpha = alpha
        self.l1_ratio = l1_ratio
        self.fit_intercept = fit_intercept
        self.max_iter = max_iter
        self.tol = tol
        self.shuffle = shuffle
        self.verbose = verbose
        self.eta0 = eta0
        self.n_jobs = n_jobs
        self.random_state = random_state
        self.early_stopping = early_stopping
        self.validation_fraction = validation_fraction
        self.n_iter_no_change = n_iter_no_change
        self.class_weight = class_weight
        self.warm_start = warm_start

    loss = property(lambda self: "perceptron")
    learning_rate = property(lambda self: "constant")
    power_t = property(lambda self: 0.5)
    epsilon = property(lambda self: DEFAULT_EPSILON)
    average = property(lambda self: False)


class PassiveAggressiveClassifier(BaseSGDClassifier):
    """PA-I (hinge) / PA-II (squared_hinge) classifier (reference
    _passive_aggressive.py:10-260): alpha=1, no penalty, Hinge(1) loss with
    the PA step-size rule."""

    def __init__(self, *, C=1.0, fit_intercept=True, max_iter=1000, tol=1e-3,
                 early_stopping=False, validation_fraction=0.1, n_iter_no_change=5,
                 shuffle=True, verbose=0, loss="hinge", n_jobs=None, random_state=None,
                 warm_start=False, class_weight=None, average=False):
        self.C = C
        self.fit_intercept = fit_intercept
        self.max_iter = max_iter
        self.tol = tol
        self.early_stopping = early_stopping
        self.validation_fraction = validation_fraction
        self.n_iter_no_change = n_iter_no_change
        self.shuffle = shuffle
        self.verbose = verbose
        self.loss = loss
        self.n_jobs = n_jobs
        self.random_state = random_state
        self.warm_start = warm_start
        self.class_weight = class_weight
        self.average = average

    penalty = property(lambda self: None)
    alpha = property(lambda self: 1.0)
    l1_ratio = property(lambda self: 0.15)
    eta0 = property(lambda self: 1.0)
    power_t = property(lambda self: 0.5)
    epsilon = property(lambda self: DEFAULT_EPSILON)
    learning_rate = property(lambda self: "pa1")

    def _validate_params(self, for_partial_fit=False):
        if self.loss not in ("hinge", "squared_hinge"):
            raise ValueError("The loss %s is not supported. " % self.loss)
        super()._validate_params(for_partial_fit)

    def partial_fit(self, X, y, classes=None):
        self._validate_params(for_partial_fit=True)
        if self.class_weight == "balanced":
            raise ValueError("class_weight 'balanced' is not supported for partial_fit.")
        lr = "pa1" if self.loss == "hinge" else "pa2"
        return self._partial_fit(X, y, alpha=1.0, C=self.C, loss="hinge", learning_rate=lr,
                                 max_iter=1, classes=classes, sample_weight=None,
                                 coef_init=None, intercept_init=None)

    def fit(self, X, y, coef_init=None, intercept_init=None):
        self._validate_params()
        lr = "pa1" if self.loss == "hinge" else "pa2"
        return self._fit(X, y, alpha=1.0, C=self.C, loss="hinge", learning_rate=lr,
                         coef_init=coef_init, intercept_init=intercept_init)


class BaseSGDRegressor(RegressorMixin, BaseSGD):
    """SGD regressor core (reference _stochastic_gradient.py:1145-1400)."""

    loss_functions = {k: None for k in ("squared_error", "squared_loss", "huber",
                                        "epsilon_insensitive", "squared_epsilon_insensitive")}

    def _partial_fit(self, X, y, alpha, C, loss, learning_rate, max_iter, sample_weight,
                     coef_init, intercept_init):
        first_call = getattr(self, "coef_", None) is None
        X = _as_sgd_X(X)
        y = np.asarray(y, dtype=np.float64)
        if y.ndim == 2 and y.shape[1] == 1:
            y = y.ravel()
        n, d = X.shape
        if n != y.shape[0]:
            raise ValueError("Found input variables with inconsistent numbers of samples: "
                             "[%d, %d]" % (n, y.shape[0]))
        if first_call:
            self.n_features_in_ = d
        elif d != self.coef_.shape[-1]:
            raise ValueError("Number of features %d does not match previous data %d."
                             % (d, self.coef_.shape[-1]))
        sample_weight = self._sample_weight(sample_weight, n)
        if first_call:
            self._allocate_parameter_mem(1, d, coef_init, intercept_init)
        if self.average > 0 and getattr(self, "_average_coef", None) is None:
            self._average_coef = np.zeros(d, dtype=np.float64)
            self._average_intercept = np.zeros(1, dtype=np.float64)
        self._fit_regressor(X, y, alpha, C, loss, learning_rate, sample_weight, max_iter)
        return self

    def partial_fit(self, X, y, sample_weight=None):
        self._validate_params(for_partial_fit=True)
        return self._partial_fit(X, y, self.alpha, C=1.0, loss=self.loss,
                                 learning_rate=self.learning_rate, max_iter=1,
                                 sample_weight=sample_weight, coef_init=None,
                                 intercept_init=None)

    def _fit(self, X, y, alpha, C, loss, learning_rate, coef_init=None, intercept_init=None,
             sample_weight=None):
        self._validate_params()
        if self.warm_start and getattr(self, "coef_", None) is not None:
            if coef_init is None:
                coef_init = self.coef_
            if intercept_init is None:
                intercept_init = self.intercept_
        else:
            self.coef_ = None
            self.intercept_ = None
        self.t_ = 1.0
        self._partial_fit(X, y, alpha, C, loss, learning_rate, self.max_iter, sample_weight,
                          coef_init, intercept_init)
        if self.tol is not None and self.tol > -np.inf and self.n_iter_ == self.max_iter:
            warnings.warn("Maximum number of iteration reached before convergence. Consider "
                          "increasing max_iter to improve the fit.", ConvergenceWarning)
        return self

    def fit(self, X, y, coef_init=None, intercept_init=None, sample_weight=None):
        return self._fit(X, y, alpha=self.alpha, C=1.0, loss=self.loss,
                         learning_rate=self.learning_rate, coef_init=coef_init,
                         intercept_init=intercept_init, sample_weight=sample_weight)

    def _decision_function(self, X):
        X = self._check_X_predict(X)
        coef = self.coef_.toarray() if sp.issparse(self.coef_) else self.coef_
        return (np.asarray(X @ np.ravel(coef)) + self.intercept_).ravel()

    def predict(self, X):
        return self._decision_function(X)

    def _fit_regressor(self, X, y, alpha, C, loss, learning_rate, sample_weight, max_iter):
        _dataset_seed(None)
        if not hasattr(self, "t_"):
            self.t_ = 1.0
        validation_mask = self._make_validation_split(y)
        seed = check_random_state(self.random_state).randint(0, MAX_INT)
        if self.average:
            coef, intercept = self._standard_coef, self._standard_intercept
            average_coef, average_intercept = self._average_coef, self._average_intercept
        else:
            coef, intercept = self.coef_, self.intercept_
            average_coef, average_intercept = None, [0.0]
        intercept, average_intercept, self.n_iter_ = _plain_sgd(
            coef, intercept[0], average_coef, average_intercept[0], loss, self._loss_param(loss),
            self._get_penalty_type(self.penalty), alpha, C, self.l1_ratio, X, y, sample_weight,
            validation_mask, self.early_stopping, 1, int(self.n_iter_no_change), max_iter,
            self.tol, self.fit_intercept, self.shuffle, seed, 1.0, 1.0, learning_rate, self.eta0,
            self.power_t, 0, self.t_, self.average)
        self.t_ += self.n_iter_ * X.shape[0]
        if self.average > 0:
            self._average_intercept = np.atleast_1d(average_intercept)
            self._standard_intercept = np.atleast_1d(intercept)
            if self.average <= self.t_ - 1.0:
                self.coef_ = average_coef
                self.intercept_ = np.atleast_1d(average_intercept)
            else:
                self.coef_ = coef
                self.intercept_ = np.atleast_1d(intercept)
        else:
            self.intercept_ = np.atleast_1d(intercept)


class SGDRegressor(BaseSGDRegressor):
    """Linear regression by SGD (reference _stochastic_gradient.py:1402)."""

    def __init__(self, loss="squared_error", *, penalty="l2", alpha=0.0001, l1_ratio=0.15,
                 fit_intercept=True, max_iter=1000, tol=1e-3, shuffle=True, verbose=0,
                 epsilon=DEFAULT_EPSILON, random_state=None, learning_rate="invscaling",
                 eta0=0.01, power_t=0.25, early_stopping=False, validation_fraction=0.1,
                 n_iter_no_change=5, warm_start=False, average=False):
        self.loss = loss
        self.penalty = penalty
        self.alpha = alpha
        self.l1_ratio = l1_ratio
        self.fit_intercept = fit_intercept
        self.max_iter = max_iter
        self.tol = tol
        self.shuffle = shuffle
        self.verbose = verbose
        self.epsilon = epsilon
        self.random_state = random_state
        self.learning_rate = learning_rate
        self.eta0 = eta0
        self.power_t = power_t
        self.early_stopping = early_stopping
        self.validation_fraction = validation_fraction
        self.n_iter_no_change = n_iter_no_change
        self.warm_start = warm_start
        self.average = average


class PassiveAggressiveRegressor(BaseSGDRegressor):
    """PA-I / PA-II regression (reference _passive_aggressive.py:262-470)."""

    def __init__(self, *, C=1.0, fit_intercept=True, max_iter=1000, tol=1e-3,
                 early_stopping=False, validation_fraction=0.1, n_iter_no_change=5,
                 shuffle=True, verbose=0, loss="epsilon_insensitive", epsilon=DEFAULT_EPSILON,
                 random_state=None, warm_start=False, average=False):
        self.C = C
        self.fit_intercept = fit_intercept
        self.max_iter = max_iter
        self.tol = tol
        self.early_stopping = early_stopping
        self.validation_fraction = validation_fraction
        self.n_iter_no_change = n_iter_no_change
        self.shuffle = shuffle
        self.verbose = verbose
        self.loss = loss
        self.epsilon = epsilon
        self.random_state = random_state
        self.warm_start = warm_start
        self.average = average

    penalty = property(lambda self: None)
    alpha = property(lambda self: 1.0)
    l1_ratio = property(lambda self: 0.15)
    eta0 = property(lambda self: 1.0)
    power_t = property(lambda self: 0.5)
    learning_rate = property(lambda self: "pa1")

    def partial_fit(self, X, y):
        self._validate_params(for_partial_fit=True)
        lr = "pa1" if self.loss == "epsilon_insensitive" else "pa2"
        return self._partial_fit(X, y, alpha=1.0, C=self.C, loss="epsilon_insensitive",
                                 learning_rate=lr, max_iter=1, sample_weight=None,
                                 coef_init=None, intercept_init=None)

    def fit(self, X, y, coef_init=None, intercept_init=None):
        self._validate_params()
        lr = "pa1" if self.loss == "epsilon_insensitive" else "pa2"
        return self._fit(X, y, alpha=1.0, C=self.C, loss="epsilon_insensitive",
                         learning_rate=lr, coef_init=coef_init, intercept_init=intercept_init)


class SGDOneClassSVM(OutlierMixin, BaseSGD):
    """Linear one-class SVM by SGD (reference _stochastic_gradient.py:1663+):
    hinge loss on y=+1 with alpha = nu/2 and the offset update
    ``intercept -= 2*eta*alpha`` inside the loop."""

    loss_functions = {"hinge": None}

    def __init__(self, nu=0.5, fit_intercept=True, max_iter=1000, tol=1e-3, shuffle=True,
                 verbose=0, random_state=None, learning_rate="optimal", eta0=0.0, power_t=0.5,
                 warm_start=False, average=False):
        self.nu = nu
        self.fit_intercept = fit_intercept
        self.max_iter = max_iter
        self.tol = tol
        self.shuffle = shuffle
        self.verbose = verbose
        self.random_state = random_state
        self.learning_rate = learning_rate
        self.eta0 = eta0
        self.power_t = power_t
        self.warm_start = warm_start
        self.average = average

    loss = property(lambda self: "hinge")
    penalty = property(lambda self: "l2")
    alpha = property(lambda self: self.nu / 2)
    l1_ratio = property(lambda self: 0)
    epsilon = property(lambda self: DEFAULT_EPSILON)
    early_stopping = property(lambda self: False)
    validation_fraction = property(lambda self: 0.1)
    n_iter_no_change = property(lambda self: 5)
    C = property(lambda self: 1.0)

    def _validate_params(self, for_partial_fit=False):
        if not (0 < self.nu <= 1):
            raise ValueError("nu must be in (0, 1], got nu=%f" % self.nu)
        super()._validate_params(for_partial_fit)

    def _fit_one_class(self, X, alpha, C, sample_weight, learning_rate, max_iter):
        n = X.shape[0]
        y = np.ones(n, dtype=np.float64)
        _dataset_seed(None)
        validation_mask = self._make_validation_split(y)
        seed = check_random_state(self.random_state).randint(0, MAX_INT)
        if self.average:
            coef, intercept = self._standard_coef, self._standard_intercept
            average_coef, average_intercept = self._average_coef, self._average_intercept
        else:
            coef, intercept = self.coef_, 1 - self.offset_
            average_coef, average_intercept = None, [0.0]
        intercept, average_intercept, self.n_iter_ = _plain_sgd(
            coef, intercept[0], average_coef, average_intercept[0], "hinge", 1.0, 2, alpha, C,
            0.0, X, y, sample_weight, validation_mask, False, 1, 5, max_iter, self.tol,
            self.fit_intercept, self.shuffle, seed, 1.0, 1.0, learning_rate, self.eta0,
            self.power_t, 1, self.t_, self.average)
        self.t_ += self.n_iter_ * n
        if self.average > 0:
            self._average_intercept = np.atleast_1d(average_intercept)
            self._standard_intercept = np.atleast_1d(intercept)
            if self.average <= self.t_ - 1.0:
                self.coef_ = average_coef
                self.offset_ = 1 - np.atleast_1d(average_intercept)
            else:
                self.coef_ = coef
                self.offset_ = 1 - np.atleast_1d(intercept)
        else:
            self.offset_ = 1 - np.atleast_1d(intercept)

    def _partial_fit(self, X, alpha, C, loss, learning_rate, max_iter, sample_weight, coef_init,
                     offset_init):
        first_call = getattr(self, "coef_", None) is None
        X = _as_sgd_X(X)
        d = X.shape[1]
        if first_call:
            self.n_features_in_ = d
        sample_weight = self._sample_weight(sample_weight, X.shape[0])
        if getattr(self, "coef_", None) is None or coef_init is not None:
            self._allocate_parameter_mem(1, d, coef_init, offset_init, 1)
        elif d != self.coef_.shape[-1]:
            raise ValueError("Number of features %d does not match previous data %d."
                             % (d, self.coef_.shape[-1]))
        if self.average and getattr(self, "_average_coef", None) is None:
            self._average_coef = np.zeros(d, dtype=np.float64)
            self._average_intercept = np.zeros(1, dtype=np.float64)
        self.loss_function_ = make_loss(loss, self._loss_param(loss))
        if not hasattr(self, "t_"):
            self.t_ = 1.0
        self._fit_one_class(X, alpha, C, sample_weight, learning_rate, max_iter)
        return self

    def partial_fit(self, X, y=None, sample_weight=None):
        self._validate_params(for_partial_fit=True)
        return self._partial_fit(X, self.nu / 2, 1.0, "hinge", self.learning_rate, 1,
                                 sample_weight, None, None)

    def _fit(self, X, alpha, C, loss, learning_rate, coef_init=None, offset_init=None,
             sample_weight=None):
        self._validate_params()
        if self.warm_start and getattr(self, "coef_", None) is not None:
            if coef_init is None:
                coef_init = self.coef_
            if offset_init is None:
                offset_init = self.offset_
        else:
            self.coef_ = None
            self.offset_ = None
        self.t_ = 1.0
        self._partial_fit(X, alpha, C, loss, learning_rate, self.max_iter, sample_weight,
                          coef_init, offset_init)
        if self.tol is not None and self.tol > -np.inf and self.n_iter_ == self.max_iter:
            warnings.warn("Maximum number of iteration reached before convergence. Consider "
                          "increasing max_iter to improve the fit.", ConvergenceWarning)
        return self

    def fit(self, X, y=None, coef_init=None, offset_init=None, sample_weight=None):
        return self._fit(X, self.nu / 2, 1.0, "hinge", self.learning_rate, coef_init,
                         offset_init, sample_weight)

    def decision_function(self, X):
        X = self._check_X_predict(X)
        return (np.asarray(X @ np.ravel(self.coef_)) - self.offset_).ravel()

    def score_samples(self, X):
        return self.decision_function(X) + self.offset_

    def predict(self, X):
        y = (self.decision_function(X) >= 0).astype(np.int32)
        y[y == 0] = -1
        return y


__all__ = ["SGDClassifier", "SGDRegressor", "SGDOneClassSVM", "Perceptron",
           "PassiveAggressiveClassifier", "PassiveAggressiveRegressor"]
