"""Hyper-parameter search and learning curves (reference
``model_selection/_search.py`` - ``ParameterGrid`` :49, ``ParameterSampler``
:188, ``BaseSearchCV`` :402, ``GridSearchCV`` :1040, ``RandomizedSearchCV``
:1382; ``_search_successive_halving.py``; ``_validation.py`` -
``permutation_test_score`` :1100, ``learning_curve`` :1260,
``validation_curve`` :1520).

Candidates x folds are evaluated in this process: each fit already owns
the GPU (data resident in HBM), so fanning out to worker processes like
the reference's joblib pool would only contend for the device.
``cv_results_`` carries the reference's keys (``mean_fit_time``,
``param_<name>`` masked arrays, ``split<i>_test_<metric>``, ranks, ...).
"""

import time
import warnings
from ..parallel.tasks import Parallel
from ..utils.fixes import delayed
from collections import defaultdict
from collections.abc import Iterable as Iterable_
from collections.abc import Mapping, Sequence
from functools import reduce
from itertools import product
from operator import mul

import numpy as np

from ..base import BaseEstimator, clone, is_classifier
from ..utils.random import sample_without_replacement
from ..utils.validation import check_random_state
from ._split import _safe_index, check_cv
from ._validation import _fit_and_score, get_scorer


class ParameterGrid:
    """Iterable / indexable grid of parameter dicts."""

    def __init__(self, param_grid):
        if not isinstance(param_grid, (Mapping, Iterable_)):
            raise TypeError("Parameter grid is not a dict or a list ({!r})".format(param_grid))
        if isinstance(param_grid, Mapping):
            param_grid = [param_grid]
        for grid in param_grid:
            if not isinstance(grid, dict):
                raise TypeError("Parameter grid is not a dict ({!r})".format(grid))
            for key in grid:
                v = grid[key]
                if isinstance(v, np.ndarray) and v.ndim > 1:
                    raise ValueError("Parameter array should be one-dimensional.")
                if isinstance(v, str) or not isinstance(v, (np.ndarray, Sequence)):
                    raise TypeError("Parameter grid value is not iterable (key={!r}, value={!r})"
                                    .format(key, v))
                if len(v) == 0:
                    raise ValueError("Parameter values for parameter ({}) need to be a non-empty "
                                     "sequence.".format(key))
        self.param_grid = param_grid

    def __iter__(self):
        for p in self.param_grid:
            items = sorted(p.items())
            if not items:
                yield {}
            else:
                keys, values = zip(*items)
                for v in product(*values):
                    yield dict(zip(keys, v))

    def __len__(self):
        return sum(reduce(mul, (len(v) for v in p.values()), 1) for p in self.param_grid)

    def __getitem__(self, ind):
        for sub in self.param_grid:
            if not sub:
                if ind == 0:
                    return {}
                ind -= 1
                continue
            keys, values = zip(*sorted(sub.items())[::-1])
            sizes = [len(v) for v in values]
            total = int(np.prod(sizes))
            if ind >= total:
                ind -= total
            else:
                out = {}
                for key, v, n in zip(keys, values, sizes):
                    ind, off = divmod(ind, n)
                    out[key] = v[off]
                return out
        raise IndexError("ParameterGrid index out of range")


class ParameterSampler:
    """Random parameter draws: sampling without replacement over an all-list
    space, else per-key ``rvs`` / uniform list choice."""

    def __init__(self, param_distributions, n_iter, *, random_state=None):
        if not isinstance(param_distributions, (Mapping, Iterable_)):
            raise TypeError("Parameter distribution is not a dict or a list ({!r})"
                            .format(param_distributions))
        if isinstance(param_distributions, Mapping):
            param_distributions = [param_distributions]
        for dist in param_distributions:
            if not isinstance(dist, dict):
                raise TypeError("Parameter distribution is not a dict ({!r})".format(dist))
            for key in dist:
                if not isinstance(dist[key], Iterable_) and not hasattr(dist[key], "rvs"):
                    raise TypeError("Parameter value is not iterable or distribution (key={!r}, "
                                    "value={!r})".format(key, dist[key]))
        self.n_iter = n_iter
        self.random_state = random_state
        self.param_distributions = param_distributions

    def _all_lists(self):
        return all(all(not hasattr(v, "rvs") for v in d.values())
                   for d in self.param_distributions)

    def __iter__(self):
        rng = check_random_state(self.random_state)
        if self._all_lists():
            grid = ParameterGrid(self.param_distributions)
            size = len(grid)
            n_iter = self.n_iter
            if size < n_iter:
                warnings.warn("The total space of parameters %d is smaller than n_iter=%d. "
                              "Running %d iterations. For exhaustive searches, use GridSearchCV."
                              % (size, self.n_iter, size), UserWarning)
                n_iter = size
            for i in sample_without_replacement(size, n_iter, random_state=rng):
                yield grid[i]
        else:
            for _ in range(self.n_iter):
                dist = rng.choice(self.param_distributions)
                params = {}
                for k, v in sorted(dist.items()):
                    params[k] = v.rvs(random_state=rng) if hasattr(v, "rvs") \
                        else v[rng.randint(len(v))]
                yield params

    def __len__(self):
        if self._all_lists():
            return min(self.n_iter, len(ParameterGrid(self.param_distributions)))
        return self.n_iter


def _scorers(scoring):
    if scoring is None or callable(scoring) or isinstance(scoring, str):
        return {"score": get_scorer(scoring)}, False
    if isinstance(scoring, dict):
        return {k: get_scorer(v) for k, v in scoring.items()}, True
    return {s: get_scorer(s) for s in scoring}, True


def _rank(a):
    """min-rank of -a with NaN last (reference _search.py _store ranking)."""
    a = np.asarray(a, dtype=float)
    key = np.where(np.isnan(a), np.inf, -a)
    order = np.argsort(key, kind="stable")
    ranks = np.empty(len(a), dtype=np.int32)
    sk = key[order]
    r = 1
    for i in range(len(a)):
        if i > 0 and sk[i] != sk[i - 1]:
            r = i + 1
        ranks[order[i]] = r
    return ranks


class BaseSearchCV(BaseEstimator):
    def __init__(self, estimator, *, scoring=None, n_jobs=None, refit=True, cv=None, verbose=0,
                 pre_dispatch="2*n_jobs", error_score=np.nan, return_train_score=False):
        self.estimator = estimator
        self.scoring = scoring
        self.n_jobs = n_jobs
        self.refit = refit
        self.cv = cv
        self.verbose = verbose
        self.pre_dispatch = pre_dispatch
        self.error_score = error_score
        self.return_train_score = return_train_score

    @property
    def _estimator_type(self):
        return getattr(self.estimator, "_estimator_type", None)

    def _evaluate(self, candidates, X, y, groups, fit_params, cv=None, scorers=None,
                  n_resources=None):
        cv = cv or check_cv(self.cv, y, classifier=is_classifier(self.estimator))
        splits = list(cv.split(X, y, groups))
        # every (candidate, fold) fit is one task (reference _search.py:795)
        flat = Parallel(n_jobs=self.n_jobs)(
            delayed(_fit_and_score)(clone(self.estimator).set_params(**params), X, y, train,
                                    test, scorers, fit_params, self.return_train_score,
                                    self.error_score)
            for params in candidates for train, test in splits)
        ns = len(splits)
        out = [flat[i * ns:(i + 1) * ns] for i in range(len(candidates))]
        return out, ns

    def _format_results(self, candidates, results, n_splits, scorers):
        res = {}
        nc = len(candidates)
        for key in ("fit_time", "score_time"):
            arr = np.array([[f[key] for f in r] for r in results])
            res["mean_" + key], res["std_" + key] = arr.mean(1), arr.std(1)
        masks = defaultdict(lambda: np.ma.MaskedArray(np.empty(nc, dtype=object),
                                                      mask=True))
        for i, p in enumerate(candidates):
            for name, val in p.items():
                masks["param_" + name][i] = val
        res.update(masks)
        res["params"] = candidates
        for m in scorers:
            suffix = "score" if not self.multimetric_ else m
            for split in ("test", "train") if self.return_train_score else ("test",):
                arr = np.array([[f[split][m] for f in r] for r in results], dtype=float)
                for s in range(n_splits):
                    res["split%d_%s_%s" % (s, split, suffix)] = arr[:, s]
                res["mean_%s_%s" % (split, suffix)] = arr.mean(1)
                res["std_%s_%s" % (split, suffix)] = arr.std(1)
                if split == "test":
                    res["rank_test_%s" % suffix] = _rank(arr.mean(1))
        return res

    def fit(self, X, y=None, *, groups=None, **fit_params):
        scorers, self.multimetric_ = _scorers(self.scoring)
        if self.multimetric_ and self.refit is not False and not callable(self.refit) \
                and self.refit not in scorers:
            raise ValueError("For multi-metric scoring, the parameter refit must be set to a "
                             "scorer key or a callable to refit an estimator with the best "
                             "parameter setting on the whole data and make the best_* "
                             "attributes available for that metric. If this is not needed, "
                             "refit should be set to False explicitly. %r was passed."
                             % self.refit)
        self.scorer_ = scorers if self.multimetric_ else scorers["score"]
        candidates, results, n_splits = self._run_search(X, y, groups, fit_params, scorers)
        self.cv_results_ = self._format_results(candidates, results, n_splits, scorers)
        self.n_splits_ = n_splits
        refit_metric = self.refit if self.multimetric_ else "score"
        if self.refit or not self.multimetric_:
            if callable(self.refit):
                self.best_index_ = int(self.refit(self.cv_results_))
            else:
                self.best_index_ = int(self.cv_results_["rank_test_%s" % refit_metric].argmin())
                self.best_score_ = float(
                    self.cv_results_["mean_test_%s" % refit_metric][self.best_index_])
            self.best_params_ = self.cv_results_["params"][self.best_index_]
        if self.refit:
            self.best_estimator_ = clone(clone(self.estimator).set_params(**self.best_params_))
            t0 = time.perf_counter()
            if y is None:
                self.best_estimator_.fit(X, **fit_params)
            else:
                self.best_estimator_.fit(X, y, **fit_params)
            self.refit_time_ = time.perf_counter() - t0
            if hasattr(self.best_estimator_, "classes_"):
                self.classes_ = self.best_estimator_.classes_
            if hasattr(self.best_estimator_, "n_features_in_"):
                self.n_features_in_ = self.best_estimator_.n_features_in_
        return self

    def _run_search(self, X, y, groups, fit_params, scorers):
        cands = list(self._candidates())
        results, n_splits = self._evaluate(cands, X, y, groups, fit_params, scorers=scorers)
        return cands, results, n_splits

    def score(self, X, y=None):
        scorer = self.scorer_[self.refit] if self.multimetric_ else self.scorer_
        return scorer(self.best_estimator_, X, y)

    def _best(self, name):
        if not self.refit:
            raise AttributeError("This %s instance was initialized with refit=False. %s is "
                                 "available only after refitting on the best parameters."
                                 % (type(self).__name__, name))
        return getattr(self.best_estimator_, name)

    # delegated methods exist only when the refitted estimator has them
    # (reference _search.py uses available_if for the same effect)
    predict = property(lambda self: self._best("predict"))
    predict_proba = property(lambda self: self._best("predict_proba"))
    predict_log_proba = property(lambda self: self._best("predict_log_proba"))
    decision_function = property(lambda self: self._best("decision_function"))
    transform = property(lambda self: self._best("transform"))
    inverse_transform = property(lambda self: self._best("inverse_transform"))
    score_samples = property(lambda self: self._best("score_samples"))


class GridSearchCV(BaseSearchCV):
    """Exhaustive search over ``param_grid``."""

    def __init__(self, estimator, param_grid, *, scoring=None, n_jobs=None, refit=True, cv=None,
                 verbose=0, pre_dispatch="2*n_jobs", error_score=np.nan,
                 return_train_score=False):
        super().__init__(estimator, scoring=scoring, n_jobs=n_jobs, refit=refit, cv=cv,
                         verbose=verbose, pre_dispatch=pre_dispatch, error_score=error_score,
                         return_train_score=return_train_score)
        self.param_grid = param_grid

    def _candidates(self):
        return ParameterGrid(self.param_grid)


class RandomizedSearchCV(BaseSearchCV):
    """Search over ``n_iter`` draws from ``param_distributions``."""

    def __init__(self, estimator, param_distributions, *, n_iter=10, scoring=None, n_jobs=None,
                 refit=True, cv=None, verbose=0, pre_dispatch="2*n_jobs", random_state=None,
                 error_score=np.nan, return_train_score=False):
        super().__init__(estimator, scoring=scoring, n_jobs=n_jobs, refit=refit, cv=cv,
                         verbose=verbose, pre_dispatch=pre_dispatch, error_score=error_score,
                         return_train_score=return_train_score)
        self.param_distributions = param_distributions
        self.n_iter = n_iter
        self.random_state = random_state

    def _candidates(self):
        return ParameterSampler(self.param_distributions, self.n_iter,
                                random_state=self.random_state)


class _SubsampleCV:
    """Wraps a CV so each train fold is subsampled to ``n`` samples
    (resource='n_samples' halving)."""

    def __init__(self, base, n, random_state, stratify):
        self.base, self.n, self.random_state, self.stratify = base, n, random_state, stratify

    def split(self, X, y=None, groups=None):
        for train, test in self.base.split(X, y, groups):
            rng = check_random_state(self.random_state)
            if self.n < len(train):
                if self.stratify and y is not None:
                    from ._split import StratifiedShuffleSplit
                    sss = StratifiedShuffleSplit(1, train_size=self.n, random_state=rng)
                    sub, _ = next(sss.split(np.zeros(len(train)), np.asarray(y)[train]))
                    train = train[np.sort(sub)]
                else:
                    train = np.sort(rng.choice(train, self.n, replace=False))
            yield train, test

    def get_n_splits(self, *a, **k):
        return self.base.get_n_splits(*a, **k)


class BaseSuccessiveHalving(BaseSearchCV):
    """Successive halving (reference _search_successive_halving.py): every
    iteration keeps the top 1/factor candidates and multiplies the
    resource budget by ``factor``."""

    def __init__(self, estimator, *, scoring=None, n_jobs=None, refit=True, cv=5, verbose=0,
                 random_state=None, error_score=np.nan, return_train_score=True,
                 max_resources="auto", min_resources="exhaust", resource="n_samples", factor=3,
                 aggressive_elimination=False):
        super().__init__(estimator, scoring=scoring, n_jobs=n_jobs, refit=refit, cv=cv,
                         verbose=verbose, error_score=error_score,
                         return_train_score=return_train_score)
        self.random_state = random_state
        self.max_resources = max_resources
        self.min_resources = min_resources
        self.resource = resource
        self.factor = factor
        self.aggressive_elimination = aggressive_elimination

    def _run_search(self, X, y, groups, fit_params, scorers):
        cands = list(self._candidates())
        n = X.shape[0] if hasattr(X, "shape") else len(X)
        max_res = n if self.max_resources == "auto" else int(self.max_resources)
        base_cv = check_cv(self.cv, y, classifier=is_classifier(self.estimator))
        n_splits = base_cv.get_n_splits(X, y, groups)
        if self.resource == "n_samples":
            min_small = 2 * n_splits * (len(np.unique(y)) if is_classifier(self.estimator)
                                        and y is not None else 1)
        else:
            min_small = 1
        if self.min_resources == "smallest":
            min_res = min_small
        elif self.min_resources == "exhaust":
            n_req = int(np.floor(np.log(max(len(cands), 1)) / np.log(self.factor))) + 1
            min_res = max(min_small, max_res // (self.factor ** (n_req - 1)))
        else:
            min_res = int(self.min_resources)
        n_possible = 1 + int(np.log(max_res / min_res) / np.log(self.factor)) \
            if max_res >= min_res else 1
        n_required = 1 + int(np.floor(np.log(max(len(cands), 1)) / np.log(self.factor)))
        n_iterations = min(n_possible, n_required) if not self.aggressive_elimination \
            else n_required
        self.n_resources_, self.n_candidates_ = [], []
        all_cands, all_results, iters = [], [], []
        rem = cands
        for it in range(n_iterations):
            power = it if not self.aggressive_elimination else max(0, it - n_required + n_possible)
            n_res = int(min(max_res, min_res * self.factor ** power))
            self.n_resources_.append(n_res)
            self.n_candidates_.append(len(rem))
            if self.resource == "n_samples":
                cv = _SubsampleCV(base_cv, n_res, self.random_state, is_classifier(self.estimator))
                params = rem
            else:
                cv = base_cv
                params = [dict(p, **{self.resource: n_res}) for p in rem]
            results, _ = self._evaluate(params, X, y, groups, fit_params, cv=cv, scorers=scorers)
            all_cands += params
            all_results += results
            iters += [it] * len(params)
            key = next(iter(scorers)) if not self.multimetric_ else self.refit
            means = np.array([np.mean([f["test"][key] for f in r]) for r in results])
            keep = max(1, int(np.ceil(len(rem) / self.factor)))
            order = np.argsort(-np.nan_to_num(means, nan=-np.inf), kind="stable")[:keep]
            rem = [rem[i] for i in order]
        self.n_iterations_ = n_iterations
        self.n_possible_iterations_ = n_possible
        self.n_required_iterations_ = n_required
        self.min_resources_, self.max_resources_ = min_res, max_res
        self._iters = np.array(iters)
        return all_cands, all_results, n_splits

    def _format_results(self, candidates, results, n_splits, scorers):
        res = super()._format_results(candidates, results, n_splits, scorers)
        res["iter"] = self._iters
        res["n_resources"] = np.array([self.n_resources_[i] for i in self._iters])
        # the winner must come from the last iteration (reference ranks by
        # iteration first, then score)
        key = "mean_test_score" if not self.multimetric_ else "mean_test_%s" % self.refit
        last = self._iters == self._iters.max()
        score = np.where(last, np.nan_to_num(res[key], nan=-np.inf), -np.inf)
        rk = "rank_test_score" if not self.multimetric_ else "rank_test_%s" % self.refit
        res[rk] = _rank(np.where(np.isinf(score), np.nan, score))
        if self.resource != "n_samples":
            res["params"] = [{k: v for k, v in p.items() if k != self.resource}
                             for p in res["params"]]
        return res


class HalvingGridSearchCV(BaseSuccessiveHalving):
    def __init__(self, estimator, param_grid, *, factor=3, resource="n_samples",
                 max_resources="auto", min_resources="exhaust", aggressive_elimination=False,
                 cv=5, scoring=None, refit=True, error_score=np.nan, return_train_score=True,
                 random_state=None, n_jobs=None, verbose=0):
        super().__init__(estimator, scoring=scoring, n_jobs=n_jobs, refit=refit, verbose=verbose,
                         cv=cv, random_state=random_state, error_score=error_score,
                         return_train_score=return_train_score, max_resources=max_resources,
                         resource=resource, factor=factor, min_resources=min_resources,
                         aggressive_elimination=aggressive_elimination)
        self.param_grid = param_grid

    def _candidates(self):
        return ParameterGrid(self.param_grid)


class HalvingRandomSearchCV(BaseSuccessiveHalving):
    def __init__(self, estimator, param_distributions, *, n_candidates="exhaust", factor=3,
                 resource="n_samples", max_resources="auto", min_resources="smallest",
                 aggressive_elimination=False, cv=5, scoring=None, refit=True,
                 error_score=np.nan, return_train_score=True, random_state=None, n_jobs=None,
                 verbose=0):
        super().__init__(estimator, scoring=scoring, n_jobs=n_jobs, refit=refit, verbose=verbose,
                         cv=cv, random_state=random_state, error_score=error_score,
                         return_train_score=return_train_score, max_resources=max_resources,
                         resource=resource, factor=factor, min_resources=min_resources,
                         aggressive_elimination=aggressive_elimination)
        self.param_distributions = param_distributions
        self.n_candidates = n_candidates

    def _candidates(self):
        n = self.n_candidates if self.n_candidates != "exhaust" else 10
        return ParameterSampler(self.param_distributions, n, random_state=self.random_state)


def _fit_score_once(est, X, y, train, test, scorer, fit_params):
    Xtr, ytr = _safe_index(X, train), _safe_index(y, train)
    if ytr is None:
        est.fit(Xtr, **fit_params)
    else:
        est.fit(Xtr, ytr, **fit_params)
    return scorer(est, _safe_index(X, test), _safe_index(y, test))


def permutation_test_score(estimator, X, y, *, groups=None, cv=None, n_permutations=100,
                           n_jobs=None, random_state=0, verbose=0, scoring=None, fit_params=None):
    """CV score, scores under permuted labels, and the p-value."""
    cv = check_cv(cv, y, classifier=is_classifier(estimator))
    scorer = get_scorer(scoring)
    rng = check_random_state(random_state)
    fit_params = fit_params or {}

    def cv_score(yy):
        return np.mean([_fit_score_once(clone(estimator), X, yy, tr, te, scorer, fit_params)
                        for tr, te in cv.split(X, yy, groups)])

    def shuffle(yy):
        if groups is None:
            return yy[rng.permutation(len(yy))]
        idx = np.arange(len(groups))
        g = np.asarray(groups)
        for grp in np.unique(g):
            m = g == grp
            idx[m] = rng.permutation(idx[m])
        return yy[idx]

    y = np.asarray(y)
    # the permutations are drawn in order (same stream as sequential), then
    # the n_permutations + 1 cross-validations run as parallel tasks
    ys = [y] + [shuffle(y) for _ in range(n_permutations)]
    scores = Parallel(n_jobs=n_jobs)(delayed(cv_score)(yy) for yy in ys)
    score, perm = scores[0], np.array(scores[1:])
    pvalue = (np.sum(perm >= score) + 1.0) / (n_permutations + 1)
    return score, perm, pvalue


def _translate_train_sizes(train_sizes, n_max):
    ts = np.asarray(train_sizes)
    if np.issubdtype(ts.dtype, np.floating):
        if ts.min() <= 0 or ts.max() > 1:
            raise ValueError("train_sizes has been interpreted as fractions of the maximum "
                             "number of training samples and must be within (0, 1], but is "
                             "within [%f, %f]." % (ts.min(), ts.max()))
        abs_ = (ts * n_max).astype(dtype=int, copy=False)
        abs_ = np.clip(abs_, 1, n_max)
    else:
        if ts.min() <= 0 or ts.max() > n_max:
            raise ValueError("train_sizes has been interpreted as absolute numbers of training "
                             "samples and must be within (0, %d], but is within [%d, %d]."
                             % (n_max, ts.min(), ts.max()))
        abs_ = ts
    uniq = np.unique(abs_)
    if len(uniq) != len(abs_):
        warnings.warn("Removed duplicate entries from 'train_sizes'. Number of ticks will be "
                      "less than the size of 'train_sizes': %d instead of %d."
                      % (len(uniq), len(abs_)), RuntimeWarning)
    return uniq


def learning_curve(estimator, X, y, *, groups=None, train_sizes=np.linspace(0.1, 1.0, 5), cv=None,
                   scoring=None, exploit_incremental_learning=False, n_jobs=None,
                   pre_dispatch="all", verbose=0, shuffle=False, random_state=None,
                   error_score=np.nan, return_times=False, fit_params=None):
    """Train/test scores for growing training-set sizes."""
    cv = check_cv(cv, y, classifier=is_classifier(estimator))
    splits = list(cv.split(X, y, groups))
    scorer = get_scorer(scoring)
    n_max = len(splits[0][0])
    sizes = _translate_train_sizes(train_sizes, n_max)
    rng = check_random_state(random_state)
    if shuffle:
        splits = [(rng.permutation(tr), te) for tr, te in splits]
    train_scores = np.zeros((len(sizes), len(splits)))
    test_scores = np.zeros_like(train_scores)
    fit_times = np.zeros_like(train_scores)
    score_times = np.zeros_like(train_scores)
    jobs = [(i, j) for j in range(len(splits)) for i in range(len(sizes))]
    res = Parallel(n_jobs=n_jobs)(
        delayed(_fit_and_score)(clone(estimator), X, y, splits[j][0][:sizes[i]], splits[j][1],
                                {"s": scorer}, fit_params or {}, True, error_score)
        for i, j in jobs)
    for (i, j), r in zip(jobs, res):
        train_scores[i, j], test_scores[i, j] = r["train"]["s"], r["test"]["s"]
        fit_times[i, j], score_times[i, j] = r["fit_time"], r["score_time"]
    if return_times:
        return sizes, train_scores, test_scores, fit_times, score_times
    return sizes, train_scores, test_scores


def validation_curve(estimator, X, y, *, param_name, param_range, groups=None, cv=None,
                     scoring=None, n_jobs=None, pre_dispatch="all", verbose=0,
                     error_score=np.nan, fit_params=None):
    """Train/test scores across values of one parameter."""
    cv = check_cv(cv, y, classifier=is_classifier(estimator))
    splits = list(cv.split(X, y, groups))
    scorer = get_scorer(scoring)
    tr_s = np.zeros((len(param_range), len(splits)))
    te_s = np.zeros_like(tr_s)
    jobs = [(i, j) for i in range(len(param_range)) for j in range(len(splits))]
    res = Parallel(n_jobs=n_jobs)(
        delayed(_fit_and_score)(clone(estimator).set_params(**{param_name: param_range[i]}), X,
                                y, splits[j][0], splits[j][1], {"s": scorer}, fit_params or {},
                                True, error_score)
        for i, j in jobs)
    for (i, j), r in zip(jobs, res):
        tr_s[i, j], te_s[i, j] = r["train"]["s"], r["test"]["s"]
    return tr_s, te_s


def fit_grid_point(X, y, estimator, parameters, train, test, scorer, verbose,
                   error_score=np.nan, **fit_params):
    """Fit one parameter setting on one split and score it (reference
    ``_search.py:330``, deprecated there): returns (score, parameters,
    n_test_samples); ``scorer`` may be a callable or a dict of them (the
    score is then a dict)."""
    import warnings as _w
    _w.warn("fit_grid_point is deprecated in 0.23 and will be removed in 1.0 (renaming of "
            "0.25).", FutureWarning)
    multi = isinstance(scorer, dict)
    scorers = scorer if multi else {"score": scorer}
    est = clone(estimator).set_params(**parameters)
    r = _fit_and_score(est, X, y, train, test, scorers, fit_params, False, error_score)
    score = r["test"] if multi else r["test"]["score"]
    return score, parameters, len(test)


__all__ = ["ParameterGrid", "ParameterSampler", "GridSearchCV", "RandomizedSearchCV",
           "HalvingGridSearchCV", "HalvingRandomSearchCV", "permutation_test_score",
           "learning_curve", "validation_curve", "fit_grid_point"]
