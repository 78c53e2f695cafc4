"""Feature selection (reference ``sklearn/feature_selection``: univariate
scores ``f_classif`` / ``f_regression`` / ``chi2`` / ``r_regression``,
SelectKBest, SelectPercentile, SelectFpr / SelectFdr / SelectFwe,
GenericUnivariateSelect, VarianceThreshold, RFE / RFECV, SelectFromModel,
SequentialFeatureSelector, mutual information estimators)."""

import numbers
import warnings

import numpy as np
from scipy import special, stats

from .base import BaseEstimator, TransformerMixin, clone, is_classifier
from .utils.validation import check_is_fitted


def _dense(X):
    if hasattr(X, "detach"):
        X = X.detach().cpu().numpy()
    if hasattr(X, "toarray"):
        X = X.toarray()
    return np.asarray(X, dtype=np.float64)


# ------------------------------------------------------------ score functions
def f_oneway(*args):
    n_classes = len(args)
    args = [np.asarray(a, dtype=np.float64) for a in args]
    n_samples_per_class = np.array([a.shape[0] for a in args])
    n_samples = np.sum(n_samples_per_class)
    ss_alldata = sum((a ** 2).sum(axis=0) for a in args)
    sums_args = [np.asarray(a.sum(axis=0)) for a in args]
    square_of_sums_alldata = sum(sums_args) ** 2
    square_of_sums_args = [s ** 2 for s in sums_args]
    sstot = ss_alldata - square_of_sums_alldata / float(n_samples)
    ssbn = 0.0
    for k, _ in enumerate(args):
        ssbn += square_of_sums_args[k] / n_samples_per_class[k]
    ssbn -= square_of_sums_alldata / float(n_samples)
    sswn = sstot - ssbn
    dfbn = n_classes - 1
    dfwn = n_samples - n_classes
    msb = ssbn / float(dfbn)
    msw = sswn / float(dfwn)
    constant = np.where(np.abs(msw) == 0)[0]
    if constant.size and (msb[constant] != 0).any():
        warnings.warn("Features %s are constant." % constant, UserWarning)
    with np.errstate(divide="ignore", invalid="ignore"):
        f = msb / msw
    f = np.asarray(f).ravel()
    prob = special.fdtrc(dfbn, dfwn, f)
    return f, prob


def f_classif(X, y):
    X = _dense(X)
    y = np.asarray(y)
    return f_oneway(*[X[y == k] for k in np.unique(y)])


def chi2(X, y):
    X = _dense(X)
    if np.any(X < 0):
        raise ValueError("Input X must be non-negative.")
    from .preprocessing import LabelBinarizer
    Y = LabelBinarizer().fit_transform(y).astype(np.float64)
    if Y.shape[1] == 1:
        Y = np.append(1 - Y, Y, axis=1)
    observed = Y.T @ X
    feature_count = X.sum(axis=0).reshape(1, -1)
    class_prob = Y.mean(axis=0).reshape(1, -1)
    expected = class_prob.T @ feature_count
    with np.errstate(divide="ignore", invalid="ignore"):
        chisq = ((observed - expected) ** 2 / expected).sum(axis=0)
    return chisq, special.chdtrc(len(observed) - 1, chisq)


def r_regression(X, y, *, center=True):
    X = _dense(X)
    y = np.asarray(y, dtype=np.float64)
    if center:
        y = y - y.mean()
        X_means = X.mean(axis=0)
        X_norms = np.sqrt(((X - X_means) ** 2).sum(axis=0))
    else:
        X_norms = np.sqrt((X ** 2).sum(axis=0))
    corr = (y @ X) if not center else (y @ (X - X_means))
    with np.errstate(divide="ignore", invalid="ignore"):
        corr /= X_norms
        corr /= np.linalg.norm(y)
    return corr


def f_regression(X, y, *, center=True):
    corr = r_regression(X, y, center=center)
    deg = len(y) - (2 if center else 1)
    corr2 = corr ** 2
    with np.errstate(divide="ignore", invalid="ignore"):
        F = corr2 / (1 - corr2) * deg
    pv = stats.f.sf(F, 1, deg)
    return F, pv


def mutual_info_regression(X, y, *, discrete_features="auto", n_neighbors=3, copy=True,
                           random_state=None):
    return _estimate_mi(X, y, discrete_features, False, n_neighbors, random_state)


def mutual_info_classif(X, y, *, discrete_features="auto", n_neighbors=3, copy=True,
                        random_state=None):
    return _estimate_mi(X, y, discrete_features, True, n_neighbors, random_state)


def _estimate_mi(X, y, discrete_features, discrete_target, n_neighbors, random_state):
    """Kraskov (continuous) / Ross (mixed) kNN estimators (reference
    ``feature_selection/_mutual_info.py``)."""
    from scipy.special import digamma
    from .utils.validation import check_random_state
    X = _dense(X)
    y = np.asarray(y)
    n, d = X.shape
    rng = check_random_state(random_state)
    if isinstance(discrete_features, str) and discrete_features == "auto":
        discrete = np.zeros(d, dtype=bool)
    elif isinstance(discrete_features, (bool, np.bool_)):
        discrete = np.full(d, bool(discrete_features))
    else:
        discrete = np.zeros(d, dtype=bool)
        discrete[np.asarray(discrete_features)] = True
    Xs = X.copy()
    cont = ~discrete
    if cont.any():
        Xs[:, cont] = Xs[:, cont] / np.std(Xs[:, cont], axis=0)
        means = np.maximum(1, np.mean(np.abs(Xs[:, cont]), axis=0))
        Xs[:, cont] += 1e-10 * means * rng.standard_normal(size=(n, cont.sum()))
    if not discrete_target:
        y = y.astype(np.float64)
        y = y / np.std(y)
        y += 1e-10 * max(1, np.mean(np.abs(y))) * rng.standard_normal(size=n)
    out = np.zeros(d)
    for j in range(d):
        x = Xs[:, j]
        if discrete[j] and discrete_target:
            from .utils.cluster_metrics import mutual_info_score
            out[j] = mutual_info_score(x, y)
        elif discrete_target or discrete[j]:
            c, dv = (x, y) if discrete_target else (y, x)
            radius = np.empty(n)
            label_counts = np.empty(n)
            k_all = np.empty(n)
            for lab in np.unique(dv):
                m = dv == lab
                cnt = m.sum()
                if cnt > 1:
                    k = min(n_neighbors, cnt - 1)
                    cc = c[m]
                    dist = np.abs(cc[:, None] - cc[None, :])
                    radius[m] = np.nextafter(np.sort(dist, axis=1)[:, k], 0)
                    k_all[m] = k
                label_counts[m] = cnt
            keep = label_counts > 1
            nn = keep.sum()
            cc = c[keep]
            m_all = np.array([np.sum(np.abs(cc - cc[i]) <= radius[keep][i]) for i in range(nn)])
            mi = (digamma(nn) + np.mean(digamma(k_all[keep])) - np.mean(digamma(label_counts[keep]))
                  - np.mean(digamma(m_all)))
            out[j] = max(0.0, mi)
        else:
            xy = np.c_[x, y]
            dist = np.max(np.abs(xy[:, None, :] - xy[None, :, :]), axis=2)
            radius = np.nextafter(np.sort(dist, axis=1)[:, n_neighbors], 0)
            nx = np.array([np.sum(np.abs(x - x[i]) <= radius[i]) for i in range(n)]) - 1
            ny = np.array([np.sum(np.abs(y - y[i]) <= radius[i]) for i in range(n)]) - 1
            mi = (digamma(n) + digamma(n_neighbors) - np.mean(digamma(nx + 1))
                  - np.mean(digamma(ny + 1)))
            out[j] = max(0.0, mi)
    return out


# ------------------------------------------------------------- selectors
class SelectorMixin(TransformerMixin):
    def get_support(self, indices=False):
        mask = self._get_support_mask()
        return mask if not indices else np.where(mask)[0]

    def transform(self, X):
        X = _dense(X)
        mask = self.get_support()
        if X.shape[1] != len(mask):
            raise ValueError("X has a different shape than during fitting.")
        if not mask.any():
            warnings.warn("No features were selected: either the data is too noisy or the "
                          "selection test too strict.", UserWarning)
            return np.empty(0).reshape((X.shape[0], 0))
        return X[:, mask]

    def inverse_transform(self, X):
        X = _dense(X)
        support = self.get_support()
        out = np.zeros((X.shape[0], support.size), dtype=X.dtype)
        out[:, support] = X
        return out

    def get_feature_names_out(self, input_features=None):
        names = np.asarray(input_features) if input_features is not None else \
            np.array(["x%d" % i for i in range(len(self.get_support()))], dtype=object)
        return names[self.get_support()]


class _BaseFilter(SelectorMixin, BaseEstimator):
    def fit(self, X, y):
        X = _dense(X)
        self.n_features_in_ = X.shape[1]
        if not callable(self.score_func):
            raise TypeError("The score function should be a callable, %s (%s) was passed."
                            % (self.score_func, type(self.score_func)))
        self._check_params(X, y)
        res = self.score_func(X, y)
        if isinstance(res, (list, tuple)):
            self.scores_, self.pvalues_ = res
            self.pvalues_ = np.asarray(self.pvalues_)
        else:
            self.scores_, self.pvalues_ = res, None
        self.scores_ = np.asarray(self.scores_)
        return self

    def _check_params(self, X, y):
        pass


def _clean_nans(scores):
    scores = np.array(scores, dtype=np.float64)
    scores[np.isnan(scores)] = np.finfo(scores.dtype).min
    return scores


class SelectPercentile(_BaseFilter):
    def __init__(self, score_func=f_classif, *, percentile=10):
        self.score_func = score_func
        self.percentile = percentile

    def _check_params(self, X, y):
        if not 0 <= self.percentile <= 100:
            raise ValueError("percentile should be >=0, <=100; got %r" % self.percentile)

    def _get_support_mask(self):
        check_is_fitted(self)
        if self.percentile == 100:
            return np.ones(len(self.scores_), dtype=bool)
        if self.percentile == 0:
            return np.zeros(len(self.scores_), dtype=bool)
        scores = _clean_nans(self.scores_)
        threshold = np.percentile(scores, 100 - self.percentile)
        mask = scores > threshold
        ties = np.where(scores == threshold)[0]
        if len(ties):
            max_feats = int(len(scores) * self.percentile / 100)
            kept_ties = ties[:max_feats - mask.sum()]
            mask[kept_ties] = True
        return mask


class SelectKBest(_BaseFilter):
    def __init__(self, score_func=f_classif, *, k=10):
        self.score_func = score_func
        self.k = k

    def _check_params(self, X, y):
        if not (self.k == "all" or 0 <= self.k <= X.shape[1]):
            raise ValueError("k should be >=0, <= n_features = %d; got %r. Use k='all' to return "
                             "all features." % (X.shape[1], self.k))

    def _get_support_mask(self):
        check_is_fitted(self)
        if self.k == "all":
            return np.ones(self.scores_.shape, dtype=bool)
        if self.k == 0:
            return np.zeros(self.scores_.shape, dtype=bool)
        scores = _clean_nans(self.scores_)
        mask = np.zeros(scores.shape, dtype=bool)
        mask[np.argsort(scores, kind="mergesort")[-self.k:]] = 1
        return mask


class SelectFpr(_BaseFilter):
    def __init__(self, score_func=f_classif, *, alpha=5e-2):
        self.score_func = score_func
        self.alpha = alpha

    def _get_support_mask(self):
        return self.pvalues_ < self.alpha


class SelectFdr(_BaseFilter):
    def __init__(self, score_func=f_classif, *, alpha=5e-2):
        self.score_func = score_func
        self.alpha = alpha

    def _get_support_mask(self):
        n = len(self.pvalues_)
        sv = np.sort(self.pvalues_)
        selected = sv[sv <= float(self.alpha) / n * np.arange(1, n + 1)]
        if selected.size == 0:
            return np.zeros_like(self.pvalues_, dtype=bool)
        return self.pvalues_ <= selected.max()


class SelectFwe(_BaseFilter):
    def __init__(self, score_func=f_classif, *, alpha=5e-2):
        self.score_func = score_func
        self.alpha = alpha

    def _get_support_mask(self):
        return self.pvalues_ < self.alpha / len(self.pvalues_)


class GenericUnivariateSelect(_BaseFilter):
    _modes = {"percentile": SelectPercentile, "k_best": SelectKBest, "fpr": SelectFpr,
              "fdr": SelectFdr, "fwe": SelectFwe}

    def __init__(self, score_func=f_classif, *, mode="percentile", param=1e-5):
        self.score_func = score_func
        self.mode = mode
        self.param = param

    def _make_selector(self):
        sel = self._modes[self.mode](score_func=self.score_func)
        key = [p for p in sel.get_params() if p != "score_func"][0]
        sel.set_params(**{key: self.param})
        return sel

    def _get_support_mask(self):
        sel = self._make_selector()
        sel.pvalues_, sel.scores_ = self.pvalues_, self.scores_
        return sel._get_support_mask()


class VarianceThreshold(SelectorMixin, BaseEstimator):

    def _more_tags(self):
        return {"allow_nan": True}

    def __init__(self, threshold=0.0):
        self.threshold = threshold

    def fit(self, X, y=None):
        X = _dense(X)
        self.n_features_in_ = X.shape[1]
        self.variances_ = np.nanvar(X, axis=0)
        if self.threshold == 0:
            peak = np.ptp(X, axis=0)
            self.variances_ = np.nanmin([self.variances_, peak], axis=0)
        if np.all(~np.isfinite(self.variances_) | (self.variances_ <= self.threshold)):
            msg = "No feature in X meets the variance threshold {0:.5f}"
            if X.shape[0] == 1:
                msg += " (X contains only one sample)"
            raise ValueError(msg.format(self.threshold))
        return self

    def _get_support_mask(self):
        check_is_fitted(self)
        return self.variances_ > self.threshold


def _importances(est, getter="auto", transform_func=None):
    if getter == "auto":
        if hasattr(est, "coef_"):
            imp = np.abs(np.asarray(est.coef_))
            if imp.ndim > 1:
                imp = np.linalg.norm(imp, axis=0, ord=1)
        elif hasattr(est, "feature_importances_"):
            imp = np.asarray(est.feature_importances_)
        else:
            raise ValueError("when `importance_getter=='auto'`, the underlying estimator %s "
                             "should have `coef_` or `feature_importances_` attribute."
                             % est.__class__.__name__)
    elif callable(getter):
        imp = np.asarray(getter(est))
    else:
        obj = est
        for a in getter.split("."):
            obj = getattr(obj, a)
        imp = np.asarray(obj)
        if imp.ndim > 1:
            imp = np.linalg.norm(imp, axis=0, ord=1)
    return imp


class SelectFromModel(SelectorMixin, BaseEstimator):
    def __init__(self, estimator, *, threshold=None, prefit=False, norm_order=1,
                 max_features=None, importance_getter="auto"):
        self.estimator = estimator
        self.threshold = threshold
        self.prefit = prefit
        self.importance_getter = importance_getter
        self.norm_order = norm_order
        self.max_features = max_features

    def _threshold(self, imp):
        t = self.threshold
        if t is None:
            est_name = type(self.estimator).__name__
            t = 1e-5 if ("Lasso" in est_name or getattr(self.estimator, "penalty", None) == "l1") \
                else "mean"
        if isinstance(t, str):
            if "*" in t:
                scale, ref = t.split("*")
                scale = float(scale.strip())
                ref = ref.strip()
            else:
                scale, ref = 1.0, t
            ref = np.median(imp) if ref == "median" else (np.mean(imp) if ref == "mean" else None)
            if ref is None:
                raise ValueError("Expected threshold='mean' or threshold='median' got %s" % t)
            return scale * ref
        return float(t)

    def _get_support_mask(self):
        est = self.estimator_ if hasattr(self, "estimator_") else self.estimator
        imp = _importances(est, self.importance_getter)
        thr = self._threshold(imp)
        mask = imp >= thr
        if self.max_features is not None:
            mask = np.zeros_like(imp, dtype=bool)
            top = np.argsort(-imp, kind="mergesort")[:self.max_features]
            mask[top] = True
            mask &= imp >= thr
        return mask

    @property
    def threshold_(self):
        est = self.estimator_ if hasattr(self, "estimator_") else self.estimator
        return self._threshold(_importances(est, self.importance_getter))

    def fit(self, X, y=None, **fit_params):
        if self.prefit:
            raise ValueError("Either fit the model before transform or set 'prefit=True' while "
                             "passing the fitted estimator to the constructor.")
        self.estimator_ = clone(self.estimator).fit(X, y, **fit_params)
        self.n_features_in_ = _dense(X).shape[1]
        return self

    def partial_fit(self, X, y=None, **fit_params):
        if not hasattr(self, "estimator_"):
            self.estimator_ = clone(self.estimator)
        self.estimator_.partial_fit(X, y, **fit_params)
        return self


class RFE(SelectorMixin, BaseEstimator):
    def __init__(self, estimator, *, n_features_to_select=None, step=1, verbose=0,
                 importance_getter="auto"):
        self.estimator = estimator
        self.n_features_to_select = n_features_to_select
        self.step = step
        self.importance_getter = importance_getter
        self.verbose = verbose

    @property
    def classes_(self):
        return self.estimator_.classes_

    def fit(self, X, y, **fit_params):
        return self._fit(X, y, **fit_params)

    def _fit(self, X, y, step_score=None, **fit_params):
        X = _dense(X)
        n_features = X.shape[1]
        self.n_features_in_ = n_features
        if self.n_features_to_select is None:
            n_sel = n_features // 2
        elif isinstance(self.n_features_to_select, numbers.Integral):
            n_sel = self.n_features_to_select
        else:
            n_sel = int(n_features * self.n_features_to_select)
        step = int(max(1, self.step * n_features)) if 0.0 < self.step < 1.0 else int(self.step)
        if step <= 0:
            raise ValueError("Step must be >0")
        support = np.ones(n_features, dtype=bool)
        ranking = np.ones(n_features, dtype=int)
        if step_score:
            self.scores_ = []
        while np.sum(support) > n_sel:
            features = np.arange(n_features)[support]
            est = clone(self.estimator)
            est.fit(X[:, features], y, **fit_params)
            imp = _importances(est, self.importance_getter)
            ranks = np.ravel(np.argsort(imp, kind="mergesort"))
            threshold = min(step, np.sum(support) - n_sel)
            if step_score:
                self.scores_.append(step_score(est, features))
            support[features[ranks][:threshold]] = False
            ranking[np.logical_not(support)] += 1
        features = np.arange(n_features)[support]
        self.estimator_ = clone(self.estimator).fit(X[:, features], y, **fit_params)
        if step_score:
            self.scores_.append(step_score(self.estimator_, features))
        self.n_features_ = support.sum()
        self.support_ = support
        self.ranking_ = ranking
        return self

    def _get_support_mask(self):
        check_is_fitted(self)
        return self.support_

    def predict(self, X):
        return self.estimator_.predict(self.transform(X))

    def score(self, X, y, **kw):
        return self.estimator_.score(self.transform(X), y, **kw)

    def decision_function(self, X):
        return self.estimator_.decision_function(self.transform(X))

    def predict_proba(self, X):
        return self.estimator_.predict_proba(self.transform(X))


class RFECV(RFE):
    def __init__(self, estimator, *, step=1, min_features_to_select=1, cv=None, scoring=None,
                 verbose=0, n_jobs=None, importance_getter="auto"):
        self.estimator = estimator
        self.step = step
        self.importance_getter = importance_getter
        self.cv = cv
        self.scoring = scoring
        self.verbose = verbose
        self.n_jobs = n_jobs
        self.min_features_to_select = min_features_to_select

    def fit(self, X, y, groups=None):
        from .metrics import check_scoring
        from .model_selection import check_cv
        X = _dense(X)
        y = np.asarray(y)
        cv = check_cv(self.cv, y, classifier=is_classifier(self.estimator))
        scorer = check_scoring(self.estimator, scoring=self.scoring)
        n_features = X.shape[1]
        step = int(max(1, self.step * n_features)) if 0.0 < self.step < 1.0 else int(self.step)
        all_scores = []
        for tr, te in cv.split(X, y):
            rfe = RFE(self.estimator, n_features_to_select=self.min_features_to_select,
                      importance_getter=self.importance_getter, step=self.step)
            rfe._fit(X[tr], y[tr], lambda est, feats: scorer(est, X[te][:, feats], y[te]))
            all_scores.append(rfe.scores_[::-1])
        scores = np.array(all_scores)
        scores_sum = np.sum(scores, axis=0)
        n_features_to_select = max(n_features - (np.argmax(scores_sum[::-1]) * step),
                                   self.min_features_to_select)
        rfe = RFE(self.estimator, n_features_to_select=n_features_to_select, step=self.step,
                  importance_getter=self.importance_getter).fit(X, y)
        self.support_ = rfe.support_
        self.n_features_ = rfe.n_features_
        self.ranking_ = rfe.ranking_
        self.estimator_ = rfe.estimator_
        self.n_features_in_ = n_features
        self.cv_results_ = {"mean_test_score": scores.mean(0), "std_test_score": scores.std(0)}
        self.grid_scores_ = scores.T
        return self


class SequentialFeatureSelector(SelectorMixin, BaseEstimator):
    def __init__(self, estimator, *, n_features_to_select=None, direction="forward",
                 scoring=None, cv=5, n_jobs=None):
        self.estimator = estimator
        self.n_features_to_select = n_features_to_select
        self.direction = direction
        self.scoring = scoring
        self.cv = cv
        self.n_jobs = n_jobs

    def fit(self, X, y=None):
        from .model_selection import cross_val_score
        X = _dense(X)
        n_features = X.shape[1]
        self.n_features_in_ = n_features
        if self.n_features_to_select is None:
            k = n_features // 2
        elif isinstance(self.n_features_to_select, numbers.Integral):
            k = self.n_features_to_select
        else:
            k = int(n_features * self.n_features_to_select)
        if self.direction not in ("forward", "backward"):
            raise ValueError("direction must be either 'forward' or 'backward'. Got %s."
                             % self.direction)
        current = np.zeros(n_features, dtype=bool)
        n_iter = k if self.direction == "forward" else n_features - k
        for _ in range(n_iter):
            cands = np.flatnonzero(~current)
            scores = {}
            for f in cands:
                mask = current.copy()
                mask[f] = True
                if self.direction == "backward":
                    mask = ~mask
                scores[f] = cross_val_score(clone(self.estimator), X[:, mask], y, cv=self.cv,
                                            scoring=self.scoring).mean()
            best = max(scores, key=lambda f: scores[f])
            current[best] = True
        if self.direction == "backward":
            current = ~current
        self.support_ = current
        self.n_features_to_select_ = int(current.sum())
        return self

    def _get_support_mask(self):
        check_is_fitted(self)
        return self.support_


__all__ = ["f_classif", "f_regression", "r_regression", "chi2", "f_oneway",
           "mutual_info_regression", "mutual_info_classif", "SelectKBest", "SelectPercentile",
           "SelectFpr", "SelectFdr", "SelectFwe", "GenericUnivariateSelect", "VarianceThreshold",
           "SelectFromModel", "RFE", "RFECV", "SequentialFeatureSelector", "SelectorMixin"]

from .utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
