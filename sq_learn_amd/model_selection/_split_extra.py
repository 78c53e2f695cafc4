"""Remaining CV splitters (reference ``model_selection/_split.py``):
``LeaveOneOut`` :125, ``LeavePOut`` :203, ``GroupKFold`` :453,
``StratifiedGroupKFold`` :718, ``TimeSeriesSplit`` :870,
``LeaveOneGroupOut`` :997, ``LeavePGroupsOut`` :1096, ``_RepeatedSplits``
:1220, ``RepeatedKFold`` :1302, ``RepeatedStratifiedKFold`` :1353,
``GroupShuffleSplit`` :1582, ``PredefinedSplit`` :1934.

Index bookkeeping only; the same seeds yield the same folds as the
reference."""

import itertools
import numbers
from collections import defaultdict

import numpy as np

from ..runtime.device import to_numpy
from ..utils.validation import check_random_state
from ._split import (BaseCrossValidator, KFold, ShuffleSplit, StratifiedKFold, _BaseKFold,
                     _indexable_len)


def _groups(groups):
    if groups is None:
        raise ValueError("The 'groups' parameter should not be None.")
    return np.asarray(to_numpy(groups)).reshape(-1)


class LeaveOneOut(BaseCrossValidator):
    def _iter_test_indices(self, X, y=None, groups=None):
        n = _indexable_len(X)
        if n <= 1:
            raise ValueError("Cannot perform LeaveOneOut with n_samples={}.".format(n))
        return range(n)

    def get_n_splits(self, X, y=None, groups=None):
        if X is None:
            raise ValueError("The 'X' parameter should not be None.")
        return _indexable_len(X)


class LeavePOut(BaseCrossValidator):
    def __init__(self, p):
        self.p = p

    def _iter_test_indices(self, X, y=None, groups=None):
        n = _indexable_len(X)
        if n <= self.p:
            raise ValueError("p={} must be strictly less than the number of samples={}"
                             .format(self.p, n))
        for comb in itertools.combinations(range(n), self.p):
            yield np.array(comb)

    def get_n_splits(self, X, y=None, groups=None):
        from math import comb
        if X is None:
            raise ValueError("The 'X' parameter should not be None.")
        return comb(_indexable_len(X), self.p)


class GroupKFold(_BaseKFold):
    """Non-overlapping groups, folds balanced greedily by group size."""

    def __init__(self, n_splits=5):
        super().__init__(n_splits, shuffle=False, random_state=None)

    def _iter_test_indices(self, X, y, groups):
        groups = _groups(groups)
        unique, gidx = np.unique(groups, return_inverse=True)
        if self.n_splits > len(unique):
            raise ValueError("Cannot have number of splits n_splits=%d greater than the number "
                             "of groups: %d." % (self.n_splits, len(unique)))
        per_group = np.bincount(gidx)
        order = np.argsort(per_group)[::-1]
        per_group = per_group[order]
        per_fold = np.zeros(self.n_splits)
        group_to_fold = np.zeros(len(unique))
        for gi, w in enumerate(per_group):
            light = np.argmin(per_fold)
            per_fold[light] += w
            group_to_fold[order[gi]] = light
        fold_of = group_to_fold[gidx]
        for f in range(self.n_splits):
            yield np.where(fold_of == f)[0]

    def split(self, X, y=None, groups=None):
        return super().split(X, y, groups)


class StratifiedGroupKFold(_BaseKFold):
    """Groups kept whole while folds approximate the class distribution
    (greedy assignment minimising the std of per-class fold fractions)."""

    def __init__(self, n_splits=5, shuffle=False, random_state=None):
        super().__init__(n_splits=n_splits, shuffle=shuffle, random_state=random_state)

    def _iter_test_indices(self, X, y, groups):
        rng = check_random_state(self.random_state)
        y = np.asarray(to_numpy(y)).reshape(-1)
        _, y_inv, y_cnt = np.unique(y, return_inverse=True, return_counts=True)
        if np.all(self.n_splits > y_cnt):
            raise ValueError("n_splits=%d cannot be greater than the number of members in each "
                             "class." % self.n_splits)
        groups = _groups(groups)
        _, g_inv, g_cnt = np.unique(groups, return_inverse=True, return_counts=True)
        y_counts_per_group = np.zeros((len(g_cnt), len(y_cnt)))
        for ci, gi in zip(y_inv, g_inv):
            y_counts_per_group[gi, ci] += 1
        y_counts_per_fold = np.zeros((self.n_splits, len(y_cnt)))
        groups_per_fold = defaultdict(set)
        if self.shuffle:
            rng.shuffle(y_counts_per_group)
        order = np.argsort(-np.std(y_counts_per_group, axis=1), kind="mergesort")
        for gi in order:
            gy = y_counts_per_group[gi]
            best_fold, min_eval, min_samples = None, np.inf, None
            for f in range(self.n_splits):
                y_counts_per_fold[f] += gy
                std = np.std(y_counts_per_fold / y_cnt.reshape(1, -1), axis=0)
                y_counts_per_fold[f] -= gy
                ev = np.mean(std)
                ns = np.sum(y_counts_per_fold[f])
                if ev < min_eval or (np.isclose(ev, min_eval) and ns < min_samples):
                    min_eval, min_samples, best_fold = ev, ns, f
            y_counts_per_fold[best_fold] += gy
            groups_per_fold[best_fold].add(gi)
        for f in range(self.n_splits):
            yield [i for i, g in enumerate(g_inv) if g in groups_per_fold[f]]


class TimeSeriesSplit(_BaseKFold):
    """Expanding-window splits for ordered samples, optional gap and cap."""

    def __init__(self, n_splits=5, *, max_train_size=None, test_size=None, gap=0):
        super().__init__(n_splits, shuffle=False, random_state=None)
        self.max_train_size = max_train_size
        self.test_size = test_size
        self.gap = gap

    def split(self, X, y=None, groups=None):
        n = _indexable_len(X)
        n_splits, gap = self.n_splits, self.gap
        n_folds = n_splits + 1
        test_size = self.test_size if self.test_size is not None else n // n_folds
        if n_folds > n:
            raise ValueError(f"Cannot have number of folds={n_folds} greater than the number of "
                             f"samples={n}.")
        if n - gap - test_size * n_splits <= 0:
            raise ValueError(f"Too many splits={n_splits} for number of samples={n} with "
                             f"test_size={test_size} and gap={gap}.")
        idx = np.arange(n)
        for test_start in range(n - n_splits * test_size, n, test_size):
            train_end = test_start - gap
            if self.max_train_size and self.max_train_size < train_end:
                yield idx[train_end - self.max_train_size:train_end], \
                    idx[test_start:test_start + test_size]
            else:
                yield idx[:train_end], idx[test_start:test_start + test_size]


class LeaveOneGroupOut(BaseCrossValidator):
    def _iter_test_masks(self, X, y, groups):
        groups = _groups(groups)
        uniq = np.unique(groups)
        if len(uniq) <= 1:
            raise ValueError("The groups parameter contains fewer than 2 unique groups (%s). "
                             "LeaveOneGroupOut expects at least 2." % uniq)
        for g in uniq:
            yield groups == g

    def get_n_splits(self, X=None, y=None, groups=None):
        return len(np.unique(_groups(groups)))

    def split(self, X, y=None, groups=None):
        return super().split(X, y, groups)


class LeavePGroupsOut(BaseCrossValidator):
    def __init__(self, n_groups):
        self.n_groups = n_groups

    def _iter_test_masks(self, X, y, groups):
        groups = _groups(groups)
        uniq = np.unique(groups)
        if self.n_groups >= len(uniq):
            raise ValueError("The groups parameter contains fewer than (or equal to) n_groups "
                             "(%d) numbers of unique groups (%s). LeavePGroupsOut expects that "
                             "at least n_groups + 1 (%d) unique groups be present"
                             % (self.n_groups, uniq, self.n_groups + 1))
        for comb in itertools.combinations(range(len(uniq)), self.n_groups):
            mask = np.zeros(len(groups), dtype=bool)
            for g in uniq[np.array(comb)]:
                mask[groups == g] = True
            yield mask

    def get_n_splits(self, X=None, y=None, groups=None):
        from math import comb
        return comb(len(np.unique(_groups(groups))), self.n_groups)

    def split(self, X, y=None, groups=None):
        return super().split(X, y, groups)


class _RepeatedSplits:
    def __init__(self, cv, *, n_repeats=10, random_state=None, **cvargs):
        if not isinstance(n_repeats, numbers.Integral):
            raise ValueError("Number of repetitions must be of Integral type.")
        if n_repeats <= 0:
            raise ValueError("Number of repetitions must be greater than 0.")
        if any(k in cvargs for k in ("random_state", "shuffle")):
            raise ValueError("cvargs must not contain random_state or shuffle.")
        self.cv = cv
        self.n_repeats = n_repeats
        self.random_state = random_state
        self.cvargs = cvargs

    def split(self, X, y=None, groups=None):
        rng = check_random_state(self.random_state)
        for _ in range(self.n_repeats):
            cv = self.cv(random_state=rng, shuffle=True, **self.cvargs)
            for train, test in cv.split(X, y, groups):
                yield train, test

    def get_n_splits(self, X=None, y=None, groups=None):
        rng = check_random_state(self.random_state)
        cv = self.cv(random_state=rng, shuffle=True, **self.cvargs)
        return cv.get_n_splits(X, y, groups) * self.n_repeats

    def __repr__(self):
        return "%s(n_repeats=%d, n_splits=%d, random_state=%r)" % (
            type(self).__name__, self.n_repeats, self.cvargs.get("n_splits"), self.random_state)


class RepeatedKFold(_RepeatedSplits):
    def __init__(self, *, n_splits=5, n_repeats=10, random_state=None):
        super().__init__(KFold, n_repeats=n_repeats, random_state=random_state, n_splits=n_splits)


class RepeatedStratifiedKFold(_RepeatedSplits):
    def __init__(self, *, n_splits=5, n_repeats=10, random_state=None):
        super().__init__(StratifiedKFold, n_repeats=n_repeats, random_state=random_state,
                         n_splits=n_splits)


class GroupShuffleSplit(ShuffleSplit):
    """ShuffleSplit over unique groups (default test_size 0.2)."""

    def __init__(self, n_splits=5, *, test_size=None, train_size=None, random_state=None):
        super().__init__(n_splits=n_splits, test_size=test_size, train_size=train_size,
                         random_state=random_state)
        self._default_test_size = 0.2

    def split(self, X, y=None, groups=None):
        groups = _groups(groups)
        classes, gidx = np.unique(groups, return_inverse=True)
        for gtrain, gtest in super().split(classes):
            yield (np.flatnonzero(np.isin(gidx, gtrain)), np.flatnonzero(np.isin(gidx, gtest)))


class PredefinedSplit(BaseCrossValidator):
    def __init__(self, test_fold):
        self.test_fold = np.asarray(test_fold, dtype=int)
        self.unique_folds = np.unique(self.test_fold)
        self.unique_folds = self.unique_folds[self.unique_folds != -1]

    def split(self, X=None, y=None, groups=None):
        ind = np.arange(len(self.test_fold))
        for f in self.unique_folds:
            test = np.where(self.test_fold == f)[0]
            mask = np.ones(len(ind), dtype=bool)
            mask[test] = False
            yield ind[mask], test

    def get_n_splits(self, X=None, y=None, groups=None):
        return len(self.unique_folds)


__all__ = ["LeaveOneOut", "LeavePOut", "GroupKFold", "StratifiedGroupKFold", "TimeSeriesSplit",
           "LeaveOneGroupOut", "LeavePGroupsOut", "RepeatedKFold", "RepeatedStratifiedKFold",
           "GroupShuffleSplit", "PredefinedSplit"]
