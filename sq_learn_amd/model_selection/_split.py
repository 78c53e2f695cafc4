"""Cross-validation splitters (reference ``sklearn/model_selection/_split.py``:
``KFold`` :348, ``StratifiedKFold`` :553, ``ShuffleSplit`` :1418,
``StratifiedShuffleSplit`` :1708, ``train_test_split`` :2090).

Index bookkeeping is host-side numpy (splits are tiny next to the fits they
drive); the same seeds give the same folds as the reference, so a pipeline
evaluated by the reference's ``cross_validate`` (``MnistTrial.py``) sees the
same train/test partitions here.
"""

import numbers

import numpy as np

from ..runtime.device import to_numpy
from ..utils.validation import _num_samples, check_random_state


def _indexable_len(X):
    return _num_samples(X)


class BaseCrossValidator:
    def split(self, X, y=None, groups=None):
        n = _indexable_len(X)
        idx = np.arange(n)
        for test in self._iter_test_masks(X, y, groups):
            yield idx[~test], idx[test]

    def _iter_test_masks(self, X, y=None, groups=None):
        n = _indexable_len(X)
        for test_index in self._iter_test_indices(X, y, groups):
            mask = np.zeros(n, dtype=bool)
            mask[test_index] = True
            yield mask

    def _iter_test_indices(self, X, y=None, groups=None):  # pragma: no cover
        raise NotImplementedError

    def __repr__(self):
        keys = sorted(k for k in self.__dict__ if not k.startswith("_"))
        return f"{type(self).__name__}(" + ", ".join(f"{k}={getattr(self, k)!r}" for k in keys) + ")"


class _BaseKFold(BaseCrossValidator):
    def __init__(self, n_splits, *, shuffle, random_state):
        if not isinstance(n_splits, numbers.Integral):
            raise ValueError(f"The number of folds must be of Integral type. {n_splits!r} given.")
        n_splits = int(n_splits)
        if n_splits <= 1:
            raise ValueError("k-fold cross-validation requires at least one train/test split "
                             f"by setting n_splits=2 or more, got n_splits={n_splits}.")
        if not isinstance(shuffle, bool):
            raise TypeError(f"shuffle must be True or False; got {shuffle}")
        if not shuffle and random_state is not None:
            raise ValueError("Setting a random_state has no effect since shuffle is False. "
                             "You should leave random_state to its default (None), or set "
                             "shuffle=True.")
        self.n_splits = n_splits
        self.shuffle = shuffle
        self.random_state = random_state

    def split(self, X, y=None, groups=None):
        n = _indexable_len(X)
        if self.n_splits > n:
            raise ValueError(f"Cannot have number of splits n_splits={self.n_splits} greater "
                             f"than the number of samples: n_samples={n}.")
        return super().split(X, y, groups)

    def get_n_splits(self, X=None, y=None, groups=None):
        return self.n_splits


class KFold(_BaseKFold):
    def __init__(self, n_splits=5, *, shuffle=False, random_state=None):
        super().__init__(n_splits, shuffle=shuffle, random_state=random_state)

    def _iter_test_indices(self, X, y=None, groups=None):
        n = _indexable_len(X)
        indices = np.arange(n)
        if self.shuffle:
            check_random_state(self.random_state).shuffle(indices)
        sizes = np.full(self.n_splits, n // self.n_splits, dtype=int)
        sizes[: n % self.n_splits] += 1
        cur = 0
        for s in sizes:
            yield indices[cur:cur + s]
            cur += s


class StratifiedKFold(_BaseKFold):
    """Folds preserving class proportions (reference ``_split.py:553-716``)."""

    def __init__(self, n_splits=5, *, shuffle=False, random_state=None):
        super().__init__(n_splits, shuffle=shuffle, random_state=random_state)

    def _make_test_folds(self, X, y):
        rng = check_random_state(self.random_state)
        y = np.asarray(to_numpy(y))
        if y.ndim != 1:
            y = y.reshape(-1)
        _, y_idx, y_inv = np.unique(y, return_index=True, return_inverse=True)
        # classes numbered in order of first appearance
        _, class_perm = np.unique(y_idx, return_inverse=True)
        y_enc = class_perm[y_inv]
        n_classes = len(y_idx)
        y_counts = np.bincount(y_enc)
        if np.all(self.n_splits > y_counts):
            raise ValueError(f"n_splits={self.n_splits} cannot be greater than the number of "
                             "members in each class.")
        # deterministic, balanced allocation of each class to the folds
        y_order = np.sort(y_enc)
        allocation = np.asarray([np.bincount(y_order[i::self.n_splits], minlength=n_classes)
                                 for i in range(self.n_splits)])
        test_folds = np.empty(len(y), dtype=int)
        for k in range(n_classes):
            folds_for_class = np.arange(self.n_splits).repeat(allocation[:, k])
            if self.shuffle:
                rng.shuffle(folds_for_class)
            test_folds[y_enc == k] = folds_for_class
        return test_folds

    def _iter_test_masks(self, X, y=None, groups=None):
        test_folds = self._make_test_folds(X, y)
        for i in range(self.n_splits):
            yield test_folds == i

    def split(self, X, y, groups=None):
        return super().split(X, y, groups)


class BaseShuffleSplit(BaseCrossValidator):
    """Base of the random-permutation splitters (reference
    ``model_selection/_split.py`` BaseShuffleSplit): ``n_splits`` independent
    train / test draws."""

    def get_n_splits(self, X=None, y=None, groups=None):
        return self.n_splits


class ShuffleSplit(BaseShuffleSplit):
    def __init__(self, n_splits=10, *, test_size=None, train_size=None, random_state=None):
        self.n_splits = n_splits
        self.test_size = test_size
        self.train_size = train_size
        self.random_state = random_state
        self._default_test_size = 0.1

    def split(self, X, y=None, groups=None):
        n = _indexable_len(X)
        n_train, n_test = _validate_shuffle_split(n, self.test_size, self.train_size,
                                                  self._default_test_size)
        rng = check_random_state(self.random_state)
        for _ in range(self.n_splits):
            perm = rng.permutation(n)
            yield perm[n_test:n_test + n_train], perm[:n_test]

    def get_n_splits(self, X=None, y=None, groups=None):
        return self.n_splits


class StratifiedShuffleSplit(ShuffleSplit):
    """Random stratified splits (reference ``_split.py:1708``): per class, the
    test/train counts follow the class proportions (largest remainders)."""

    def split(self, X, y, groups=None):
        n = _indexable_len(X)
        y = np.asarray(to_numpy(y)).reshape(-1)
        n_train, n_test = _validate_shuffle_split(n, self.test_size, self.train_size,
                                                  self._default_test_size)
        classes, y_ind = np.unique(y, return_inverse=True)
        class_counts = np.bincount(y_ind)
        if np.min(class_counts) < 2:
            raise ValueError("The least populated class in y has only 1 member, which is too "
                             "few. The minimum number of groups for any class cannot be less "
                             "than 2.")
        class_indices = np.split(np.argsort(y_ind, kind="mergesort"), np.cumsum(class_counts)[:-1])
        rng = check_random_state(self.random_state)
        for _ in range(self.n_splits):
            n_i = _approximate_mode(class_counts, n_train, rng)
            t_i = _approximate_mode(class_counts - n_i, n_test, rng)
            train, test = [], []
            for i in range(len(classes)):
                perm = rng.permutation(class_counts[i])
                sel = class_indices[i][perm]
                train.extend(sel[:n_i[i]])
                test.extend(sel[n_i[i]:n_i[i] + t_i[i]])
            yield rng.permutation(np.asarray(train, dtype=int)), rng.permutation(np.asarray(test, dtype=int))


def _approximate_mode(class_counts, n_draws, rng):
    """Per-class draw counts summing to n_draws, proportional to class_counts
    (floor, then remainders assigned largest-first with random tie-break)."""
    continuous = class_counts / class_counts.sum() * n_draws
    floored = np.floor(continuous).astype(int)
    need = int(n_draws - floored.sum())
    if need > 0:
        rem = continuous - floored
        values = np.sort(np.unique(rem))[::-1]
        for v in values:
            (inds,) = np.where(rem == v)
            take = min(len(inds), need)
            inds = rng.choice(inds, size=take, replace=False)
            floored[inds] += 1
            need -= take
            if need == 0:
                break
    return floored


def _validate_shuffle_split(n, test_size, train_size, default_test_size=None):
    if test_size is None and train_size is None:
        test_size = default_test_size
    if test_size is not None and np.asarray(test_size).dtype.kind == "f":
        if not 0 < test_size < 1:
            raise ValueError(f"test_size={test_size} should be in (0, 1)")
        n_test = int(np.ceil(test_size * n))
    elif test_size is not None:
        n_test = int(test_size)
    else:
        n_test = None
    if train_size is not None and np.asarray(train_size).dtype.kind == "f":
        if not 0 < train_size < 1:
            raise ValueError(f"train_size={train_size} should be in (0, 1)")
        n_train = int(np.floor(train_size * n))
    elif train_size is not None:
        n_train = int(train_size)
    else:
        n_train = None
    if n_train is None:
        n_train = n - n_test
    if n_test is None:
        n_test = n - n_train
    if n_train + n_test > n:
        raise ValueError(f"The sum of train_size and test_size = {n_train + n_test}, should be "
                         f"smaller than the number of samples {n}.")
    if n_train <= 0 or n_test <= 0:
        raise ValueError("With n_samples={}, test_size={} and train_size={}, the resulting "
                         "train set will be empty.".format(n, test_size, train_size))
    return n_train, n_test


def _safe_index(a, idx):
    if a is None:
        return None
    if hasattr(a, "index_select"):   # torch tensor (possibly on device)
        import torch
        return a.index_select(0, torch.as_tensor(idx, device=a.device))
    if hasattr(a, "iloc"):
        return a.iloc[idx]
    if isinstance(a, list):
        return [a[i] for i in idx]
    return np.asarray(a)[idx]


def train_test_split(*arrays, test_size=None, train_size=None, random_state=None, shuffle=True,
                     stratify=None):
    """Split arrays into random train and test subsets (reference ``:2090``)."""
    if not arrays:
        raise ValueError("At least one array required as input")
    n = _indexable_len(arrays[0])
    for a in arrays[1:]:
        if _indexable_len(a) != n:
            raise ValueError("Found input variables with inconsistent numbers of samples")
    n_train, n_test = _validate_shuffle_split(n, test_size, train_size, default_test_size=0.25)
    if not shuffle:
        if stratify is not None:
            raise ValueError("Stratified train/test split is not implemented for shuffle=False")
        train, test = np.arange(n_train), np.arange(n_train, n_train + n_test)
    else:
        cls = StratifiedShuffleSplit if stratify is not None else ShuffleSplit
        cv = cls(test_size=n_test, train_size=n_train, random_state=random_state)
        train, test = next(cv.split(X=arrays[0], y=stratify))
    out = []
    for a in arrays:
        out += [_safe_index(a, train), _safe_index(a, test)]
    return out


def check_cv(cv=5, y=None, *, classifier=False):
    """int / None / splitter / iterable -> splitter (reference ``:2013``)."""
    cv = 5 if cv is None else cv
    if isinstance(cv, numbers.Integral):
        if classifier and y is not None:
            yy = np.asarray(to_numpy(y))
            if yy.ndim == 1 and (yy.dtype.kind in "iub" or yy.dtype.kind == "O"
                                 or len(np.unique(yy)) <= max(2, len(yy) // 2)):
                return StratifiedKFold(cv)
        return KFold(cv)
    if hasattr(cv, "split"):
        return cv
    return _CVIterableWrapper(cv)


class _CVIterableWrapper(BaseCrossValidator):
    def __init__(self, cv):
        self.cv = list(cv)

    def get_n_splits(self, X=None, y=None, groups=None):
        return len(self.cv)

    def split(self, X=None, y=None, groups=None):
        for train, test in self.cv:
            yield train, test


# The group / leave-out / repeated / predefined splitters live in
# _split_extra.py (which imports this module); the reference exposes them
# from model_selection/_split.py, so they resolve here lazily (PEP 562).
_EXTRA_SPLITTERS = ("GroupKFold", "LeaveOneGroupOut", "LeaveOneOut", "LeavePGroupsOut",
                    "LeavePOut", "RepeatedStratifiedKFold", "RepeatedKFold", "GroupShuffleSplit",
                    "StratifiedGroupKFold", "PredefinedSplit", "TimeSeriesSplit")


def __getattr__(name):
    if name in _EXTRA_SPLITTERS:
        from . import _split_extra
        return getattr(_split_extra, name)
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
