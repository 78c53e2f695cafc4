"""Splitters, parameter sampling, searches and learning curves against
scikit-learn (reference sklearn/model_selection/_split.py, _search.py,
_validation.py)."""
import warnings

import numpy as np
import pytest

pytest.importorskip("sklearn")
import sklearn.model_selection as S  # noqa: E402
from scipy.stats import randint, uniform  # noqa: E402
from sklearn.neighbors import KNeighborsClassifier as SK  # noqa: E402

import sq_learn_amd.model_selection as M  # noqa: E402
from sq_learn_amd.neighbors import KNeighborsClassifier as MK  # noqa: E402

X = np.random.RandomState(0).randn(40, 3)
y = np.arange(40) % 3
g = np.arange(40) // 3


def _same_splits(a, b):
    a, b = list(a), list(b)
    assert len(a) == len(b)
    for (tr1, te1), (tr2, te2) in zip(a, b):
        assert np.array_equal(np.sort(tr1), np.sort(tr2))
        assert np.array_equal(np.sort(te1), np.sort(te2))


@pytest.mark.parametrize("name,args,kw", [
    ("LeaveOneOut", (), {}), ("LeavePOut", (2,), {}), ("GroupKFold", (), dict(n_splits=3)),
    ("StratifiedGroupKFold", (), dict(n_splits=3)),
    ("StratifiedGroupKFold", (), dict(n_splits=3, shuffle=True, random_state=0)),
    ("TimeSeriesSplit", (), dict(n_splits=4, gap=1)), ("TimeSeriesSplit", (), dict(max_train_size=10)),
    ("LeaveOneGroupOut", (), {}), ("LeavePGroupsOut", (2,), {}),
    ("RepeatedKFold", (), dict(n_splits=3, n_repeats=2, random_state=0)),
    ("RepeatedStratifiedKFold", (), dict(n_splits=3, n_repeats=2, random_state=0)),
    ("GroupShuffleSplit", (), dict(random_state=0)), ("PredefinedSplit", (y,), {})])
def test_splitters(name, args, kw):
    _same_splits(getattr(S, name)(*args, **kw).split(X, y, g),
                 getattr(M, name)(*args, **kw).split(X, y, g))


def test_parameter_sampling_and_search():
    pd = {"a": [1, 2, 3], "b": ["x", "y"]}
    assert all(S.ParameterGrid(pd)[i] == M.ParameterGrid(pd)[i] for i in range(6))
    assert list(S.ParameterSampler(pd, 4, random_state=0)) == list(M.ParameterSampler(pd, 4, random_state=0))
    pd2 = {"a": uniform(0, 1), "b": [1, 2, 3]}
    assert list(S.ParameterSampler(pd2, 4, random_state=0)) == list(M.ParameterSampler(pd2, 4, random_state=0))
    a = S.RandomizedSearchCV(SK(), {"n_neighbors": randint(1, 20)}, n_iter=5, random_state=0, cv=3).fit(X, y)
    b = M.RandomizedSearchCV(MK(), {"n_neighbors": randint(1, 20)}, n_iter=5, random_state=0, cv=3).fit(X, y)
    assert a.best_params_ == b.best_params_
    np.testing.assert_allclose(b.cv_results_["mean_test_score"], a.cv_results_["mean_test_score"])
    assert (a.cv_results_["rank_test_score"] == b.cv_results_["rank_test_score"]).all()
    kw = dict(scoring=["accuracy", "f1_macro"], refit="accuracy", cv=3)
    a = S.GridSearchCV(SK(), {"n_neighbors": [1, 3, 5]}, **kw).fit(X, y)
    b = M.GridSearchCV(MK(), {"n_neighbors": [1, 3, 5]}, **kw).fit(X, y)
    assert not (set(a.cv_results_) - set(b.cv_results_))
    np.testing.assert_allclose(b.cv_results_["mean_test_f1_macro"], a.cv_results_["mean_test_f1_macro"])
    assert a.best_index_ == b.best_index_


def test_curves_and_halving():
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for u, v in zip(S.learning_curve(SK(), X, y, cv=3), M.learning_curve(MK(), X, y, cv=3)):
            np.testing.assert_allclose(v, u, equal_nan=True)
    for u, v in zip(S.validation_curve(SK(), X, y, param_name="n_neighbors", param_range=[1, 3, 5], cv=3),
                    M.validation_curve(MK(), X, y, param_name="n_neighbors", param_range=[1, 3, 5], cv=3)):
        np.testing.assert_allclose(v, u)
    a = S.permutation_test_score(SK(), X, y, cv=3, n_permutations=5)
    b = M.permutation_test_score(MK(), X, y, cv=3, n_permutations=5)
    assert a[0] == b[0] and np.allclose(a[1], b[1]) and a[2] == b[2]
    X2 = np.random.RandomState(0).randn(200, 3)
    y2 = (X2[:, 0] > 0).astype(int)
    h = M.HalvingGridSearchCV(MK(), {"n_neighbors": [1, 3, 5, 7, 9, 11]}, cv=3, random_state=0).fit(X2, y2)
    assert h.n_resources_ == [66, 198] and h.n_candidates_ == [6, 2]
    assert h.best_estimator_.score(X2, y2) > 0.9
