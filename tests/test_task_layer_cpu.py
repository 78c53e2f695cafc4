"""Task fan-out of the meta-estimators over the task layer
(parallel/tasks.py; reference joblib ``Parallel(n_jobs)`` at
``multiclass.py:281,641``, ``ensemble/_bagging.py:382``,
``multioutput.py:186``, ``ensemble/_voting.py:74``): fits with n_jobs > 1
run on worker threads and give the n_jobs = 1 result; parallel_backend /
register_parallel_backend select the executor (reference
``utils/__init__.py:49-53``)."""
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from sq_learn_amd.utils import parallel_backend, register_parallel_backend, DataConversionWarning
from sq_learn_amd.parallel.tasks import Parallel, effective_n_jobs
from sq_learn_amd.utils.fixes import delayed


def _data(n=120, d=5, k=3, seed=0):
    rs = np.random.RandomState(seed)
    X = rs.randn(n, d)
    y = (X[:, 0] * 2 + X[:, 1] > 0).astype(int) + (X[:, 2] > 0.5).astype(int)
    return X, y[:n] % k


class _Spy:
    names = set()


def _record(est_cls):
    orig = est_cls.fit

    def fit(self, *a, **kw):
        _Spy.names.add(threading.current_thread().name)
        return orig(self, *a, **kw)
    return orig, fit


@pytest.mark.parametrize("kind", ["ovr", "ovo", "occ", "bagging", "multioutput", "voting",
                                  "stacking"])
def test_meta_estimators_fan_out_and_match_sequential(kind, monkeypatch):
    from sq_learn_amd.models.linear_model import LogisticRegression, Ridge
    from sq_learn_amd import multiclass, multioutput
    from sq_learn_amd.models.ensemble import _meta
    X, y = _data()
    Y = np.c_[X[:, 0] + X[:, 1], X[:, 2] - X[:, 3]]
    orig, fit = _record(LogisticRegression)
    monkeypatch.setattr(LogisticRegression, "fit", fit)
    orig_r, fit_r = _record(Ridge)
    monkeypatch.setattr(Ridge, "fit", fit_r)

    def make(nj):
        if kind == "ovr":
            return multiclass.OneVsRestClassifier(LogisticRegression(), n_jobs=nj), (X, y)
        if kind == "ovo":
            return multiclass.OneVsOneClassifier(LogisticRegression(), n_jobs=nj), (X, y)
        if kind == "occ":
            return multiclass.OutputCodeClassifier(LogisticRegression(), random_state=0,
                                                   n_jobs=nj), (X, y)
        if kind == "bagging":
            return _meta.BaggingClassifier(LogisticRegression(), n_estimators=6, random_state=0,
                                           n_jobs=nj), (X, y)
        if kind == "multioutput":
            return multioutput.MultiOutputRegressor(Ridge(), n_jobs=nj), (X, Y)
        if kind == "voting":
            return _meta.VotingClassifier([("a", LogisticRegression()),
                                           ("b", LogisticRegression(C=0.1))], n_jobs=nj), (X, y)
        return _meta.StackingClassifier([("a", LogisticRegression()),
                                         ("b", LogisticRegression(C=0.1))], cv=3,
                                        n_jobs=nj), (X, y)

    _Spy.names.clear()
    e1, (Xa, ya) = make(1)
    p1 = e1.fit(Xa, ya).predict(Xa)
    assert _Spy.names == {"MainThread"}
    _Spy.names.clear()
    e2, _ = make(3)
    p2 = e2.fit(Xa, ya).predict(Xa)
    assert any(n.startswith("sq-task") for n in _Spy.names), _Spy.names
    np.testing.assert_array_equal(p1, p2)


def test_parallel_backend_context_and_registry():
    assert effective_n_jobs(None) == 1
    with parallel_backend("threading", n_jobs=3):
        assert effective_n_jobs(None) == 3
        names = Parallel()(delayed(lambda i: threading.current_thread().name)(i)
                           for i in range(6))
        assert all(n.startswith("sq-task") for n in names)
        with parallel_backend("sequential"):
            assert Parallel(n_jobs=4)(delayed(lambda: threading.current_thread().name)()
                                      for _ in range(2)) == ["MainThread"] * 2
    register_parallel_backend("custom_pool",
                              lambda n: ThreadPoolExecutor(n, thread_name_prefix="custom"))
    with parallel_backend("custom_pool", n_jobs=2):
        got = Parallel()(delayed(lambda i: (i, threading.current_thread().name))(i)
                         for i in range(4))
    assert [g[0] for g in got] == [0, 1, 2, 3]
    assert all(g[1].startswith("custom") for g in got)
    with pytest.raises(ValueError):
        with parallel_backend("no_such_backend"):
            pass
    assert issubclass(DataConversionWarning, UserWarning)


def test_forest_per_tree_builds_fan_out_identically():
    """Bootstrap + min_weight_fraction_leaf gives every tree its own leaf
    weight floor: one native build per tree over the task layer
    (reference ``ensemble/_forest.py:396``); n_jobs must not change a tree."""
    import numpy as np
    from sq_learn_amd.models.ensemble._forest import RandomForestClassifier
    X = np.random.RandomState(0).randn(400, 6)
    y = (X[:, 0] + X[:, 1] > 0).astype(int)
    kw = dict(n_estimators=6, min_weight_fraction_leaf=0.05, random_state=0)
    a = RandomForestClassifier(n_jobs=1, **kw).fit(X, y)
    b = RandomForestClassifier(n_jobs=3, **kw).fit(X, y)
    np.testing.assert_array_equal(a.predict_proba(X), b.predict_proba(X))
    assert [e.tree_.node_count for e in a.estimators_] == [e.tree_.node_count for e in b.estimators_]


def test_nested_parallel_inherits_backend_and_registered_backend_pins():
    """A Parallel inside a worker task sees the caller's parallel_backend
    (the context stack travels with the task), and registered executors run
    tasks through the same per-task wrapper as the threading backend."""
    seen = []

    def inner(i):
        seen.append(effective_n_jobs(None))
        return i

    def outer(i):
        return sum(Parallel(n_jobs=None)(delayed(inner)(j) for j in range(2)))

    with parallel_backend("threading", n_jobs=3):
        out = Parallel(n_jobs=2)(delayed(outer)(i) for i in range(4))
    assert out == [1, 1, 1, 1]
    assert seen and all(v == 3 for v in seen)

    calls = []

    class Exec(ThreadPoolExecutor):
        def submit(self, fn, *a, **kw):
            calls.append(getattr(fn, "__name__", ""))
            return super().submit(fn, *a, **kw)

    register_parallel_backend("pinned_exec", lambda n: Exec(max_workers=n))
    with parallel_backend("pinned_exec", n_jobs=2):
        r = Parallel(n_jobs=2)(delayed(lambda v: v * 2)(i) for i in range(3))
    assert r == [0, 2, 4]
    assert calls and all(c == "_run" for c in calls)
