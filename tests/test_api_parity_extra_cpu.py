"""Round-2 API parity: SGD loss objects (``_sgd_fast.pyx``), SplineTransformer
(``preprocessing/_polynomial.py:337``), the task layer with config
propagation (``utils/fixes.py:205``), fit_grid_point,
if_delegate_has_method, private module paths and the testing helpers."""
import pickle
import threading

import numpy as np
import pytest

import sq_learn_amd
from sq_learn_amd import config_context, get_config, set_config
from sq_learn_amd.linear_model import (Hinge, Huber, Log, ModifiedHuber, SGDClassifier,
                                       SquaredLoss)
from sq_learn_amd.parallel.tasks import Parallel, effective_n_jobs
from sq_learn_amd.utils.fixes import delayed


def _num_grad(loss, p, y, h=1e-6):
    return (loss.loss(p + h, y) - loss.loss(p - h, y)) / (2 * h)


@pytest.mark.parametrize("loss", [Hinge(1.0), Hinge(0.0), Log(), ModifiedHuber(), SquaredLoss(),
                                  Huber(0.5)])
def test_sgd_loss_objects(loss):
    rs = np.random.RandomState(0)
    for p, y in zip(rs.randn(50) * 3, rs.choice([-1.0, 1.0], 50)):
        # derivative consistent with the loss (away from kinks)
        if isinstance(loss, (Hinge, ModifiedHuber)) and min(abs(p * y - 1), abs(p * y + 1),
                                                            abs(p * y)) < 1e-3:
            continue
        assert loss.py_dloss(p, y) == pytest.approx(_num_grad(loss, p, y), abs=1e-4)
        assert loss.py_loss(p, y) >= 0
    assert pickle.loads(pickle.dumps(loss)) == loss
    assert Log().loss(100.0, 1.0) == pytest.approx(np.exp(-100.0))
    assert Log().loss(-100.0, 1.0) == pytest.approx(100.0)


def test_sgd_loss_function_attribute():
    X = np.random.RandomState(0).randn(60, 3)
    y = (X[:, 0] > 0).astype(int)
    clf = SGDClassifier(loss="hinge", max_iter=5, tol=None, random_state=0).fit(X, y)
    assert clf.loss_function_ == Hinge(1.0)
    clf = SGDClassifier(loss="log", max_iter=5, tol=None, random_state=0).fit(X, y)
    assert isinstance(clf.loss_function_, Log)


def test_spline_transformer_matches_sklearn():
    sk = pytest.importorskip("sklearn.preprocessing")
    from sq_learn_amd.preprocessing import SplineTransformer
    rs = np.random.RandomState(0)
    X, Xt = rs.randn(60, 2), rs.randn(50, 2) * 2
    for kw in [{}, {"degree": 1}, {"knots": "quantile", "n_knots": 4},
               {"extrapolation": "linear"}, {"extrapolation": "continue"},
               {"extrapolation": "periodic", "n_knots": 6, "degree": 2},
               {"include_bias": False}]:
        a = SplineTransformer(**kw).fit(X).transform(Xt)
        b = sk.SplineTransformer(**kw).fit(X).transform(Xt)
        np.testing.assert_allclose(a, b, atol=1e-12, err_msg=str(kw))
    # linear extrapolation of degree <= 1: per column, as a one-column fit
    a = SplineTransformer(extrapolation="linear", degree=1).fit(X).transform(Xt)
    for j in range(2):
        b = sk.SplineTransformer(extrapolation="linear", degree=1).fit(X[:, [j]]) \
            .transform(Xt[:, [j]])
        np.testing.assert_allclose(a[:, j * 5:(j + 1) * 5], b, atol=1e-12)
    with pytest.raises(ValueError):
        SplineTransformer(extrapolation="error").fit(X).transform(Xt * 10)
    st = SplineTransformer(n_knots=3, degree=2).fit(X)
    assert list(st.get_feature_names_out())[:2] == ["x0_sp_0", "x0_sp_1"]


def test_config_is_thread_local_and_propagated():
    seen = {}

    def worker():
        seen["plain"] = get_config()["working_memory"]

    with config_context(working_memory=77):
        t = threading.Thread(target=worker)
        t.start()
        t.join()
        # delayed() carries the dispatching thread's config into the worker
        out = Parallel(n_jobs=3)(delayed(lambda: get_config()["working_memory"])()
                                 for _ in range(6))
    assert seen["plain"] != 77
    assert out == [77] * 6
    assert get_config()["working_memory"] != 77


def test_parallel_order_and_errors():
    assert effective_n_jobs(None) == 1 and effective_n_jobs(2) == 2 and effective_n_jobs(-1) >= 1
    res = Parallel(n_jobs=4)(delayed(pow)(i, 2) for i in range(20))
    assert res == [i * i for i in range(20)]

    def boom(i):
        if i in (3, 5):
            raise ValueError(f"task {i}")
        return i
    with pytest.raises(ValueError, match="task 3"):
        Parallel(n_jobs=4)(delayed(boom)(i) for i in range(8))


def test_cross_validation_n_jobs_matches_sequential():
    from sq_learn_amd.linear_model import LogisticRegression
    from sq_learn_amd.model_selection import (GridSearchCV, cross_val_predict, cross_val_score,
                                              learning_curve, validation_curve)
    rs = np.random.RandomState(0)
    X = rs.randn(120, 4)
    y = (X[:, 0] + 0.3 * rs.randn(120) > 0).astype(int)
    est = LogisticRegression()
    np.testing.assert_allclose(cross_val_score(est, X, y, cv=4, n_jobs=4),
                               cross_val_score(est, X, y, cv=4))
    np.testing.assert_array_equal(cross_val_predict(est, X, y, cv=3, n_jobs=3),
                                  cross_val_predict(est, X, y, cv=3))
    g1 = GridSearchCV(est, {"C": [0.1, 1.0, 10.0]}, cv=3, n_jobs=4).fit(X, y)
    g2 = GridSearchCV(est, {"C": [0.1, 1.0, 10.0]}, cv=3).fit(X, y)
    np.testing.assert_allclose(g1.cv_results_["mean_test_score"],
                               g2.cv_results_["mean_test_score"])
    a = learning_curve(est, X, y, cv=3, n_jobs=3, train_sizes=[0.5, 1.0])
    b = learning_curve(est, X, y, cv=3, train_sizes=[0.5, 1.0])
    np.testing.assert_allclose(a[2], b[2])
    a = validation_curve(est, X, y, param_name="C", param_range=[0.1, 1.0], cv=3, n_jobs=2)
    b = validation_curve(est, X, y, param_name="C", param_range=[0.1, 1.0], cv=3)
    np.testing.assert_allclose(a[1], b[1])


def test_fit_grid_point():
    from sq_learn_amd.linear_model import LogisticRegression
    from sq_learn_amd.metrics import make_scorer, accuracy_score
    from sq_learn_amd.model_selection import fit_grid_point
    rs = np.random.RandomState(0)
    X = rs.randn(80, 3)
    y = (X[:, 0] > 0).astype(int)
    tr, te = np.arange(60), np.arange(60, 80)
    with pytest.warns(FutureWarning):
        score, params, n = fit_grid_point(X, y, LogisticRegression(), {"C": 1.0}, tr, te,
                                          make_scorer(accuracy_score), 0)
    ref = LogisticRegression(C=1.0).fit(X[tr], y[tr]).score(X[te], y[te])
    assert score == pytest.approx(ref) and params == {"C": 1.0} and n == 20


def test_if_delegate_has_method():
    from sq_learn_amd.utils.metaestimators import if_delegate_has_method

    class Inner:
        def predict(self, X):
            return "p"

    class Meta:
        def __init__(self, sub):
            self.sub = sub

        @if_delegate_has_method(delegate="sub")
        def predict(self, X):
            return self.sub.predict(X)

        @if_delegate_has_method(delegate=("sub_", "sub"))
        def transform(self, X):
            return "t"

    m = Meta(Inner())
    assert hasattr(m, "predict") and m.predict(None) == "p"
    assert not hasattr(m, "transform")


def test_private_module_paths():
    import importlib
    for path, name in [("sq_learn_amd.ensemble._forest", "RandomForestClassifier"),
                       ("sq_learn_amd.compose._column_transformer", "ColumnTransformer"),
                       ("sq_learn_amd.compose._target", "TransformedTargetRegressor"),
                       ("sq_learn_amd.model_selection._split", "GroupKFold"),
                       ("sq_learn_amd.model_selection._validation", "learning_curve"),
                       ("sq_learn_amd.preprocessing._data", "StandardScaler"),
                       ("sq_learn_amd.tree._classes", "BaseDecisionTree"),
                       ("sq_learn_amd.linear_model._glm", "GeneralizedLinearRegressor"),
                       ("sq_learn_amd.utils.deprecation", "deprecated"),
                       ("sq_learn_amd.metrics.cluster._bicluster", "consensus_score")]:
        assert hasattr(importlib.import_module(path), name), path
    from sq_learn_amd.datasets import load_sample_image
    img = load_sample_image("flower.jpg")
    assert img.shape == (427, 640, 3) and img.dtype == np.uint8


def test_testing_helpers():
    import warnings
    from sq_learn_amd.utils import _testing as T
    T.assert_array_equal([1, 2], [1, 2])
    T.assert_warns(UserWarning, warnings.warn, "x")
    T.assert_raise_message(ValueError, "bad", lambda: (_ for _ in ()).throw(ValueError("bad x")))

    @T.ignore_warnings
    def noisy():
        warnings.warn("y")
        return 3
    assert noisy() == 3
    with T.raises(ValueError, match="oops"):
        raise ValueError("oops here")
    with T.raises(KeyError, may_pass=True):
        pass
    clf = T.MinimalClassifier().fit([[0], [1], [1]], [0, 1, 1])
    assert (clf.predict([[5]]) == 1).all()
    with T.TempMemmap(np.arange(5.0)) as d:
        assert d[3] == 3.0
