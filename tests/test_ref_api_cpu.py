"""Reference private module paths and the smaller public helpers kept for
API parity (utils/_aliases.py REF_LAYOUT / REF_NAMES, utils/_ref_api.py,
utils/_ref_nn.py, _loss/glm_distribution.py).  Behaviour checked against the
installed scikit-learn where it still has the helper, else against closed
forms."""

import importlib

import numpy as np
import pytest


@pytest.mark.parametrize("path,name", [
    ("sq_learn_amd.linear_model._ridge", "Ridge"),
    ("sq_learn_amd.linear_model._glm.link", "LogLink"),
    ("sq_learn_amd.cluster._dmeans", "qMeans_"),
    ("sq_learn_amd.cluster._dmeans", "labels_estimation"),
    ("sq_learn_amd.decomposition._qPCA", "qPCA"),
    ("sq_learn_amd.svm._qSVM", "QLSSVC"),
    ("sq_learn_amd.metrics._plot.roc_curve", "RocCurveDisplay"),
    ("sq_learn_amd.metrics.cluster._unsupervised", "silhouette_score"),
    ("sq_learn_amd.metrics.cluster._unsupervised", "check_number_of_labels"),
    ("sq_learn_amd.ensemble._hist_gradient_boosting.loss", "LeastSquares"),
    ("sq_learn_amd.ensemble._forest", "ForestClassifier"),
    ("sq_learn_amd.neural_network._stochastic_optimizers", "AdamOptimizer"),
    ("sq_learn_amd.covariance._graph_lasso", "graphical_lasso_path"),
    ("sq_learn_amd.datasets._samples_generator", "make_blobs"),
    ("sq_learn_amd._loss.glm_distribution", "TweedieDistribution"),
    ("sq_learn_amd.QuantumUtility.Utility", "vectorize_aux_fun"),
    ("sq_learn_amd.gaussian_process.kernels", "KernelOperator"),
])
def test_reference_private_paths(path, name):
    mod = importlib.import_module(path)
    assert hasattr(mod, name), (path, name)


def test_extmath_helpers():
    from sq_learn_amd.utils import extmath as E
    from scipy.special import softmax as sp_softmax
    rs = np.random.RandomState(0)
    X = rs.randn(6, 4)
    np.testing.assert_allclose(E.softmax(X), sp_softmax(X, axis=1))
    np.testing.assert_allclose(E.log_logistic(X), -np.log1p(np.exp(-X)))
    assert E.density(np.array([[0, 1], [2, 0]])) == 0.5
    c = E.cartesian(([1, 2], [3, 4, 5]))
    assert c.shape == (6, 2) and c[0].tolist() == [1, 3] and c[-1].tolist() == [2, 5]
    mode, score = E.weighted_mode(np.array([4, 1, 4, 2, 4, 2]), np.array([1, 1, 1, 1, 1, 1]))
    assert mode[0] == 4 and score[0] == 3
    mode, score = E.weighted_mode(np.array([4, 1, 4, 2, 4, 2]), np.array([1, 3, 0.5, 1.5, 1, 2]))
    assert mode[0] == 2 and score[0] == 3.5
    assert E.make_nonnegative(np.array([-2.0, 1.0])).min() == 0


def test_utils_helpers():
    from sq_learn_amd import utils as U
    assert U.indices_to_mask([0, 2], 4).tolist() == [True, False, True, False]
    assert U.axis0_safe_slice(np.ones((3, 2)), np.zeros(3, bool), 0).shape == (0, 2)
    assert U.tosequence((1, 2)) == (1, 2)
    assert U.get_chunk_n_rows(8, working_memory=1) >= 1


def test_pairwise_checks():
    from sq_learn_amd.metrics import pairwise as P
    X, Y = P.check_pairwise_arrays(np.ones((3, 2), np.float32), np.ones((4, 2), np.float32))
    assert X.dtype == np.float32 and Y.shape == (4, 2)
    X, Y = P.check_pairwise_arrays(np.ones((3, 2), np.float32), np.ones((4, 2)))
    assert X.dtype == np.float64
    with pytest.raises(ValueError):
        P.check_pairwise_arrays(np.ones((3, 2)), np.ones((3, 3)))
    with pytest.raises(ValueError):
        P.check_paired_arrays(np.ones((3, 2)), np.ones((4, 2)))
    assert "euclidean" in P.distance_metrics() and "rbf" in P.kernel_metrics()


def test_tweedie_deviance_matches_sklearn():
    from sklearn.metrics import mean_tweedie_deviance
    from sq_learn_amd._loss.glm_distribution import TweedieDistribution
    rs = np.random.RandomState(1)
    y = rs.gamma(2.0, size=50)
    mu = rs.gamma(2.0, size=50)
    for p in (0, 1, 1.5, 2, 3):
        d = TweedieDistribution(power=p)
        np.testing.assert_allclose(d.deviance(y, mu) / len(y),
                                   mean_tweedie_deviance(y, mu, power=p), rtol=1e-10)
    with pytest.raises(ValueError):
        TweedieDistribution(power=0.5)
    # derivative by finite differences
    d = TweedieDistribution(power=1.5)
    h = 1e-6
    fd = (d.unit_deviance(y, mu + h) - d.unit_deviance(y, mu - h)) / (2 * h)
    np.testing.assert_allclose(d.unit_deviance_derivative(y, mu), fd, rtol=1e-5)


def test_glm_regressor_accepts_distribution_object():
    from sq_learn_amd.linear_model import GeneralizedLinearRegressor
    from sq_learn_amd._loss.glm_distribution import PoissonDistribution
    rs = np.random.RandomState(0)
    X = rs.randn(80, 3)
    y = rs.poisson(np.exp(X @ [0.3, -0.2, 0.1]))
    a = GeneralizedLinearRegressor(family=PoissonDistribution(), link="log").fit(X, y)
    b = GeneralizedLinearRegressor(family="poisson", link="log").fit(X, y)
    np.testing.assert_allclose(a.coef_, b.coef_)


def test_covariance_helpers():
    from sq_learn_amd.covariance import alpha_max, graphical_lasso_path, select_candidates
    rs = np.random.RandomState(0)
    X = rs.randn(60, 4)
    C = np.cov(X.T, bias=True)
    off = np.abs(C - np.diag(np.diag(C))).max()
    assert alpha_max(C) == off
    covs, precs = graphical_lasso_path(X, [0.5 * off, 0.1 * off])
    assert len(covs) == 2 and covs[0].shape == (4, 4)
    locs, covs2, sup, dist = select_candidates(X, 40, 5, select=2, random_state=0)
    assert locs.shape == (2, 4) and sup.shape == (2, 60) and sup[0].sum() == 40


def test_nn_optimizers_and_activations():
    from sq_learn_amd.neural_network import AdamOptimizer, SGDOptimizer, inplace_relu
    Z = np.array([[-1.0, 2.0]])
    inplace_relu(Z)
    assert Z.tolist() == [[0.0, 2.0]]
    p = [np.zeros(3)]
    SGDOptimizer(p, learning_rate_init=0.1, momentum=0.0, nesterov=False).update_params(
        p, [np.ones(3)])
    np.testing.assert_allclose(p[0], -0.1)
    p = [np.zeros(2)]
    AdamOptimizer(p, learning_rate_init=0.01).update_params(p, [np.array([1.0, -1.0])])
    np.testing.assert_allclose(p[0], [-0.01, 0.01], rtol=1e-6)


def test_dmeans_labels_estimation_band():
    from sq_learn_amd.cluster import labels_estimation
    rs = np.random.RandomState(0)
    X = rs.randn(30, 3)
    C = X[:4]
    lab, D, inertia = labels_estimation(X, C, 0.5, None, False)
    mins = D.min(1)
    assert all(D[i, l] <= mins[i] + 0.5 for i, l in enumerate(lab))
    assert np.isclose(inertia, mins.sum())


def test_mocking_doubles():
    from sq_learn_amd.utils._mocking import (CheckingClassifier, MockDataFrame,
                                             NoSampleWeightWrapper)
    from sq_learn_amd.model_selection import cross_val_score
    from sq_learn_amd.linear_model import LogisticRegression
    X = np.arange(40.0).reshape(20, 2)
    y = np.arange(20) % 2
    df = MockDataFrame(X)
    assert len(df) == 20 and isinstance(df.iloc[:5], MockDataFrame)
    assert np.asarray(df.iloc[:5]).shape == (5, 2)
    clf = CheckingClassifier(check_X=lambda A: A.shape[1] == 2, foo_param=2).fit(X, y)
    assert (clf.predict(X) == 0).all() and clf.score() == 1.0
    with pytest.raises(AssertionError):
        CheckingClassifier(check_X=lambda A: False).fit(X, y)
    with pytest.raises(AssertionError):
        CheckingClassifier(expected_fit_params=["spam"]).fit(X, y)
    s = cross_val_score(CheckingClassifier(foo_param=2), X, y, cv=2)
    assert np.all(s == 1.0)
    w = NoSampleWeightWrapper(LogisticRegression()).fit(X, y)
    assert w.predict(X).shape == (20,)
