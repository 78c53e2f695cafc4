"""LS-SVM / QLSSVC (reference ``svm/_classes.py:1406-1530``, ``_qSVM.py``) and
brute-force KNN vs scikit-learn on the CPU path."""
import numpy as np
import pytest

from sq_learn_amd.models.neighbors import KNeighborsClassifier, KNeighborsRegressor, NearestNeighbors
from sq_learn_amd.models.svm import LSSVC, QLSSVC
from sq_learn_amd.utils.datasets import make_blobs, make_classification

skn = pytest.importorskip("sklearn.neighbors")


def _binary(n=200, d=5, seed=0):
    X, y = make_blobs(n_samples=n, centers=2, n_features=d, cluster_std=1.0, random_state=seed)
    return X, np.where(y == 0, -1.0, 1.0)


def _solve_lssvm(K, y, gamma_pen):
    """Dense solve of the LS-SVM KKT system [[0, 1^T], [1, K + I/C]]."""
    N = len(y)
    F = np.zeros((N + 1, N + 1))
    F[0, 1:] = 1
    F[1:, 0] = 1
    F[1:, 1:] = K + np.eye(N) / gamma_pen
    sol = np.linalg.solve(F, np.concatenate([[0.0], y]))
    return sol[0], sol[1:]


@pytest.mark.parametrize("kernel", ["linear", "rbf", "poly"])
def test_lssvc_matches_dense_kkt_solution(kernel):
    X, y = _binary()
    m = LSSVC(kernel=kernel, penalty=0.5).fit(X, y)
    K = m.get_kernel(X).cpu().numpy() if hasattr(m.get_kernel(X), "cpu") else m.get_kernel(X)
    b, a = _solve_lssvm(np.asarray(K), y, 0.5)
    np.testing.assert_allclose(m.b_, b, rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(m.alpha_, a, rtol=1e-6, atol=1e-8)
    assert m.score(X, y) > 0.95


@pytest.mark.parametrize("kernel", ["linear", "rbf"])
def test_lssvc_cg_equals_classic(kernel):
    X, y = _binary(seed=1)
    a = LSSVC(kernel=kernel, penalty=1.0, algorithm="classic").fit(X, y)
    b = LSSVC(kernel=kernel, penalty=1.0, algorithm="cg").fit(X, y)
    np.testing.assert_allclose(a.alpha_, b.alpha_, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(a.b_, b.b_, rtol=1e-5, atol=1e-7)
    np.testing.assert_array_equal(a.predict(X), b.predict(X))


def test_lssvc_sigmoid_non_spd_falls_back():
    X, y = _binary(seed=2)
    m = LSSVC(kernel="sigmoid", penalty=1.0, algorithm="cg").fit(X, y)
    assert np.all(np.isfinite(m.alpha_))


def test_qlssvc_classical_part_equals_lssvc():
    X, y = _binary(seed=3)
    q = QLSSVC(kernel="linear", penalty=0.5, random_state=0).fit(X, y)
    c = LSSVC(kernel="linear", penalty=0.5).fit(X, y)
    np.testing.assert_allclose(q.alpha_, c.alpha_, rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(q.b_, c.b_, rtol=1e-6, atol=1e-8)
    np.testing.assert_array_equal(q.classical_predict(X), c.predict(X))
    assert q.cond >= 1.0 and q.normF > 0


def test_qlssvc_noisy_predict_mostly_agrees():
    X, y = _binary(n=300, seed=4)
    q = QLSSVC(kernel="linear", penalty=0.5, absolute_error=0.01, random_state=0).fit(X, y)
    agree = np.mean(q.predict(X) == q.classical_predict(X))
    assert agree > 0.9
    assert q.get_training_complexity() > 0


def test_qlssvc_low_rank_truncation():
    X, y = _binary(seed=5)
    q = QLSSVC(kernel="rbf", penalty=1.0, low_rank=True, var=0.9, random_state=0).fit(X, y)
    s = q.singular_values_F_
    assert (s == 0).any() and (s > 0).any()


def test_qlssvc_bad_error_type():
    with pytest.raises(Exception):
        QLSSVC(error_type="nope")


@pytest.mark.parametrize("weights", ["uniform", "distance"])
def test_knn_classifier_matches_sklearn(weights):
    X, y = make_classification(n_samples=300, n_features=8, n_informative=5, n_classes=3,
                               random_state=0)
    Xq = X[:50] + 0.01
    ours = KNeighborsClassifier(n_neighbors=5, weights=weights).fit(X, y)
    ref = skn.KNeighborsClassifier(n_neighbors=5, weights=weights).fit(X, y)
    np.testing.assert_array_equal(ours.predict(Xq), ref.predict(Xq))
    np.testing.assert_allclose(ours.predict_proba(Xq), ref.predict_proba(Xq), atol=1e-12)
    d1, i1 = ours.kneighbors(Xq)
    d2, i2 = ref.kneighbors(Xq)
    np.testing.assert_allclose(d1, d2, rtol=1e-9, atol=1e-9)
    np.testing.assert_array_equal(i1, i2)


def test_knn_regressor_and_self_query():
    X, y = make_classification(n_samples=200, n_features=6, random_state=1)
    yr = X[:, 0] * 2 + 0.5
    ours = KNeighborsRegressor(n_neighbors=4).fit(X, yr)
    ref = skn.KNeighborsRegressor(n_neighbors=4).fit(X, yr)
    np.testing.assert_allclose(ours.predict(X[:30]), ref.predict(X[:30]), rtol=1e-10)
    nn = NearestNeighbors(n_neighbors=3).fit(X)
    ref_nn = skn.NearestNeighbors(n_neighbors=3).fit(X)
    d1, i1 = nn.kneighbors()
    d2, i2 = ref_nn.kneighbors()
    np.testing.assert_array_equal(i1, i2)
    np.testing.assert_allclose(d1, d2, rtol=1e-9, atol=1e-9)
