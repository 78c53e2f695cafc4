"""liblinear's trust-region Newton primal solver (csrc/host/tron.cpp,
reference ``svm/src/liblinear/tron.cpp`` + ``linear.cpp`` types 0 / 2 / 11)
against scikit-learn's bundled liblinear: coefficients to rounding and the
same iteration counts."""
import warnings

import numpy as np
import pytest

skl = pytest.importorskip("sklearn.linear_model")
sks = pytest.importorskip("sklearn.svm")

import sq_learn_amd.linear_model as L  # noqa: E402
import sq_learn_amd.svm as S  # noqa: E402

rs = np.random.RandomState(0)
X = rs.randn(400, 7)
y2 = (X[:, 0] + 0.5 * X[:, 1] + 0.5 * rs.randn(400) > 0).astype(int)
y3 = np.digitize(X[:, 0] + 0.3 * rs.randn(400), [-0.5, 0.5])
yr = X @ rs.randn(7) + 0.1 * rs.randn(400)


@pytest.fixture(autouse=True)
def _quiet():
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        yield


@pytest.mark.parametrize("y", [y2, y3])
@pytest.mark.parametrize("C,scaling,cw", [(0.1, 1.0, None), (10.0, 3.0, "balanced")])
def test_logistic_liblinear_l2(y, C, scaling, cw):
    kw = dict(solver="liblinear", C=C, intercept_scaling=scaling, class_weight=cw)
    a, b = L.LogisticRegression(**kw).fit(X, y), skl.LogisticRegression(**kw).fit(X, y)
    np.testing.assert_allclose(a.coef_, b.coef_, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(a.intercept_, b.intercept_, rtol=1e-10, atol=1e-12)
    np.testing.assert_array_equal(a.n_iter_, b.n_iter_)


def test_linear_svc_and_svr_primal():
    a = S.LinearSVC(dual=False, C=0.5).fit(X, y3)
    b = sks.LinearSVC(dual=False, C=0.5).fit(X, y3)
    np.testing.assert_allclose(a.coef_, b.coef_, rtol=1e-10, atol=1e-12)
    assert a.n_iter_ == b.n_iter_
    kw = dict(dual=False, loss="squared_epsilon_insensitive", epsilon=0.1, C=2.0)
    a, b = S.LinearSVR(**kw).fit(X, yr), sks.LinearSVR(**kw).fit(X, yr)
    np.testing.assert_allclose(a.coef_, b.coef_, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(a.intercept_, b.intercept_, rtol=1e-10, atol=1e-12)
    assert a.n_iter_ == b.n_iter_
