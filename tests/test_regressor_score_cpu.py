"""``RegressorMixin.score`` and the forest OOB R^2 against scikit-learn.

The reference's ``RegressorMixin.score`` is the full ``metrics.r2_score``
(``/root/reference/sklearn/base.py:564-566``): 1-D targets are reconciled
with ``(n, 1)`` predictions and multi-output scores are uniformly averaged.
The forest OOB score is the same function on the OOB predictions
(``/root/reference/sklearn/ensemble/_forest.py:944``).  sklearn (importable
here) is the oracle, on identical predictions."""

import numpy as np
import pytest

sk_metrics = pytest.importorskip("sklearn.metrics")

from sq_learn_amd.base import RegressorMixin  # noqa: E402
from sq_learn_amd.utils.metrics import r2_score  # noqa: E402


def _data(n=120, d=6, n_out=1, seed=0):
    rng = np.random.RandomState(seed)
    X = rng.randn(n, d)
    W = rng.randn(d, n_out)
    Y = X @ W + 0.5 * rng.randn(n, n_out)
    return X, (Y[:, 0] if n_out == 1 else Y)


class _Fixed(RegressorMixin):
    def __init__(self, pred):
        self.pred = pred

    def predict(self, X):
        return self.pred


@pytest.mark.parametrize("yshape,pshape", [((-1,), (-1, 1)), ((-1, 1), (-1,)),
                                           ((-1, 1), (-1, 1)), ((-1,), (-1,))])
def test_r2_reconciles_column_vectors(yshape, pshape):
    rng = np.random.RandomState(1)
    y = rng.randn(50)
    p = y + 0.3 * rng.randn(50)
    got = _Fixed(p.reshape(pshape)).score(None, y.reshape(yshape))
    want = sk_metrics.r2_score(y, p)
    assert got == pytest.approx(want, rel=1e-12)


@pytest.mark.parametrize("mo", ["uniform_average", "raw_values", "variance_weighted"])
def test_r2_multioutput_modes(mo):
    rng = np.random.RandomState(2)
    Y = rng.randn(80, 3) * np.array([1.0, 5.0, 0.2])
    P = Y + 0.4 * rng.randn(80, 3)
    w = rng.rand(80)
    for sw in (None, w):
        got = r2_score(Y, P, sample_weight=sw, multioutput=mo)
        want = sk_metrics.r2_score(Y, P, sample_weight=sw, multioutput=mo)
        np.testing.assert_allclose(got, want, rtol=1e-12)


def test_r2_constant_target():
    y = np.ones(10)
    assert r2_score(y, y) == 1.0
    assert r2_score(y, y + 0.1) == 0.0
    with pytest.raises(ValueError):
        r2_score(np.ones(4), np.ones(5))


def test_pls_score_matches_sklearn():
    from sklearn.cross_decomposition import PLSRegression as SkPLS
    from sq_learn_amd.cross_decomposition import PLSRegression
    X, y = _data(n_out=1)
    ours = PLSRegression(2).fit(X, y)
    ref = SkPLS(2).fit(X, y)
    np.testing.assert_allclose(np.asarray(ours.predict(X)).reshape(-1),
                               np.asarray(ref.predict(X)).reshape(-1), atol=1e-8)
    assert ours.score(X, y) == pytest.approx(ref.score(X, y), rel=1e-9)


@pytest.mark.parametrize("name", ["Ridge", "LinearRegression"])
def test_multioutput_linear_score(name):
    import sklearn.linear_model as skl
    import sq_learn_amd.linear_model as ours_lm
    X, Y = _data(n_out=3, seed=3)
    ours = getattr(ours_lm, name)().fit(X, Y)
    ref = getattr(skl, name)().fit(X, Y)
    np.testing.assert_allclose(np.asarray(ours.predict(X)), ref.predict(X), atol=1e-8)
    assert ours.score(X, Y) == pytest.approx(ref.score(X, Y), rel=1e-9)
    sw = np.random.RandomState(4).rand(X.shape[0])
    assert ours.score(X, Y, sample_weight=sw) == pytest.approx(
        ref.score(X, Y, sample_weight=sw), rel=1e-9)


def test_forest_score_and_oob_semantics():
    from sq_learn_amd.ensemble import RandomForestRegressor
    X, Y = _data(n=150, n_out=2, seed=5)
    f = RandomForestRegressor(n_estimators=15, oob_score=True, random_state=0).fit(X, Y)
    # score is sklearn's r2 of this forest's own predictions
    assert f.score(X, Y) == pytest.approx(sk_metrics.r2_score(Y, f.predict(X)), rel=1e-12)
    # OOB R^2 is sklearn's r2 of the OOB predictions (uniform average over outputs)
    assert f.oob_prediction_.shape == Y.shape
    assert f.oob_score_ == pytest.approx(sk_metrics.r2_score(Y, f.oob_prediction_), rel=1e-12)
    X1, y1 = _data(n=150, n_out=1, seed=6)
    f1 = RandomForestRegressor(n_estimators=15, oob_score=True, random_state=0).fit(X1, y1)
    assert f1.oob_prediction_.shape == y1.shape
    assert f1.oob_score_ == pytest.approx(sk_metrics.r2_score(y1, f1.oob_prediction_), rel=1e-12)
