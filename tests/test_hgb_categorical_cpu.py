"""Native categorical splits of histogram gradient boosting (reference
``ensemble/_hist_gradient_boosting/splitting.pyx``
``_find_best_bin_to_split_category``, ``_predictor.pyx`` bitsets)."""
import warnings

import numpy as np
import pytest

from sq_learn_amd.ensemble import HistGradientBoostingClassifier as QC
from sq_learn_amd.ensemble import HistGradientBoostingRegressor as QR

SE = pytest.importorskip("sklearn.ensemble")


@pytest.fixture(scope="module")
def data():
    rng = np.random.RandomState(0)
    n = 1500
    Xc = rng.randint(0, 12, size=(n, 2)).astype(float)
    Xn = rng.randn(n, 3)
    eff = rng.randn(12)
    y = eff[Xc[:, 0].astype(int)] + 0.5 * eff[::-1][Xc[:, 1].astype(int)] + Xn[:, 0]
    y += 0.1 * rng.randn(n)
    Xm = np.c_[Xc, Xn]
    Xm[rng.rand(n) < 0.1, 0] = np.nan
    return np.c_[Xc, Xn], Xm, y


@pytest.mark.parametrize("missing", [False, True])
@pytest.mark.parametrize("cf", [[0, 1], [True, False, False, False, False]])
def test_regressor_categorical_parity(data, missing, cf):
    X, Xm, y = data
    X = Xm if missing else X
    kw = dict(categorical_features=cf, max_iter=25, random_state=0, early_stopping=False)
    a = SE.HistGradientBoostingRegressor(**kw).fit(X, y)
    b = QR(**kw).fit(X, y)
    Xt = X.copy()
    Xt[:5, 0] = 13          # unknown category follows the missing direction
    np.testing.assert_allclose(a.predict(Xt), b.predict(Xt), atol=1e-10)


def test_classifier_categorical_parity(data):
    _, Xm, y = data
    yc = (y > 0).astype(int) + (y > 1)
    kw = dict(categorical_features=[0, 1], max_iter=15, random_state=0, early_stopping=False)
    a = SE.HistGradientBoostingClassifier(**kw).fit(Xm, yc)
    b = QC(**kw).fit(Xm, yc)
    np.testing.assert_allclose(a.predict_proba(Xm), b.predict_proba(Xm), atol=1e-10)
    kw = dict(categorical_features=[0], max_iter=15, random_state=0)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a = SE.HistGradientBoostingClassifier(**kw).fit(Xm, yc > 0)
    b = QC(**kw).fit(Xm, yc > 0)
    assert a.n_iter_ == b.n_iter_
    np.testing.assert_allclose(a.predict_proba(Xm), b.predict_proba(Xm), atol=1e-10)


def test_categorical_validation(data):
    X, _, y = data
    with pytest.raises(ValueError):
        QR(categorical_features=[7]).fit(X, y)
    with pytest.raises(ValueError):
        QR(categorical_features=[True, False]).fit(X, y)
    with pytest.raises(ValueError):
        QR(categorical_features=["a"]).fit(X, y)
    with pytest.raises(ValueError):
        QR(categorical_features=[2], max_bins=10).fit(X * 100, y)
    with pytest.raises(ValueError):
        QR(categorical_features=[0], monotonic_cst=[1, 0, 0, 0, 0]).fit(X, y)
