"""Bagging, IsolationForest, AdaBoost, Voting and Stacking against
scikit-learn (reference sklearn/ensemble/_bagging.py, _iforest.py,
_weight_boosting.py, _voting.py, _stacking.py).  Members are the
framework's native CART trees, so whole ensembles match bit for bit.
AdaBoost SAMME.R was removed in sklearn 1.6 and SAMME's predict_proba
scaling changed in 1.4: those compare fitted weights and predictions."""
import warnings

import numpy as np
import pytest

pytest.importorskip("sklearn")
import sklearn.ensemble as S  # noqa: E402
from sklearn.datasets import make_classification, make_regression  # noqa: E402
from sklearn.linear_model import Ridge as SR  # noqa: E402
from sklearn.naive_bayes import GaussianNB as SNB  # noqa: E402
from sklearn.tree import DecisionTreeClassifier as SDT  # noqa: E402

import sq_learn_amd.ensemble as M  # noqa: E402
from sq_learn_amd.linear_model import Ridge as MR  # noqa: E402
from sq_learn_amd.naive_bayes import GaussianNB as MNB  # noqa: E402
from sq_learn_amd.tree import DecisionTreeClassifier as MDT  # noqa: E402

X, y = make_classification(300, 8, n_informative=5, n_classes=3, random_state=0)
Xr, yr = make_regression(300, 8, noise=5, random_state=0)


@pytest.fixture(autouse=True)
def _quiet():
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        yield


@pytest.mark.parametrize("kw", [{}, dict(max_samples=0.5, max_features=0.7),
                                dict(bootstrap=False, max_samples=0.6),
                                dict(bootstrap_features=True, oob_score=True)])
def test_bagging(kw):
    a = S.BaggingClassifier(random_state=0, **kw).fit(X, y)
    b = M.BaggingClassifier(random_state=0, **kw).fit(X, y)
    np.testing.assert_array_equal(b.predict_proba(X), a.predict_proba(X))
    a = S.BaggingRegressor(random_state=0, **kw).fit(Xr, yr)
    b = M.BaggingRegressor(random_state=0, **kw).fit(Xr, yr)
    np.testing.assert_allclose(b.predict(Xr), a.predict(Xr), atol=1e-12)
    if kw.get("oob_score"):
        assert a.oob_score_ == pytest.approx(b.oob_score_)


@pytest.mark.parametrize("kw", [{}, dict(contamination=0.1), dict(max_features=0.5),
                                dict(max_samples=100, bootstrap=True)])
def test_isolation_forest(kw):
    a = S.IsolationForest(random_state=0, **kw).fit(Xr)
    b = M.IsolationForest(random_state=0, **kw).fit(Xr)
    np.testing.assert_allclose(b.score_samples(Xr), a.score_samples(Xr), atol=1e-12)
    assert (a.predict(Xr) == b.predict(Xr)).all()


def test_adaboost():
    a = S.AdaBoostClassifier(algorithm="SAMME", random_state=0).fit(X, y)
    b = M.AdaBoostClassifier(algorithm="SAMME", random_state=0).fit(X, y)
    np.testing.assert_allclose(b.estimator_weights_, a.estimator_weights_)
    assert (a.predict(X) == b.predict(X)).all()
    r = M.AdaBoostClassifier(random_state=0).fit(X, y)
    assert r.score(X, y) > 0.6 and np.allclose(r.predict_proba(X).sum(1), 1)
    for loss in ["linear", "square", "exponential"]:
        a = S.AdaBoostRegressor(loss=loss, random_state=0).fit(Xr, yr)
        b = M.AdaBoostRegressor(loss=loss, random_state=0).fit(Xr, yr)
        np.testing.assert_allclose(b.predict(Xr), a.predict(Xr), atol=1e-12)


def test_voting_stacking():
    for v in ["hard", "soft"]:
        a = S.VotingClassifier([("nb", SNB()), ("dt", SDT(random_state=0))], voting=v,
                               weights=[1, 2]).fit(X, y)
        b = M.VotingClassifier([("nb", MNB()), ("dt", MDT(random_state=0))], voting=v,
                               weights=[1, 2]).fit(X, y)
        assert (a.predict(X) == b.predict(X)).all()
        np.testing.assert_allclose(b.transform(X), a.transform(X), atol=1e-12)
    a = S.VotingRegressor([("r", SR()), ("r2", SR(alpha=10))]).fit(Xr, yr)
    b = M.VotingRegressor([("r", MR()), ("r2", MR(alpha=10))]).fit(Xr, yr)
    np.testing.assert_allclose(b.predict(Xr), a.predict(Xr), atol=1e-9)
    a = S.StackingClassifier([("nb", SNB()), ("dt", SDT(random_state=0))],
                             final_estimator=SNB()).fit(X, y)
    b = M.StackingClassifier([("nb", MNB()), ("dt", MDT(random_state=0))],
                             final_estimator=MNB()).fit(X, y)
    np.testing.assert_allclose(b.predict_proba(X), a.predict_proba(X), atol=1e-10)
    a = S.StackingRegressor([("r", SR()), ("rf", S.RandomForestRegressor(n_estimators=5, random_state=0))],
                            final_estimator=SR()).fit(Xr, yr)
    b = M.StackingRegressor([("r", MR()), ("rf", M.RandomForestRegressor(n_estimators=5, random_state=0))],
                            final_estimator=MR()).fit(Xr, yr)
    np.testing.assert_allclose(b.predict(Xr), a.predict(Xr), atol=1e-8)
