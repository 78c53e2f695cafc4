"""Calibration, semi-supervised learning, PLS/CCA and inspection against
scikit-learn (reference sklearn/calibration.py, semi_supervised/,
cross_decomposition/_pls.py, inspection/)."""
import warnings

import numpy as np
import pytest

pytest.importorskip("sklearn")
import sklearn.calibration as SCa  # noqa: E402
import sklearn.cross_decomposition as SCD  # noqa: E402
import sklearn.inspection as SI  # noqa: E402
import sklearn.semi_supervised as SSS  # noqa: E402
from sklearn.datasets import make_classification  # noqa: E402
from sklearn.linear_model import LogisticRegression as SLR  # noqa: E402
from sklearn.naive_bayes import GaussianNB as SNB  # noqa: E402

import sq_learn_amd.calibration as MCa  # noqa: E402
import sq_learn_amd.cross_decomposition as MCD  # noqa: E402
import sq_learn_amd.inspection as MI  # noqa: E402
import sq_learn_amd.semi_supervised as MSS  # noqa: E402
from sq_learn_amd.naive_bayes import GaussianNB as MNB  # noqa: E402

X, y = make_classification(300, 6, n_informative=4, n_classes=3, random_state=0)
Xb, yb = make_classification(300, 6, random_state=1)


@pytest.fixture(autouse=True)
def _quiet():
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        yield


@pytest.mark.parametrize("method", ["sigmoid", "isotonic"])
@pytest.mark.parametrize("ensemble", [True, False])
def test_calibrated_classifier(method, ensemble):
    for XX, yy in [(X, y), (Xb, yb)]:
        a = SCa.CalibratedClassifierCV(SNB(), method=method, cv=3, ensemble=ensemble).fit(XX, yy)
        b = MCa.CalibratedClassifierCV(MNB(), method=method, cv=3, ensemble=ensemble).fit(XX, yy)
        np.testing.assert_allclose(b.predict_proba(XX), a.predict_proba(XX), atol=1e-6)


def test_calibration_curve():
    p = SNB().fit(Xb, yb).predict_proba(Xb)[:, 1]
    for st in ["uniform", "quantile"]:
        for u, v in zip(SCa.calibration_curve(yb, p, n_bins=7, strategy=st),
                        MCa.calibration_curve(yb, p, n_bins=7, strategy=st)):
            np.testing.assert_allclose(v, u)


@pytest.mark.parametrize("cls", ["LabelPropagation", "LabelSpreading"])
@pytest.mark.parametrize("kw", [dict(kernel="rbf", gamma=1), dict(kernel="knn")])
def test_label_propagation(cls, kw):
    ys = y.copy()
    ys[np.random.RandomState(0).rand(len(y)) < 0.7] = -1
    Xs = X / X.std(0) / 3
    a = getattr(SSS, cls)(**kw).fit(Xs, ys)
    b = getattr(MSS, cls)(**kw).fit(Xs, ys)
    np.testing.assert_allclose(b.label_distributions_, a.label_distributions_, atol=1e-12)
    np.testing.assert_allclose(b.predict_proba(Xs), a.predict_proba(Xs), atol=1e-12)
    assert a.n_iter_ == b.n_iter_


def test_self_training():
    ys = y.copy()
    ys[np.random.RandomState(0).rand(len(y)) < 0.7] = -1
    a = SSS.SelfTrainingClassifier(SNB()).fit(X, ys)
    b = MSS.SelfTrainingClassifier(MNB()).fit(X, ys)
    assert (a.transduction_ == b.transduction_).all() and a.n_iter_ == b.n_iter_
    assert a.termination_condition_ == b.termination_condition_


@pytest.mark.parametrize("cls", ["PLSRegression", "PLSCanonical", "CCA", "PLSSVD"])
def test_pls(cls):
    rng = np.random.RandomState(0)
    Y = np.c_[X[:, 0] + 0.1 * X[:, 1], X[:, 2] * 2, X[:, 3] - X[:, 4]] + 0.1 * rng.randn(300, 3)
    a = getattr(SCD, cls)(2).fit(X, Y)
    b = getattr(MCD, cls)(2).fit(X, Y)
    for u, v in zip(a.transform(X, Y), b.transform(X, Y)):
        np.testing.assert_allclose(v, u, atol=1e-10)
    if cls != "PLSSVD":
        np.testing.assert_allclose(b.predict(X), a.predict(X), atol=1e-10)


def test_inspection():
    m = SLR().fit(Xb, yb)
    a = SI.permutation_importance(m, Xb, yb, n_repeats=3, random_state=0)
    b = MI.permutation_importance(m, Xb, yb, n_repeats=3, random_state=0)
    np.testing.assert_allclose(b.importances, a.importances)
    a = SI.partial_dependence(m, Xb, [0, 2], kind="both", grid_resolution=10)
    b = MI.partial_dependence(m, Xb, [0, 2], kind="both", grid_resolution=10)
    np.testing.assert_allclose(b["average"], a["average"])
    np.testing.assert_allclose(b["individual"], a["individual"])
