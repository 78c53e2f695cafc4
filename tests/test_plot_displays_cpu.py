"""Visualisation API: metrics displays (reference ``metrics/_plot``) and
partial dependence plots (``inspection/_plot/partial_dependence.py``) drawn
with the Agg backend; the plotted data is checked against scikit-learn's own
curve functions and the artists / labels against the reference behaviour."""
import matplotlib

matplotlib.use("Agg")

import matplotlib.pyplot as plt  # noqa: E402
import numpy as np  # noqa: E402
import pytest  # noqa: E402
from scipy.stats import norm  # noqa: E402

from sq_learn_amd.inspection import PartialDependenceDisplay, plot_partial_dependence  # noqa: E402
from sq_learn_amd.linear_model import LinearRegression, LogisticRegression  # noqa: E402
from sq_learn_amd.metrics import (ConfusionMatrixDisplay, DetCurveDisplay,  # noqa: E402
                                  PrecisionRecallDisplay, RocCurveDisplay, confusion_matrix,
                                  precision_recall_curve,
                                  plot_confusion_matrix, plot_roc_curve)

skm = pytest.importorskip("sklearn.metrics")


@pytest.fixture(autouse=True)
def _close():
    yield
    plt.close("all")


def _binary():
    rs = np.random.RandomState(0)
    X = rs.randn(300, 4)
    y = (X[:, 0] + 0.5 * X[:, 1] + 0.3 * rs.randn(300) > 0).astype(int)
    return X, y, LogisticRegression().fit(X, y)


def test_roc_display_from_estimator():
    X, y, clf = _binary()
    disp = RocCurveDisplay.from_estimator(clf, X, y)
    p = clf.predict_proba(X)[:, 1]
    fpr, tpr, _ = skm.roc_curve(y, p)
    np.testing.assert_allclose(disp.fpr, fpr)
    np.testing.assert_allclose(disp.tpr, tpr)
    assert disp.roc_auc == pytest.approx(skm.roc_auc_score(y, p))
    assert disp.line_.get_label() == f"LogisticRegression (AUC = {disp.roc_auc:0.2f})"
    assert disp.ax_.get_xlabel() == "False Positive Rate (Positive label: 1)"
    assert disp.figure_ is disp.ax_.figure
    with pytest.warns(FutureWarning):
        d2 = plot_roc_curve(clf, X, y, name="m")
    assert d2.line_.get_label().startswith("m (AUC")


def test_roc_display_decision_function_pos_label():
    X, y, clf = _binary()
    d = RocCurveDisplay.from_estimator(clf, X, y, response_method="decision_function",
                                       pos_label=0)
    fpr, tpr, _ = skm.roc_curve(y, -clf.decision_function(X), pos_label=0)
    np.testing.assert_allclose(d.fpr, fpr)
    np.testing.assert_allclose(d.tpr, tpr)


def test_pr_and_det_displays():
    X, y, clf = _binary()
    p = clf.predict_proba(X)[:, 1]
    pr = PrecisionRecallDisplay.from_predictions(y, p, name="clf")
    # (the reference's curve stops at full recall, ``_ranking.py:830``;
    # newer scikit-learn keeps the tail: compare with this package's curve)
    prec, rec, _ = precision_recall_curve(y, p)
    k = len(rec)
    sp, sr, _ = skm.precision_recall_curve(y, p)
    np.testing.assert_allclose(prec[1:], sp[-k + 1:])
    np.testing.assert_allclose(pr.precision, prec)
    np.testing.assert_allclose(pr.recall, rec)
    assert pr.average_precision == pytest.approx(skm.average_precision_score(y, p))
    assert pr.line_.get_drawstyle() == "steps-post"
    assert pr.line_.get_label().startswith("clf (AP = ")
    det = DetCurveDisplay.from_estimator(clf, X, y)
    fpr, fnr, _ = skm.det_curve(y, p)
    np.testing.assert_allclose(det.fpr, fpr)
    np.testing.assert_allclose(det.fnr, fnr)
    np.testing.assert_allclose(det.line_.get_xdata(), norm.ppf(fpr))
    assert det.ax_.get_xlim() == (-3, 3)


def test_confusion_matrix_display():
    rs = np.random.RandomState(1)
    y = rs.randint(0, 3, 200)
    yp = np.where(rs.rand(200) < 0.7, y, rs.randint(0, 3, 200))
    d = ConfusionMatrixDisplay.from_predictions(y, yp, display_labels=["a", "b", "c"])
    cm = skm.confusion_matrix(y, yp)
    np.testing.assert_array_equal(d.confusion_matrix, cm)
    assert d.text_.shape == (3, 3)
    assert d.text_[0, 0].get_text() == str(cm[0, 0])
    assert [t.get_text() for t in d.ax_.get_xticklabels()] == ["a", "b", "c"]
    assert d.ax_.get_ylabel() == "True label" and d.ax_.get_xlabel() == "Predicted label"
    # text colour flips at the colour-map midpoint
    lo, hi = d.im_.cmap(0), d.im_.cmap(1.0)
    thresh = (cm.max() + cm.min()) / 2.0
    for i in range(3):
        for j in range(3):
            assert d.text_[i, j].get_color() == (hi if cm[i, j] < thresh else lo)
    dn = ConfusionMatrixDisplay.from_predictions(y, yp, normalize="true", values_format=".3f",
                                                 include_values=True, colorbar=False)
    np.testing.assert_allclose(dn.confusion_matrix, skm.confusion_matrix(y, yp, normalize="true"))
    assert dn.text_[1, 1].get_text() == format(dn.confusion_matrix[1, 1], ".3f")
    X, yb, clf = _binary()
    with pytest.warns(FutureWarning):
        dd = plot_confusion_matrix(clf, X, yb, include_values=False)
    assert dd.text_ is None


def test_confusion_matrix_weights_and_normalize():
    rs = np.random.RandomState(0)
    a, b, w = rs.randint(0, 4, 300), rs.randint(0, 4, 300), rs.rand(300)
    for kw in [{}, {"labels": [3, 1, 0]}, {"sample_weight": w}, {"normalize": "pred"},
               {"normalize": "all", "sample_weight": w}]:
        ours, ref = confusion_matrix(a, b, **kw), skm.confusion_matrix(a, b, **kw)
        np.testing.assert_allclose(ours, ref)
        assert ours.dtype.kind == ref.dtype.kind
    with pytest.raises(ValueError):
        confusion_matrix(a, b, normalize="rows")
    with pytest.raises(ValueError):
        confusion_matrix(a, b, labels=[])


def test_partial_dependence_display_one_and_two_way():
    rs = np.random.RandomState(0)
    X = rs.randn(200, 3)
    y = 2 * X[:, 0] - X[:, 1] + 0.1 * rs.randn(200)
    reg = LinearRegression().fit(X, y)
    disp = plot_partial_dependence(reg, X, [0, 1, (0, 1)], grid_resolution=20,
                                   feature_names=["a", "b", "c"])
    assert disp.axes_.shape == (1, 3)
    line = disp.lines_[0, 0]
    # linear model: the PD of feature 0 is a line of slope 2
    xs, ys = line.get_xdata(), line.get_ydata()
    np.testing.assert_allclose(np.diff(ys) / np.diff(xs), reg.coef_[0], rtol=1e-6)
    assert disp.axes_[0, 0].get_xlabel() == "a"
    assert disp.axes_[0, 0].get_ylabel() == "Partial dependence"
    assert disp.contours_[0, 2] is not None
    assert disp.deciles_vlines_[0, 0] is not None and disp.deciles_hlines_[0, 2] is not None
    assert len(disp.deciles[0]) == 9


def test_partial_dependence_display_ice():
    rs = np.random.RandomState(0)
    X = rs.randn(150, 2)
    y = X[:, 0] ** 2 + X[:, 1]
    reg = LinearRegression().fit(X, y)
    disp = PartialDependenceDisplay.from_estimator(reg, X, [0], kind="both", subsample=20,
                                                   random_state=0, grid_resolution=10)
    lines = disp.lines_[0, 0]
    assert len(lines) == 21            # 20 ICE curves + the average
    assert lines[-1].get_label() == "average"
    with pytest.raises(ValueError):
        PartialDependenceDisplay.from_estimator(reg, X, [(0, 1)], kind="individual")
    fig, axs = plt.subplots(1, 2)
    d2 = PartialDependenceDisplay.from_estimator(reg, X, [0, 1], ax=axs)
    assert d2.bounding_ax_ is None and d2.axes_.shape == (2,)
