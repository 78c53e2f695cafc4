"""Trees, forests and boosting against scikit-learn
(the reference's upstream code): host-native growth must reproduce the
reference's trees - same splits, values and importances - because the
splitter streams, criteria and growth orders are the reference's."""
import warnings

import numpy as np
import pytest

sk = pytest.importorskip("sklearn")
import sklearn.ensemble as ske  # noqa: E402
import sklearn.tree as skt  # noqa: E402
from sklearn.datasets import make_classification, make_regression  # noqa: E402

from sq_learn_amd.models.ensemble import (ExtraTreesClassifier, ExtraTreesRegressor,  # noqa: E402
                                          GradientBoostingClassifier,
                                          GradientBoostingRegressor,
                                          HistGradientBoostingClassifier,
                                          HistGradientBoostingRegressor,
                                          RandomForestClassifier, RandomForestRegressor,
                                          RandomTreesEmbedding)
from sq_learn_amd.models.tree import (DecisionTreeClassifier, DecisionTreeRegressor,  # noqa: E402
                                      ExtraTreeClassifier, ExtraTreeRegressor, export_graphviz,
                                      export_text)

Xc, yc = make_classification(500, 8, n_informative=5, n_classes=3, random_state=0)
Xr, yr = make_regression(400, 6, noise=5.0, random_state=0)


def _same_tree(a, b):
    assert a.node_count == b.node_count
    np.testing.assert_array_equal(a.feature, b.feature)
    np.testing.assert_allclose(a.threshold, b.threshold)
    np.testing.assert_array_equal(a.children_left, b.children_left)
    np.testing.assert_allclose(a.impurity, b.impurity, atol=1e-12)


@pytest.mark.parametrize("criterion", ["gini", "entropy"])
@pytest.mark.parametrize("kw", [{}, {"max_depth": 4}, {"max_leaf_nodes": 12},
                                {"max_features": 3}, {"min_samples_leaf": 5,
                                                      "class_weight": "balanced"}])
def test_classifier_tree_matches_reference(criterion, kw):
    a = DecisionTreeClassifier(criterion=criterion, random_state=1, **kw).fit(Xc, yc)
    b = skt.DecisionTreeClassifier(criterion=criterion, random_state=1, **kw).fit(Xc, yc)
    _same_tree(a.tree_, b.tree_)
    np.testing.assert_allclose(a.predict_proba(Xc), b.predict_proba(Xc))
    np.testing.assert_allclose(a.feature_importances_, b.feature_importances_, atol=1e-12)
    np.testing.assert_array_equal(a.apply(Xc), b.apply(Xc))
    assert (a.decision_path(Xc) != b.decision_path(Xc)).nnz == 0


@pytest.mark.parametrize("criterion", ["squared_error", "friedman_mse", "absolute_error",
                                       "poisson"])
def test_regressor_tree_matches_reference(criterion):
    y = np.abs(yr) + 1 if criterion == "poisson" else yr
    a = DecisionTreeRegressor(criterion=criterion, random_state=0, max_leaf_nodes=10).fit(Xr, y)
    b = skt.DecisionTreeRegressor(criterion=criterion, random_state=0, max_leaf_nodes=10).fit(Xr, y)
    _same_tree(a.tree_, b.tree_)
    np.testing.assert_allclose(a.predict(Xr), b.predict(Xr), rtol=1e-10)


def test_extra_trees_and_pruning_match_reference():
    a = ExtraTreeClassifier(random_state=3, max_features=None).fit(Xc, yc)
    b = skt.ExtraTreeClassifier(random_state=3, max_features=None).fit(Xc, yc)
    _same_tree(a.tree_, b.tree_)
    a = ExtraTreeRegressor(random_state=3, max_features=None).fit(Xr, yr)
    b = skt.ExtraTreeRegressor(random_state=3, max_features=None).fit(Xr, yr)
    np.testing.assert_allclose(a.predict(Xr), b.predict(Xr))
    a = DecisionTreeClassifier(random_state=0, ccp_alpha=0.01).fit(Xc, yc)
    b = skt.DecisionTreeClassifier(random_state=0, ccp_alpha=0.01).fit(Xc, yc)
    _same_tree(a.tree_, b.tree_)
    pa = DecisionTreeClassifier(random_state=0).cost_complexity_pruning_path(Xc, yc)
    pb = skt.DecisionTreeClassifier(random_state=0).cost_complexity_pruning_path(Xc, yc)
    np.testing.assert_allclose(pa.ccp_alphas, pb.ccp_alphas)
    np.testing.assert_allclose(pa.impurities, pb.impurities)


def test_export():
    a = DecisionTreeClassifier(max_depth=2, random_state=0).fit(Xc, yc)
    b = skt.DecisionTreeClassifier(max_depth=2, random_state=0).fit(Xc, yc)
    assert export_text(a) == skt.export_text(b)
    assert export_graphviz(a).startswith("digraph Tree {")


@pytest.mark.parametrize("cls,ref,kw", [
    (RandomForestClassifier, ske.RandomForestClassifier,
     dict(n_estimators=10, random_state=1, max_samples=0.5, oob_score=True, max_depth=6,
          max_features="sqrt")),
    (RandomForestClassifier, ske.RandomForestClassifier,
     dict(n_estimators=8, random_state=2, class_weight="balanced_subsample", max_features="sqrt")),
    (ExtraTreesClassifier, ske.ExtraTreesClassifier,
     dict(n_estimators=8, random_state=2, max_features="sqrt"))])
def test_forest_classifiers_match_reference(cls, ref, kw):
    a, b = cls(**kw).fit(Xc, yc), ref(**kw).fit(Xc, yc)
    np.testing.assert_allclose(a.predict_proba(Xc), b.predict_proba(Xc))
    np.testing.assert_allclose(a.feature_importances_, b.feature_importances_, atol=1e-12)
    if kw.get("oob_score"):
        assert a.oob_score_ == pytest.approx(b.oob_score_)


def test_forest_regressors_match_reference():
    for cls, ref in [(RandomForestRegressor, ske.RandomForestRegressor),
                     (ExtraTreesRegressor, ske.ExtraTreesRegressor)]:
        kw = dict(n_estimators=10, random_state=0, max_features=1.0)
        a, b = cls(**kw).fit(Xr, yr), ref(**kw).fit(Xr, yr)
        np.testing.assert_allclose(a.predict(Xr), b.predict(Xr), rtol=1e-10)
    emb = RandomTreesEmbedding(n_estimators=5, random_state=0).fit_transform(Xr)
    assert emb.shape[0] == Xr.shape[0] and np.all(np.asarray(emb.sum(axis=1)).ravel() == 5)


def test_gradient_boosting_matches_reference():
    X2, y2 = make_classification(400, 8, n_informative=5, random_state=0)
    for kw in [dict(n_estimators=20), dict(n_estimators=15, loss="exponential")]:
        a = GradientBoostingClassifier(random_state=0, **kw).fit(X2, y2)
        b = ske.GradientBoostingClassifier(random_state=0, **kw).fit(X2, y2)
        np.testing.assert_allclose(a.predict_proba(X2), b.predict_proba(X2), atol=1e-12)
    a = GradientBoostingClassifier(n_estimators=10, random_state=0).fit(Xc, yc)
    b = ske.GradientBoostingClassifier(n_estimators=10, random_state=0).fit(Xc, yc)
    np.testing.assert_allclose(a.predict_proba(Xc), b.predict_proba(Xc), atol=1e-12)
    for loss in ["squared_error", "absolute_error", "huber", "quantile"]:
        a = GradientBoostingRegressor(loss=loss, n_estimators=15, random_state=0,
                                      subsample=0.8).fit(Xr, yr)
        b = ske.GradientBoostingRegressor(loss=loss, n_estimators=15, random_state=0,
                                          subsample=0.8).fit(Xr, yr)
        np.testing.assert_allclose(a.predict(Xr), b.predict(Xr), rtol=1e-9, atol=1e-9)
    staged = list(a.staged_predict(Xr[:5]))
    np.testing.assert_allclose(staged[-1], a.predict(Xr[:5]))


def test_hist_gradient_boosting_matches_reference():
    X, y = make_regression(2000, 8, noise=5.0, random_state=0)
    X[::9, 2] = np.nan
    for kw in [dict(max_iter=20), dict(max_iter=15, max_depth=3, l2_regularization=1.0),
               dict(max_iter=15, loss="absolute_error"),
               dict(max_iter=15, monotonic_cst=[1] + [0] * 7)]:
        a = HistGradientBoostingRegressor(random_state=0, early_stopping=False, **kw).fit(X, y)
        b = ske.HistGradientBoostingRegressor(random_state=0, early_stopping=False,
                                              **kw).fit(X, y)
        np.testing.assert_allclose(a.predict(X), b.predict(X), rtol=1e-9, atol=1e-9)
    X3, y3 = make_classification(2000, 8, n_informative=5, n_classes=3, random_state=0)
    a = HistGradientBoostingClassifier(random_state=0, max_iter=15, early_stopping=False).fit(X3, y3)
    b = ske.HistGradientBoostingClassifier(random_state=0, max_iter=15,
                                           early_stopping=False).fit(X3, y3)
    np.testing.assert_allclose(a.predict_proba(X3), b.predict_proba(X3), atol=1e-12)
    a = HistGradientBoostingClassifier(random_state=0, max_iter=200, early_stopping=True,
                                       n_iter_no_change=5).fit(X3, y3)
    b = ske.HistGradientBoostingClassifier(random_state=0, max_iter=200, early_stopping=True,
                                           n_iter_no_change=5).fit(X3, y3)
    assert a.n_iter_ == b.n_iter_
