"""HIP forest inference (``csrc/forest.hip``) against the host-native
traversal: identical leaf ids and identical averaged predictions."""
import numpy as np
import pytest
import torch

from sq_learn_amd.models.ensemble import (ExtraTreesRegressor, GradientBoostingClassifier,
                                          RandomForestClassifier)
from sq_learn_amd.models.tree import DecisionTreeClassifier
from sq_learn_amd.models.tree._tree import forest_apply_device, forest_apply_host
from sq_learn_amd.utils.datasets import make_classification

pytestmark = pytest.mark.gpu


def test_forest_apply_and_predict_device(cuda):
    X, y = make_classification(3000, 12, n_informative=6, n_classes=3, random_state=0)
    rf = RandomForestClassifier(n_estimators=25, max_features="sqrt", random_state=0).fit(X, y)
    trees = [e.tree_ for e in rf.estimators_]
    Xd = torch.as_tensor(X, dtype=torch.float32, device=cuda)
    np.testing.assert_array_equal(forest_apply_device(trees, Xd), forest_apply_host(trees, X))
    np.testing.assert_allclose(rf.predict_proba(Xd), rf.predict_proba(X), rtol=0, atol=1e-12)
    np.testing.assert_array_equal(rf.predict(Xd), rf.predict(X))
    t = DecisionTreeClassifier(random_state=0).fit(X, y)
    np.testing.assert_array_equal(t.apply(Xd), t.apply(X))


def test_forest_regressor_device(cuda):
    rng = np.random.RandomState(0)
    X = rng.randn(2000, 7)
    y = X[:, 0] * 2 + np.sin(X[:, 1])
    et = ExtraTreesRegressor(n_estimators=20, random_state=0).fit(X, y)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=cuda)
    np.testing.assert_allclose(et.predict(Xd), et.predict(X), rtol=1e-12, atol=1e-12)
