"""utils.multiclass (reference utils/multiclass.py) against the installed
scikit-learn's, plus the experimental import switches."""
import importlib
import warnings

import numpy as np
import pytest
import scipy.sparse as sp

from sq_learn_amd.utils import multiclass as M

skm = pytest.importorskip("sklearn.utils.multiclass")

CASES = [
    [0, 1, 1, 0], [1, 2, 3], ["a", "b", "a"], [0.5, 1.5], [1.0, 2.0, 3.0],
    np.array([[0, 1], [1, 0]]), np.array([[1, 2], [3, 1]]), np.array([[0.5, 1.0], [1.5, 2]]),
    np.array([[1], [0]]), np.array([[]]).reshape(1, 0), sp.csr_matrix(np.array([[0, 1], [1, 1]])),
    np.array([0, 0, 0]), np.array([[0, 1, 2]]),
]


@pytest.mark.parametrize("y", CASES, ids=range(len(CASES)))
def test_type_of_target_matches(y):
    assert M.type_of_target(y) == skm.type_of_target(y)
    assert M.is_multilabel(y) == skm.is_multilabel(y)


def test_unique_labels_and_errors():
    np.testing.assert_array_equal(M.unique_labels([3, 5, 5], [1, 3]), [1, 3, 5])
    np.testing.assert_array_equal(M.unique_labels(np.eye(3, dtype=int)), [0, 1, 2])
    with pytest.raises(ValueError, match="Mix type"):
        M.unique_labels([1, 2], np.eye(2, dtype=int))
    with pytest.raises(ValueError, match="string and number"):
        M.unique_labels(["a", "b"], [1, 2])
    with pytest.raises(ValueError, match="different numbers"):
        M.unique_labels(np.eye(2, dtype=int), np.eye(3, dtype=int))
    M.check_classification_targets([0, 1, 2])
    with pytest.raises(ValueError, match="Unknown label type"):
        M.check_classification_targets([0.5, 1.5])


@pytest.mark.parametrize("sparse", [False, True])
def test_class_distribution_matches(sparse):
    y = np.array([[1, 0, 0, 1], [2, 2, 0, 1], [1, 3, 0, 1], [4, 2, 0, 1], [2, 0, 0, 1],
                  [1, 3, 0, 1]])
    sw = np.array([1, 2, 1, 1, 3, 1.0])
    yy = sp.csc_matrix(y) if sparse else y
    for w in (None, sw):
        a = M.class_distribution(yy, w)
        b = skm.class_distribution(yy, w)
        for u, v in zip(a, b):
            for p, q in zip(u, v):
                np.testing.assert_allclose(p, q)


def test_ovr_decision_function_matches():
    rs = np.random.RandomState(0)
    pred = rs.randint(0, 2, (20, 6))
    conf = rs.randn(20, 6)
    np.testing.assert_allclose(M._ovr_decision_function(pred, conf, 4),
                               skm._ovr_decision_function(pred, conf, 4))


def test_experimental_switches():
    with warnings.catch_warnings(record=True):
        warnings.simplefilter("always")
        importlib.import_module("sq_learn_amd.experimental.enable_hist_gradient_boosting")
    importlib.import_module("sq_learn_amd.experimental.enable_iterative_imputer")
    importlib.import_module("sq_learn_amd.experimental.enable_halving_search_cv")
    from sq_learn_amd.impute import IterativeImputer  # noqa: F401
    from sq_learn_amd.model_selection import HalvingGridSearchCV, HalvingRandomSearchCV  # noqa
