"""The public estimator-conformance checks (``sq_learn_amd.utils.estimator_checks``,
reference ``utils/estimator_checks.py:431/486``) over every estimator of the
framework, and ``parametrize_with_checks`` on the fork's estimators."""
import warnings

import pytest

from sq_learn_amd.utils import all_estimators
from sq_learn_amd.utils.estimator_checks import check_estimator, parametrize_with_checks
from sq_learn_amd.models.cluster import QMeans, KMeans
from sq_learn_amd.models.decomposition import QPCA
from sq_learn_amd.models.svm import LSSVC, QLSSVC

from test_api_cpu import _instance


@parametrize_with_checks([QMeans(n_clusters=3, n_init=1, random_state=0, device="cpu"),
                          QMeans(n_clusters=3, n_init=1, delta=0.5, intermediate_error=True,
                                 true_distance_estimate=False, random_state=0, device="cpu"),
                          KMeans(n_clusters=3, n_init=1, random_state=0, device="cpu"),
                          QPCA(n_components=2, device="cpu"), LSSVC(), QLSSVC()])
def test_fork_estimators(estimator, check):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        check(estimator)


@pytest.mark.parametrize("name,cls", all_estimators(), ids=[n for n, _ in all_estimators()])
def test_check_estimator_all(name, cls):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        check_estimator(_instance(cls))


def test_check_estimator_rejects_classes_and_reports():
    from sq_learn_amd.models.linear_model import Ridge
    with pytest.raises(TypeError):
        check_estimator(Ridge)
    assert len(list(check_estimator(Ridge(), generate_only=True))) > 10

    class Bad(Ridge):
        def __init__(self, alpha=1.0):
            self.alpha = alpha
            self.extra = 3       # violates the constructor contract
    with pytest.raises(AssertionError):
        check_estimator(Bad())
