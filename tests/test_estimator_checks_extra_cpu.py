"""The reference's individual public estimator checks
(utils/estimator_checks.py) on representative estimators."""
import numpy as np
import pytest

from sq_learn_amd.utils import estimator_checks as EC
from sq_learn_amd.linear_model import LogisticRegression, Ridge
from sq_learn_amd.cluster import KMeans
from sq_learn_amd.decomposition import PCA
from sq_learn_amd.preprocessing import StandardScaler
from sq_learn_amd.ensemble import IsolationForest

ESTS = [LogisticRegression(max_iter=500), Ridge(), KMeans(n_clusters=3, n_init=2, random_state=0),
        PCA(n_components=2), StandardScaler(), IsolationForest(random_state=0)]
CHECKS = ["check_estimators_fit_returns_self", "check_supervised_y_no_nan",
          "check_supervised_y_2d", "check_estimator_sparse_data", "check_sample_weights_list",
          "check_sample_weights_shape", "check_sample_weights_invariance",
          "check_complex_data", "check_dict_unchanged", "check_fit2d_predict1d",
          "check_methods_subset_invariance", "check_methods_sample_order_invariance",
          "check_fit2d_1sample", "check_fit2d_1feature", "check_fit1d",
          "check_transformers_unfitted", "check_pipeline_consistency",
          "check_fit_score_takes_y", "check_clusterer_compute_labels_predict",
          "check_classifiers_one_label", "check_outliers_train", "check_classifiers_classes",
          "check_regressors_int", "check_estimators_overwrite_params",
          "check_estimators_data_not_an_array", "check_classifiers_regression_target",
          "check_decision_proba_consistency", "check_requires_y_none",
          "check_n_features_in_after_fitting", "check_class_weight_classifiers"]


@pytest.mark.parametrize("check", CHECKS)
@pytest.mark.parametrize("est", ESTS, ids=lambda e: type(e).__name__)
def test_individual_checks(check, est):
    getattr(EC, check)(type(est).__name__, est)


def test_class_weight_balanced_linear():
    EC.check_class_weight_balanced_linear_classifier("LogisticRegression", LogisticRegression)


def test_outlier_corruption_helper():
    EC.check_outlier_corruption(3, 3, np.arange(10.0))
    with pytest.raises(AssertionError):
        EC.check_outlier_corruption(2, 5, np.arange(10.0))
