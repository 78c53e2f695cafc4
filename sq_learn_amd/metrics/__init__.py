"""Reference-layout import path (``sklearn.metrics``)."""
from ..utils.metrics import (accuracy_score, adjusted_rand_score, confusion_matrix,  # noqa: F401
                            mean_squared_error, r2_score)
from ..utils.pairwise import (euclidean_distances, linear_kernel, pairwise_distances_chunked,  # noqa: F401
                             pairwise_kernels, polynomial_kernel, rbf_kernel, sigmoid_kernel)
from ..utils.cluster_metrics import (adjusted_mutual_info_score, calinski_harabasz_score,  # noqa: F401
                                    completeness_score, contingency_matrix,
                                    davies_bouldin_score, entropy, expected_mutual_information,
                                    fowlkes_mallows_score, homogeneity_completeness_v_measure,
                                    homogeneity_score, mutual_info_score,
                                    normalized_mutual_info_score, pair_confusion_matrix,
                                    rand_score, silhouette_samples, silhouette_score,
                                    v_measure_score)
from ..utils.pairwise import (PAIRWISE_DISTANCE_FUNCTIONS, PAIRWISE_KERNEL_FUNCTIONS,  # noqa: F401
                             additive_chi2_kernel, chi2_kernel, cosine_distances,
                             cosine_similarity, haversine_distances, laplacian_kernel,
                             manhattan_distances, paired_cosine_distances, paired_distances,
                             paired_euclidean_distances, paired_manhattan_distances,
                             pairwise_distances, pairwise_distances_argmin,
                             pairwise_distances_argmin_min)
from ..utils.metrics_extra import (SCORERS, auc, average_precision_score,  # noqa: F401,E402
                                  balanced_accuracy_score, brier_score_loss, check_scoring,
                                  classification_report, cohen_kappa_score, coverage_error,
                                  dcg_score, det_curve, explained_variance_score, f1_score,
                                  fbeta_score, hamming_loss, hinge_loss, jaccard_score,
                                  label_ranking_average_precision_score, label_ranking_loss,
                                  log_loss, make_scorer, matthews_corrcoef, max_error,
                                  mean_absolute_error, mean_absolute_percentage_error,
                                  mean_gamma_deviance, mean_pinball_loss, mean_poisson_deviance,
                                  mean_squared_log_error, mean_tweedie_deviance,
                                  median_absolute_error, multilabel_confusion_matrix, ndcg_score,
                                  precision_recall_curve, precision_recall_fscore_support,
                                  precision_score, recall_score, roc_auc_score, roc_curve,
                                  top_k_accuracy_score, zero_one_loss)
from ..utils.metrics_extra import get_scorer_ext as get_scorer  # noqa: F401,E402
from ..utils.metrics_extra import mean_squared_error_ext as mean_squared_error  # noqa: F401,E402,F811
from ..utils.metrics_extra import r2_score_ext as r2_score  # noqa: F401,E402,F811
from ..models.cluster._bicluster import consensus_score  # noqa: F401,E402
from .pairwise import nan_euclidean_distances  # noqa: F401,E402
from . import cluster, pairwise  # noqa: F401,E402
from ._plot import (ConfusionMatrixDisplay, DetCurveDisplay, PrecisionRecallDisplay,  # noqa: F401,E402
                    RocCurveDisplay, plot_confusion_matrix, plot_det_curve,
                    plot_precision_recall_curve, plot_roc_curve)

from ..utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
