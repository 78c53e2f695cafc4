"""Reference-layout import path (``sklearn.metrics``)."""
from .utils.metrics import (accuracy_score, adjusted_rand_score, confusion_matrix,  # noqa: F401
                            mean_squared_error, r2_score)
from .utils.pairwise import (euclidean_distances, linear_kernel, pairwise_distances_chunked,  # noqa: F401
                             pairwise_kernels, polynomial_kernel, rbf_kernel, sigmoid_kernel)
from .utils.cluster_metrics import (adjusted_mutual_info_score, calinski_harabasz_score,  # noqa: F401
                                    completeness_score, contingency_matrix,
                                    davies_bouldin_score, entropy, expected_mutual_information,
                                    fowlkes_mallows_score, homogeneity_completeness_v_measure,
                                    homogeneity_score, mutual_info_score,
                                    normalized_mutual_info_score, pair_confusion_matrix,
                                    rand_score, silhouette_samples, silhouette_score,
                                    v_measure_score)
