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
from .utils.pairwise import (PAIRWISE_DISTANCE_FUNCTIONS, PAIRWISE_KERNEL_FUNCTIONS,  # noqa: F401
                             additive_chi2_kernel, chi2_kernel, cosine_distances,
                             cosine_similarity, haversine_distances, laplacian_kernel,
                             manhattan_distances, paired_cosine_distances, paired_distances,
                             paired_euclidean_distances, paired_manhattan_distances,
                             pairwise_distances, pairwise_distances_argmin,
                             pairwise_distances_argmin_min)
