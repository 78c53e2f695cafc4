"""Reference-layout import path (``sklearn.metrics``)."""
from .utils.metrics import (accuracy_score, adjusted_rand_score, confusion_matrix,  # noqa: F401
                            mean_squared_error, r2_score)
from .utils.pairwise import (euclidean_distances, linear_kernel, pairwise_distances_chunked,  # noqa: F401
                             pairwise_kernels, polynomial_kernel, rbf_kernel, sigmoid_kernel)
