"""Reference-layout import path (``sklearn.decomposition``)."""
from .models.decomposition import PCA, QPCA, TruncatedSVD, qPCA  # noqa: F401
from .models.decomposition.incremental import IncrementalPCA  # noqa: F401
