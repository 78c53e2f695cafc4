"""Matrix decomposition: qPCA (quantum-simulated PCA), PCA, TruncatedSVD."""
from .qpca import QPCA, qPCA
from .pca import PCA, TruncatedSVD
from ._base import _BasePCA

__all__ = ["QPCA", "qPCA", "PCA", "TruncatedSVD"]
