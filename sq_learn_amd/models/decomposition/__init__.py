"""Matrix decomposition: qPCA (quantum-simulated PCA), PCA, TruncatedSVD."""
from .qpca import QPCA, qPCA
from .pca import PCA, TruncatedSVD
from ._base import _BasePCA

__all__ = ["QPCA", "qPCA", "PCA", "TruncatedSVD"]
from ._dict_learning import (DictionaryLearning, MiniBatchDictionaryLearning,  # noqa: E402,F401
                             MiniBatchSparsePCA, SparseCoder, SparsePCA, dict_learning,
                             dict_learning_online, sparse_encode)
