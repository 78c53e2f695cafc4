"""Reference-layout import path (``sklearn.decomposition``)."""
from .models.decomposition import PCA, QPCA, TruncatedSVD, qPCA  # noqa: F401
from .models.decomposition.incremental import IncrementalPCA  # noqa: F401
from .models.decomposition._extra import (NMF, FactorAnalysis, FastICA, KernelPCA,  # noqa: F401
                                           LatentDirichletAllocation, fastica,
                                           non_negative_factorization)
from .models.decomposition._dict_learning import (DictionaryLearning,  # noqa: F401
                                                  MiniBatchDictionaryLearning,
                                                  MiniBatchSparsePCA, SparseCoder, SparsePCA,
                                                  dict_learning, dict_learning_online,
                                                  sparse_encode)

from .utils._aliases import alias_submodules  # noqa: E402
alias_submodules(__name__, "_fastica", "_truncated_svd")

from .utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
