"""Reference-layout import path (``sklearn.cluster``): q-means and k-means."""
from .models.cluster import KMeans, LloydEngine, QMeans, k_means, kmeans_plusplus, qMeans_  # noqa: F401
from .models.cluster.minibatch import MiniBatchKMeans  # noqa: F401
from .models.cluster.dbscan import DBSCAN, dbscan  # noqa: F401
from .models.cluster.hierarchical import (AgglomerativeClustering, FeatureAgglomeration,  # noqa: F401
                                          linkage_tree, ward_tree)
from .models.cluster._extra import (OPTICS, AffinityPropagation, Birch, MeanShift,  # noqa: F401
                                     SpectralClustering, affinity_propagation,
                                     cluster_optics_dbscan, cluster_optics_xi,
                                     compute_optics_graph, estimate_bandwidth, get_bin_seeds,
                                     mean_shift, spectral_clustering)
from .models.cluster._bicluster import SpectralBiclustering, SpectralCoclustering  # noqa: F401,E402

from .utils._aliases import alias_submodules  # noqa: E402
alias_submodules(__name__, "_bicluster", target="sq_learn_amd.models.cluster._bicluster")

from .utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
