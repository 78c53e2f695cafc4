"""Reference-layout import path ``sklearn.metrics.cluster``."""
from ..models.cluster._bicluster import consensus_score  # noqa: F401
from ..utils.cluster_metrics import *  # noqa: F401,F403
from ..utils.metrics import adjusted_rand_score  # noqa: F401,E402

from ..utils._aliases import alias_submodules  # noqa: E402
alias_submodules(__name__, "_bicluster")
from ..utils._ref_api import check_number_of_labels  # noqa: E402,F401
