"""sq_learn_amd - an MI355X-native (gfx950) quantum-simulated machine learning
framework with the capabilities of federicomegler/sq-learn.

Top level as in the reference (``sklearn/__init__.py:80-99``): the config
functions, ``clone`` and ``show_versions``; the estimator sub-packages are
imported on first attribute access (``sq_learn_amd.cluster`` etc.)."""
import importlib

__version__ = "0.1.0"

from ._config import config_context, get_config, set_config  # noqa: E402
from .base import clone  # noqa: E402
from .utils._show_versions import show_versions  # noqa: E402

_SUBMODULES = ("calibration", "cluster", "covariance", "cross_decomposition", "datasets",
               "decomposition", "dummy", "ensemble", "exceptions", "experimental",
               "feature_extraction", "feature_selection", "gaussian_process", "inspection",
               "isotonic", "kernel_approximation", "kernel_ridge", "linear_model", "manifold",
               "metrics", "mixture", "model_selection", "multiclass", "multioutput",
               "naive_bayes", "neighbors", "neural_network", "pipeline", "preprocessing",
               "random_projection", "semi_supervised", "svm", "tree", "discriminant_analysis",
               "impute", "compose", "QuantumUtility", "utils", "parallel", "quantum")

__all__ = list(_SUBMODULES[:-3]) + ["clone", "get_config", "set_config", "config_context",
                                    "show_versions"]


def __getattr__(name):
    if name in _SUBMODULES:
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
