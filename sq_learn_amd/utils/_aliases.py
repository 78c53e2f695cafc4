"""Reference-layout private module paths.

Code written against the reference sometimes imports from its private
modules (``from sklearn.ensemble._forest import ...``,
``from sklearn.utils._testing import ...``).  This package groups the same
names differently (a flat ``compose`` module, one ``_extra`` file per
family), so each such path is registered in ``sys.modules`` as an alias of
the module that actually holds the names - the module object itself, no
copies or wrappers.  Called at the end of the owning module, so an alias
exists as soon as its parent is imported, and
``import sq_learn_amd.compose._target`` resolves through ``sys.modules``
even where the parent is a plain module."""

import importlib
import sys


def alias_submodules(parent, *subs, target=None):
    """Register ``parent.<sub>`` for each sub as the module ``target``
    (default: the parent module itself) and bind it as an attribute."""
    pmod = sys.modules[parent]
    mod = pmod if target is None else importlib.import_module(target)
    for s in subs:
        sys.modules.setdefault(f"{parent}.{s}", mod)
        if not hasattr(pmod, s):
            setattr(pmod, s, mod)


# Every private module path of the reference (sklearn/<pkg>/_<mod>.py) whose
# public names this package keeps in the parent module instead; dotted
# entries register each intermediate level too.
REF_LAYOUT = {
    "sq_learn_amd.QuantumUtility": ["Utility"],
    "sq_learn_amd._loss": ["glm_distribution"],
    "sq_learn_amd.cluster": ["_affinity_propagation", "_agglomerative", "_birch", "_dbscan",
                             "_dmeans", "_feature_agglomeration", "_kmeans", "_mean_shift",
                             "_optics", "_spectral"],
    "sq_learn_amd.covariance": ["_elliptic_envelope", "_empirical_covariance", "_graph_lasso",
                                "_robust_covariance", "_shrunk_covariance"],
    "sq_learn_amd.datasets": ["_base", "_california_housing", "_covtype", "_kddcup99", "_lfw",
                              "_olivetti_faces", "_rcv1", "_samples_generator",
                              "_species_distributions", "_svmlight_format_io",
                              "_twenty_newsgroups", "_openml"],
    "sq_learn_amd.decomposition": ["_dict_learning", "_factor_analysis", "_incremental_pca",
                                   "_kernel_pca", "_lda", "_nmf", "_pca", "_qPCA", "_sparse_pca"],
    "sq_learn_amd.ensemble": ["_base", "_gb", "_gb_losses",
                              "_hist_gradient_boosting.gradient_boosting",
                              "_hist_gradient_boosting.grower", "_hist_gradient_boosting.loss",
                              "_hist_gradient_boosting.predictor", "_stacking", "_voting"],
    "sq_learn_amd.feature_selection": ["_base", "_from_model", "_mutual_info", "_rfe",
                                       "_sequential", "_univariate_selection",
                                       "_variance_threshold"],
    "sq_learn_amd.gaussian_process": ["_gpc", "_gpr"],
    "sq_learn_amd.impute": ["_base", "_iterative", "_knn"],
    "sq_learn_amd.inspection": ["_permutation_importance", "_plot.partial_dependence"],
    "sq_learn_amd.linear_model": ["_base", "_bayes", "_coordinate_descent", "_glm.glm",
                                  "_glm.link", "_huber", "_least_angle", "_logistic", "_omp",
                                  "_passive_aggressive", "_perceptron", "_ransac", "_ridge",
                                  "_sag", "_stochastic_gradient", "_theil_sen"],
    "sq_learn_amd.manifold": ["_isomap", "_locally_linear", "_mds", "_spectral_embedding",
                              "_t_sne"],
    "sq_learn_amd.metrics": ["_classification", "_plot.confusion_matrix", "_plot.det_curve",
                             "_plot.precision_recall_curve", "_plot.roc_curve", "_ranking",
                             "_regression", "_scorer", "cluster._supervised",
                             "cluster._unsupervised"],
    "sq_learn_amd.mixture": ["_base", "_bayesian_mixture", "_gaussian_mixture"],
    "sq_learn_amd.neighbors": ["_base", "_classification", "_graph", "_kde", "_nca",
                               "_nearest_centroid", "_regression", "_unsupervised"],
    "sq_learn_amd.neural_network": ["_base", "_multilayer_perceptron", "_rbm",
                                    "_stochastic_optimizers"],
    "sq_learn_amd.preprocessing": ["_discretization", "_function_transformer"],
    "sq_learn_amd.semi_supervised": ["_label_propagation"],
    "sq_learn_amd.svm": ["_base", "_bounds", "_classes", "_qSVM"],
    "sq_learn_amd.tree": ["_export", "_reingold_tilford"],
    "sq_learn_amd.utils": ["_encode", "_estimator_html_repr", "_pprint"],
}


def alias_reference_layout(parent):
    """Register the reference's private module paths under ``parent`` (see
    REF_LAYOUT) that are not real modules here, as aliases of ``parent`` -
    or of an already-registered deeper module (``metrics.cluster``)."""
    pmod = sys.modules[parent]
    for sub in REF_LAYOUT.get(parent, ()):
        parts = sub.split(".")
        cur, cur_mod = parent, pmod
        for p in parts:
            name = f"{cur}.{p}"
            m = sys.modules.get(name)
            if m is None:
                m = getattr(cur_mod, p, None)
                if not isinstance(m, type(sys)):
                    m = cur_mod
                sys.modules[name] = m
            if not hasattr(cur_mod, p):
                setattr(cur_mod, p, m)
            cur, cur_mod = name, m
    _bind_reference_names(parent)


# Names the reference defines in those private modules, resolved from where
# this package keeps them ("module:attr"), bound on the parent (which every
# alias above points to).
_R = "sq_learn_amd.utils._ref_api:"
REF_NAMES = {
    "sq_learn_amd.QuantumUtility": {"auxiliary_fun": _R + "auxiliary_fun",
                                    "vectorize_aux_fun": _R + "vectorize_aux_fun"},
    "sq_learn_amd.cluster": {
        "discretize": "sq_learn_amd.models.cluster._extra:discretize",
        "wrapper": _R + "wrapper", "labels_estimation": _R + "labels_estimation",
        "select_labels": _R + "select_labels",
        "AgglomerationTransform": "sq_learn_amd.utils._ref_classes:AgglomerationTransform"},
    "sq_learn_amd.covariance": {"c_step": _R + "c_step",
                                "select_candidates": _R + "select_candidates",
                                "alpha_max": _R + "alpha_max",
                                "graphical_lasso_path": _R + "graphical_lasso_path"},
    "sq_learn_amd.datasets": {"OpenMLError": _R + "OpenMLError", "load_data": _R + "load_data",
                              "construct_grids": _R + "construct_grids",
                              "strip_newsgroup_header": _R + "strip_newsgroup_header",
                              "strip_newsgroup_quoting": _R + "strip_newsgroup_quoting",
                              "strip_newsgroup_footer": _R + "strip_newsgroup_footer"},
    "sq_learn_amd.decomposition": {"norm": _R + "norm", "trace_dot": _R + "trace_dot"},
    "sq_learn_amd.ensemble": {
        "BaseBagging": "sq_learn_amd.models.ensemble._meta:BaseBagging",
        "BaseWeightBoosting": "sq_learn_amd.models.ensemble._meta:BaseWeightBoosting",
        "BaseForest": "sq_learn_amd.models.ensemble._forest:BaseForest",
        "ForestClassifier": "sq_learn_amd.models.ensemble._forest:ForestClassifier",
        "ForestRegressor": "sq_learn_amd.models.ensemble._forest:ForestRegressor",
        "BaseGradientBoosting": "sq_learn_amd.models.ensemble._gb:BaseGradientBoosting",
        "BaseHistGradientBoosting":
            "sq_learn_amd.models.ensemble._hist_gradient_boosting:BaseHistGradientBoosting",
        "TreePredictor": "sq_learn_amd.models.ensemble._hist_gradient_boosting:TreePredictor",
        "BaseLoss": "sq_learn_amd.models.ensemble._hist_gradient_boosting:BaseLoss"},
    "sq_learn_amd.manifold": {
        "barycenter_weights": "sq_learn_amd.models.manifold._embed:barycenter_weights",
        "barycenter_kneighbors_graph":
            "sq_learn_amd.models.manifold._embed:barycenter_kneighbors_graph",
        "null_space": "sq_learn_amd.models.manifold._embed:null_space"},
    "sq_learn_amd.tree": {"Sentinel": _R + "Sentinel"},
    "sq_learn_amd.mixture": {},
    "sq_learn_amd.svm": {"BaseLibSVM": "sq_learn_amd.models.svm._libsvm:BaseLibSVM",
                         "BaseSVC": "sq_learn_amd.models.svm._libsvm:BaseSVC"},
    "sq_learn_amd.utils": {n: _R + n for n in (
        "axis0_safe_slice", "tosequence", "indices_to_mask", "check_matplotlib_support",
        "check_pandas_support", "KeyValTuple", "KeyValTupleParam", "estimator_html_repr",
        "MissingValues")},
}
REF_NAMES["sq_learn_amd.utils"]["get_chunk_n_rows"] = "sq_learn_amd.utils.pairwise:get_chunk_n_rows"
_GB = "sq_learn_amd.models.ensemble._gb:"
_HGB = "sq_learn_amd.models.ensemble._hist_gradient_boosting:"
REF_NAMES["sq_learn_amd.ensemble"].update(
    {n: _GB + n for n in ("LossFunction", "LeastSquaresError", "LeastAbsoluteError",
                          "HuberLossFunction", "QuantileLossFunction", "BinomialDeviance",
                          "MultinomialDeviance", "ExponentialLoss")})
REF_NAMES["sq_learn_amd.ensemble"].update(
    {n: _HGB + n for n in ("LeastSquares", "LeastAbsoluteDeviation", "Poisson",
                           "BinaryCrossEntropy", "CategoricalCrossEntropy")})
_NN = "sq_learn_amd.utils._ref_nn:"
REF_NAMES["sq_learn_amd.neural_network"] = {n: _NN + n for n in (
    "inplace_identity", "inplace_logistic", "inplace_tanh", "inplace_relu", "inplace_softmax",
    "inplace_identity_derivative", "inplace_logistic_derivative", "inplace_tanh_derivative",
    "inplace_relu_derivative", "squared_loss", "log_loss", "binary_log_loss", "ACTIVATIONS",
    "DERIVATIVES", "LOSS_FUNCTIONS", "BaseOptimizer", "SGDOptimizer", "AdamOptimizer")}
REF_NAMES["sq_learn_amd.neural_network"]["BaseMultilayerPerceptron"] = \
    "sq_learn_amd.models.neural_network._mlp:BaseMultilayerPerceptron"
_LM = "sq_learn_amd.models.linear_model."
REF_NAMES["sq_learn_amd.linear_model"] = {
    "BaseLink": _NN + "BaseLink", "IdentityLink": _NN + "IdentityLink",
    "LogLink": _NN + "LogLink", "LogitLink": _NN + "LogitLink",
    "LinearModel": _LM + "_base:LinearModel",
    "LinearClassifierMixin": _LM + "_base:LinearClassifierMixin",
    "SparseCoefMixin": _LM + "_base:SparseCoefMixin",
    "BaseSGD": _LM + "_stochastic_gradient:BaseSGD",
    "BaseSGDClassifier": _LM + "_stochastic_gradient:BaseSGDClassifier",
    "BaseSGDRegressor": _LM + "_stochastic_gradient:BaseSGDRegressor",
    "get_auto_step_size": _LM + "_sag:get_auto_step_size",
    "LinearModelCV": _LM + "_coordinate_descent:_LinearModelCV",
    "sag_solver": _LM + "_sag:sag_solver"}
REF_NAMES["sq_learn_amd.gaussian_process"] = {
    "KernelOperator": "sq_learn_amd.models.gaussian_process.kernels:KernelOperator"}


def _bind_reference_names(parent):
    """Bind REF_NAMES[parent] on the parent and on every module registered
    under one of its reference paths (an alias may point at a deeper module
    the parent re-exports from)."""
    pmod = sys.modules[parent]
    targets = [pmod] + [sys.modules[f"{parent}.{s}"] for s in REF_LAYOUT.get(parent, ())
                        if f"{parent}.{s}" in sys.modules]
    for name, spec in REF_NAMES.get(parent, {}).items():
        mod, attr = spec.split(":")
        obj = getattr(importlib.import_module(mod), attr)
        for t in targets:
            if not hasattr(t, name):
                setattr(t, name, obj)
