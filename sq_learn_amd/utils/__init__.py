"""Numerical / API substrate: validation, extmath, metrics, datasets,
model selection, tracing, checkpointing."""


def _ref_internal_names():
    """Base classes / internals exposed only for reference-layout imports
    (utils._aliases.REF_NAMES): abstract in the reference, so not listed by
    all_estimators."""
    from ._aliases import REF_NAMES
    return {n for d in REF_NAMES.values() for n in d} | {"BaseRandomProjection", "BaseMixture"}


def all_estimators(type_filter=None):
    """(name, class) of every public estimator of the framework (reference
    ``utils/__init__.py:1098``: crawls the package for ``BaseEstimator``
    subclasses).  ``type_filter``: 'classifier', 'regressor', 'cluster',
    'transformer' or a list of them."""
    import importlib
    import inspect
    import pkgutil

    import sq_learn_amd
    from ..base import (BaseEstimator, ClassifierMixin, ClusterMixin, RegressorMixin,
                        TransformerMixin)

    found = {}
    for mod in pkgutil.walk_packages(sq_learn_amd.__path__, "sq_learn_amd."):
        name = mod.name
        if any(p.startswith("_") for p in name.split(".")[1:]) or ".tests" in name:
            continue
        try:
            m = importlib.import_module(name)
        except Exception:  # pragma: no cover - optional deps
            continue
        for cname, cls in inspect.getmembers(m, inspect.isclass):
            if (issubclass(cls, BaseEstimator) and cls is not BaseEstimator
                    and not cname.startswith("_") and cls.__module__.startswith("sq_learn_amd")
                    and not inspect.isabstract(cls) and cname not in _ref_internal_names()):
                found[cls] = cname
    items = sorted(((n, c) for c, n in found.items()), key=lambda t: (t[0], t[1].__module__))
    # aliases (qMeans_ = QMeans) collapse to one entry per class
    seen, out = set(), []
    for n, c in items:
        if c in seen:
            continue
        seen.add(c)
        out.append((n, c))
    if type_filter is None:
        return out
    filters = [type_filter] if isinstance(type_filter, str) else list(type_filter)
    mix = {"classifier": ClassifierMixin, "regressor": RegressorMixin,
           "cluster": ClusterMixin, "transformer": TransformerMixin}
    return [(n, c) for n, c in out if any(issubclass(c, mix[f]) for f in filters)]
from ._bunch import Bunch  # noqa: E402,F401
from ._misc import (_safe_indexing, as_float_array, assert_all_finite,  # noqa: E402,F401
                    check_symmetric, deprecated, indexable, is_scalar_nan, resample, safe_mask,
                    safe_sqr, shuffle)
from .class_weight import compute_class_weight, compute_sample_weight  # noqa: E402,F401
from .murmurhash import murmurhash3_32  # noqa: E402,F401
from .pairwise import gen_batches, gen_even_slices  # noqa: E402,F401
from .validation import (check_array, check_consistent_length, check_random_state,  # noqa: E402,F401
                         check_scalar, check_X_y, column_or_1d, check_memory,
                         check_non_negative, has_fit_parameter)

from ..exceptions import DataConversionWarning  # noqa: E402,F401
from ..parallel.tasks import parallel_backend, register_parallel_backend  # noqa: E402,F401

from ._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
