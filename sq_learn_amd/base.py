"""Estimator protocol: ``BaseEstimator``, mixins and ``clone``.

Behavioural parity with the reference's ``sklearn/base.py``:

* ``get_params`` / ``set_params`` introspect ``__init__`` and support nested
  ``a__b`` keys (``base.py:142-255``);
* ``__repr__`` prints changed parameters only (``print_changed_only``);
* pickling adds a version tag and warns on mismatch (``base.py:296-320``).
  Unlike the reference, fitted torch tensors (possibly on a GPU) are moved to
  host numpy in ``__getstate__``, so a model fitted on MI355X can be loaded
  on a machine without a GPU;
* ``_validate_data`` / ``n_features_in_`` checking (``base.py:381-451``);
* mixins: ``ClassifierMixin.score`` (accuracy), ``RegressorMixin.score``
  (R^2), ``ClusterMixin.fit_predict``, ``TransformerMixin.fit_transform``
  (``base.py:482-780``).
"""

import copy
import functools
import inspect
import warnings
from collections import defaultdict

import numpy as np
import torch

from .exceptions import InconsistentVersionWarning


def _framework_version():
    from . import __version__
    return __version__


def clone(estimator, *, safe=True):
    """Deep copy of an estimator's *parameters* (unfitted), reference ``base.py:30``."""
    if isinstance(estimator, (list, tuple, set, frozenset)):
        return type(estimator)([clone(e, safe=safe) for e in estimator])
    if not hasattr(estimator, "get_params") or isinstance(estimator, type):
        if not safe:
            return copy.deepcopy(estimator)
        raise TypeError(f"Cannot clone object '{estimator!r}' (type {type(estimator)}): "
                        "it does not implement get_params.")
    klass = estimator.__class__
    params = estimator.get_params(deep=False)
    new_params = {k: clone(v, safe=False) for k, v in params.items()}
    new = klass(**new_params)
    got = new.get_params(deep=False)
    for name in new_params:
        if got[name] is not new_params[name] and not _same_param(got[name], new_params[name]):
            raise RuntimeError(f"Cannot clone object {estimator}, as the constructor either "
                               f"does not set or modifies parameter {name}")
    return new


def _same_param(a, b):
    try:
        if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
            return np.array_equal(np.asarray(a), np.asarray(b))
        return bool(a == b)
    except Exception:  # pragma: no cover - exotic params
        return False


def _validate_fit_y_sw(est, X, y, sample_weight):
    """Target / sample-weight half of the fit contract (reference
    ``check_X_y`` / ``_check_sample_weight`` / ``check_classification_targets``)
    for host arrays: a float y must be finite; a classifier refuses a
    continuous target; sample_weight is a scalar or a 1-D array with one
    entry per row."""
    n = X.shape[0] if isinstance(X, np.ndarray) and X.ndim >= 1 else None
    if y is not None and not isinstance(y, torch.Tensor) and hasattr(y, "__len__") \
            and not hasattr(y, "toarray"):
        ya = np.asarray(y)
        if ya.dtype.kind == "f" and ya.size and not np.isfinite(ya).all():
            raise ValueError("Input y contains NaN or infinity.")
        if ya.dtype.kind == "c":
            raise ValueError("Complex data not supported")
        if getattr(est, "_estimator_type", None) == "classifier" and ya.dtype.kind == "f" \
                and ya.ndim == 1 and ya.size and np.any(ya != np.round(ya)):
            from .utils.multiclass import check_classification_targets
            check_classification_targets(ya)
    if sample_weight is not None and n is not None and not np.isscalar(sample_weight) \
            and not isinstance(sample_weight, torch.Tensor):
        sw = np.asarray(sample_weight)
        if sw.ndim != 1:
            raise ValueError("Sample weights must be 1D array or scalar")
        if sw.shape[0] != n:
            raise ValueError(f"sample_weight.shape == {sw.shape}, expected {(n,)}!")


def _validate_fit_X(est, X):
    """The reference's ``check_array`` contract at ``fit`` for dense numeric
    host arrays (``utils/validation.py:477-760``): at least one sample and one
    feature, no NaN unless the estimator's ``allow_nan`` tag says so, never
    infinity.  Device tensors / sharded arrays are validated by the device
    layer (``models/_data.py``), other input kinds by the estimators."""
    if isinstance(X, np.ndarray) and X.dtype.kind == "c":
        raise ValueError("Complex data not supported")
    if not isinstance(X, np.ndarray) or X.ndim != 2 or X.dtype.kind not in "fiub":
        return
    tags = est._get_tags()
    if "2darray" not in tags.get("X_types", ["2darray"]):
        return
    name = type(est).__name__
    if X.shape[0] == 0:
        raise ValueError(f"Found array with 0 sample(s) (shape={X.shape}) while a minimum of 1 "
                         f"is required by {name}.")
    if X.shape[1] == 0:
        raise ValueError(f"Found array with 0 feature(s) (shape={X.shape}) while a minimum of 1 "
                         f"is required by {name}.")
    if X.dtype.kind == "f" and not np.isfinite(X).all():
        if np.isinf(X).any():
            raise ValueError(f"Input X contains infinity or a value too large for {X.dtype!r}.")
        if not tags.get("allow_nan", False):
            raise ValueError(f"Input X contains NaN. {name} does not accept missing values "
                             "encoded as NaN natively.")


def _current_cuda_device():
    import sys
    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_initialized():
        return None
    return torch.cuda.current_device()


def _validating_fit(fit):
    try:
        names = [p for p in inspect.signature(fit).parameters][1:]
    except (TypeError, ValueError):  # pragma: no cover
        names = []
    i_y = names.index("y") if "y" in names else None
    i_sw = names.index("sample_weight") if "sample_weight" in names else None

    @functools.wraps(fit)
    def fit_validated(self, *args, **kwargs):
        X = args[0] if args else kwargs.get("X")
        if X is not None:
            _validate_fit_X(self, X)
            y = args[i_y] if i_y is not None and len(args) > i_y else kwargs.get("y")
            sw = (args[i_sw] if i_sw is not None and len(args) > i_sw
                  else kwargs.get("sample_weight"))
            _validate_fit_y_sw(self, X, y, sw)
        # native launches make the data's GPU the thread's current device
        # (ops._native.stream_handle): give the caller back its own afterwards
        prev = _current_cuda_device()
        try:
            return fit(self, *args, **kwargs)
        finally:
            if prev is not None and _current_cuda_device() != prev:
                import torch
                torch.cuda.set_device(prev)
    fit_validated._sq_validated = True
    return fit_validated


class BaseEstimator:
    """Base class for all estimators of the framework."""

    def __init_subclass__(cls, **kwargs):
        # every estimator's fit validates its dense host input like the
        # reference's check_array (one wrapper per class that defines fit)
        super().__init_subclass__(**kwargs)
        fit = cls.__dict__.get("fit")
        if fit is not None and callable(fit) and not getattr(fit, "_sq_validated", False):
            cls.fit = _validating_fit(fit)

    @classmethod
    def _get_param_names(cls):
        init = getattr(cls.__init__, "deprecated_original", cls.__init__)
        if init is object.__init__:
            return []
        sig = inspect.signature(init)
        params = [p for p in sig.parameters.values() if p.name != "self" and p.kind != p.VAR_KEYWORD]
        for p in params:
            if p.kind == p.VAR_POSITIONAL:
                raise RuntimeError(f"{cls} should not have *args in __init__ ({sig}).")
        return sorted(p.name for p in params)

    def get_params(self, deep=True):
        out = {}
        for key in self._get_param_names():
            value = getattr(self, key)
            if deep and hasattr(value, "get_params") and not isinstance(value, type):
                for k, v in value.get_params().items():
                    out[f"{key}__{k}"] = v
            out[key] = value
        return out

    def set_params(self, **params):
        if not params:
            return self
        valid = self.get_params(deep=True)
        nested = defaultdict(dict)
        for key, value in params.items():
            key, delim, sub = key.partition("__")
            if key not in valid:
                raise ValueError(f"Invalid parameter {key!r} for estimator {self}. "
                                 "Check the list of available parameters with "
                                 "`estimator.get_params().keys()`.")
            if delim:
                nested[key][sub] = value
            else:
                setattr(self, key, value)
                valid[key] = value
        for key, sub in nested.items():
            valid[key].set_params(**sub)
        return self

    def __repr__(self):
        from ._config import get_config
        changed_only = get_config()["print_changed_only"]
        params = self.get_params(deep=False)
        if changed_only:
            init_params = {}
            try:
                sig = inspect.signature(self.__class__.__init__)
                init_params = {k: v.default for k, v in sig.parameters.items()}
            except (TypeError, ValueError):  # pragma: no cover
                pass
            params = {k: v for k, v in params.items()
                      if k not in init_params or not _same_param(v, init_params[k])
                      or type(v) is not type(init_params[k])}
        body = ", ".join(f"{k}={v!r}" for k, v in sorted(params.items()))
        return f"{self.__class__.__name__}({body})"

    # ------------------------------------------------------------------ pickle
    def __getstate__(self):
        state = dict(self.__dict__)
        for k, v in list(state.items()):
            if isinstance(v, torch.Tensor):
                t = v.detach()
                if t.dtype == torch.bfloat16:
                    t = t.float()
                state[k] = t.cpu().numpy()
            elif k.startswith("_engine") or k.startswith("_pg"):
                # runtime handles (process groups, kernel workspaces) are not state
                state[k] = None
        if type(self).__module__.startswith("sq_learn_amd."):
            state["_sq_learn_amd_version"] = _framework_version()
        return state

    def __setstate__(self, state):
        if type(self).__module__.startswith("sq_learn_amd."):
            v = state.pop("_sq_learn_amd_version", "pre-0.1")
            if v != _framework_version():
                warnings.warn(InconsistentVersionWarning(
                    estimator_name=self.__class__.__name__,
                    current_version=_framework_version(), original_version=v))
        self.__dict__.update(state)

    # ----------------------------------------------------------- validation
    def _more_tags(self):
        return {}

    def _get_tags(self):
        tags = {"non_deterministic": False, "requires_y": False, "X_types": ["2darray"],
                "preserves_dtype": [np.float64], "allow_nan": False, "stateless": False}
        for base in reversed(inspect.getmro(self.__class__)):
            if hasattr(base, "_more_tags") and "_more_tags" in vars(base):
                tags.update(base._more_tags(self))
        return tags

    def _check_n_features(self, X, reset):
        n = X.shape[1]
        if reset:
            self.n_features_in_ = n
            return
        if not hasattr(self, "n_features_in_"):
            return
        if n != self.n_features_in_:
            raise ValueError(f"X has {n} features, but {self.__class__.__name__} "
                             f"is expecting {self.n_features_in_} features as input.")

    def _validate_data(self, X, y="no_validation", reset=True, validate_separately=False,
                       **check_params):
        from .utils.validation import check_array, check_X_y
        no_y = isinstance(y, str) and y == "no_validation"
        if no_y:
            X = check_array(X, **check_params)
            out = X
        elif validate_separately:
            cx, cy = validate_separately
            X = check_array(X, **cx)
            y = check_array(y, **cy)
            out = X, y
        else:
            X, y = check_X_y(X, y, **check_params)
            out = X, y
        if check_params.get("ensure_2d", True):
            self._check_n_features(X, reset=reset)
        return out


class ClassifierMixin:
    _estimator_type = "classifier"

    def score(self, X, y, sample_weight=None):
        from .utils.metrics import accuracy_score
        return accuracy_score(y, self.predict(X), sample_weight=sample_weight)

    def _more_tags(self):
        return {"requires_y": True}


class RegressorMixin:
    _estimator_type = "regressor"

    def score(self, X, y, sample_weight=None):
        from .utils.metrics import r2_score
        return r2_score(y, self.predict(X), sample_weight=sample_weight)

    def _more_tags(self):
        return {"requires_y": True}


class ClusterMixin:
    _estimator_type = "clusterer"

    def fit_predict(self, X, y=None, **kw):
        self.fit(X, **kw)
        return self.labels_


class TransformerMixin:
    def fit_transform(self, X, y=None, **fit_params):
        if y is None:
            return self.fit(X, **fit_params).transform(X)
        return self.fit(X, y, **fit_params).transform(X)

    def get_feature_names_out(self, input_features=None):
        """Output feature names: ``<classname><i>`` for projecting
        transformers (those with ``components_`` / ``_n_features_out``),
        otherwise one-to-one with the input names."""
        n_out = getattr(self, "_n_features_out", None)
        comps = getattr(self, "components_", None)
        if n_out is None and comps is not None and hasattr(comps, "shape"):
            n_out = comps.shape[0]
        if n_out is not None:
            prefix = type(self).__name__.lower()
            return np.asarray([f"{prefix}{i}" for i in range(n_out)], dtype=object)
        if input_features is not None:
            return np.asarray(input_features, dtype=object)
        names = getattr(self, "feature_names_in_", None)
        if names is not None:
            return np.asarray(names, dtype=object)
        n = getattr(self, "n_features_in_", None)
        if n is None:
            raise AttributeError(f"{type(self).__name__} is not fitted; call fit first.")
        return np.asarray([f"x{i}" for i in range(n)], dtype=object)


class DensityMixin:
    _estimator_type = "DensityEstimator"

    def score(self, X, y=None):
        pass


class MetaEstimatorMixin:
    """Marker for estimators wrapping a sub-estimator."""
    _required_parameters = ["estimator"]


class MultiOutputMixin:
    """Marker: supports multi-output targets."""

    def _more_tags(self):
        return {"multioutput": True}


class BiclusterMixin:
    """Row/column index helpers for biclustering estimators."""

    @property
    def biclusters_(self):
        return self.rows_, self.columns_

    def get_indices(self, i):
        import numpy as np
        return np.nonzero(self.rows_[i])[0], np.nonzero(self.columns_[i])[0]

    def get_shape(self, i):
        r, c = self.get_indices(i)
        return len(r), len(c)

    def get_submatrix(self, i, data):
        import numpy as np
        r, c = self.get_indices(i)
        return np.asarray(data)[r[:, None], c]


class OutlierMixin:
    """Outlier detectors: ``fit_predict`` returns +1 inliers / -1 outliers
    (reference sklearn/base.py:OutlierMixin)."""
    _estimator_type = "outlier_detector"

    def fit_predict(self, X, y=None):
        return self.fit(X).predict(X)


def is_outlier_detector(est):
    return getattr(est, "_estimator_type", None) == "outlier_detector"


def is_classifier(est):
    return getattr(est, "_estimator_type", None) == "classifier"


def is_regressor(est):
    return getattr(est, "_estimator_type", None) == "regressor"


def is_clusterer(est):
    return getattr(est, "_estimator_type", None) == "clusterer"
