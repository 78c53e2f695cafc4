"""Feature scaling (reference ``sklearn/preprocessing/_data.py``:
``StandardScaler`` :582, ``MinMaxScaler`` :270, ``normalize`` :1680,
``Normalizer`` :1786; SURVEY.md §2.7 "StandardScaler is B").

Statistics are computed in fp64 on the data's device (numpy in -> numpy
out, tensor in -> tensor out).  ``partial_fit`` merges batch moments with
Chan's parallel update, which is also what a row-sharded fit reduces: pass
``comm`` (a :class:`~sq_learn_amd.parallel.comm.Comm`) and every rank ends
with the global moments after one packed all-reduce.
"""

import numpy as np
import torch

from ..base import BaseEstimator, TransformerMixin
from ..runtime.device import to_numpy
from ..utils.validation import check_array, check_is_fitted


def _as_tensor64(X):
    if isinstance(X, torch.Tensor):
        return X.to(torch.float64), True
    return torch.as_tensor(np.asarray(check_array(X), dtype=np.float64)), False


def _check_nf(est, Xt):
    if Xt.shape[1] != est.n_features_in_:
        raise ValueError(f"X has {Xt.shape[1]} features, but {type(est).__name__} is expecting "
                         f"{est.n_features_in_} features as input.")


def _out(t, was_tensor, like=None):
    if was_tensor:
        return t.to(like.dtype) if like is not None and like.is_floating_point() else t
    return t.cpu().numpy()


class StandardScaler(TransformerMixin, BaseEstimator):
    def __init__(self, *, copy=True, with_mean=True, with_std=True, comm=None):
        self.copy = copy
        self.with_mean = with_mean
        self.with_std = with_std
        self.comm = comm

    def _reset(self):
        for a in ("n_samples_seen_", "mean_", "var_", "scale_"):
            if hasattr(self, a):
                delattr(self, a)

    def fit(self, X, y=None, sample_weight=None):
        self._reset()
        return self.partial_fit(X, y, sample_weight)

    def partial_fit(self, X, y=None, sample_weight=None):
        Xt, _ = _as_tensor64(X)
        if sample_weight is None:
            w = torch.ones(Xt.shape[0], dtype=torch.float64, device=Xt.device)
        else:
            w = torch.as_tensor(np.asarray(to_numpy(sample_weight), dtype=np.float64),
                                device=Xt.device)
        n_b = w.sum()
        s1 = (Xt * w[:, None]).sum(0)
        if self.comm is not None and self.comm.world_size > 1:
            buf = torch.cat([n_b.reshape(1), s1])
            self.comm.all_reduce_(buf)
            n_b, s1 = buf[0], buf[1:]
        mean_b = s1 / n_b
        dev = Xt - mean_b
        m2_b = (dev * dev * w[:, None]).sum(0)
        if self.comm is not None and self.comm.world_size > 1:
            self.comm.all_reduce_(m2_b)
        n_b = float(n_b)
        mean_b, m2_b = mean_b.cpu().numpy(), m2_b.cpu().numpy()
        if not hasattr(self, "n_samples_seen_"):
            self.n_features_in_ = Xt.shape[1]
            n, mean, m2 = n_b, mean_b, m2_b
        else:
            if Xt.shape[1] != self.n_features_in_:
                raise ValueError(f"X has {Xt.shape[1]} features, but StandardScaler is "
                                 f"expecting {self.n_features_in_} features as input.")
            # Chan et al. pairwise update of (count, mean, M2)
            n_a, mean_a, var_a = self._running
            n = n_a + n_b
            d = mean_b - mean_a
            mean = mean_a + d * (n_b / n)
            m2 = var_a * n_a + m2_b + d * d * (n_a * n_b / n)
        var = m2 / n
        self._running = (n, mean, var)   # kept whatever with_mean / with_std say
        self.n_samples_seen_ = int(n) if float(n).is_integer() else n
        self.mean_ = mean if self.with_mean else None
        self.var_ = var if self.with_std else None
        if self.with_std:
            scale = np.sqrt(var)
            scale[scale < 10 * np.finfo(np.float64).eps] = 1.0
            self.scale_ = scale
        else:
            self.scale_ = None
        return self

    def transform(self, X, copy=None):
        check_is_fitted(self, "n_samples_seen_")
        Xt, was_t = _as_tensor64(X)
        _check_nf(self, Xt)
        if self.with_mean:
            Xt = Xt - torch.as_tensor(self.mean_, device=Xt.device)
        if self.with_std:
            Xt = Xt / torch.as_tensor(self.scale_, device=Xt.device)
        return _out(Xt, was_t, X if was_t else None)

    def inverse_transform(self, X, copy=None):
        check_is_fitted(self, "n_samples_seen_")
        Xt, was_t = _as_tensor64(X)
        _check_nf(self, Xt)
        if self.with_std:
            Xt = Xt * torch.as_tensor(self.scale_, device=Xt.device)
        if self.with_mean:
            Xt = Xt + torch.as_tensor(self.mean_, device=Xt.device)
        return _out(Xt, was_t, X if was_t else None)


class MinMaxScaler(TransformerMixin, BaseEstimator):
    def __init__(self, feature_range=(0, 1), *, copy=True, clip=False):
        self.feature_range = feature_range
        self.copy = copy
        self.clip = clip

    def fit(self, X, y=None):
        for a in ("data_min_", "n_samples_seen_"):
            if hasattr(self, a):
                delattr(self, a)
        return self.partial_fit(X)

    def partial_fit(self, X, y=None):
        lo, hi = self.feature_range
        if lo >= hi:
            raise ValueError("Minimum of desired feature range must be smaller than maximum. "
                             f"Got {self.feature_range}.")
        Xt, _ = _as_tensor64(X)
        dmin = Xt.min(0).values.cpu().numpy()
        dmax = Xt.max(0).values.cpu().numpy()
        if hasattr(self, "n_samples_seen_"):
            dmin = np.minimum(self.data_min_, dmin)
            dmax = np.maximum(self.data_max_, dmax)
            self.n_samples_seen_ += Xt.shape[0]
        else:
            self.n_samples_seen_ = Xt.shape[0]
            self.n_features_in_ = Xt.shape[1]
        rng = dmax - dmin
        rng_safe = np.where(rng == 0, 1.0, rng)
        self.scale_ = (hi - lo) / rng_safe
        self.min_ = lo - dmin * self.scale_
        self.data_min_, self.data_max_, self.data_range_ = dmin, dmax, rng
        return self

    def transform(self, X):
        check_is_fitted(self, "scale_")
        Xt, was_t = _as_tensor64(X)
        _check_nf(self, Xt)
        Xt = Xt * torch.as_tensor(self.scale_, device=Xt.device) + torch.as_tensor(self.min_,
                                                                                   device=Xt.device)
        if self.clip:
            Xt = Xt.clamp(self.feature_range[0], self.feature_range[1])
        return _out(Xt, was_t, X if was_t else None)

    def inverse_transform(self, X):
        check_is_fitted(self, "scale_")
        Xt, was_t = _as_tensor64(X)
        _check_nf(self, Xt)
        Xt = (Xt - torch.as_tensor(self.min_, device=Xt.device)) / torch.as_tensor(
            self.scale_, device=Xt.device)
        return _out(Xt, was_t, X if was_t else None)


def normalize(X, norm="l2", *, axis=1, copy=True, return_norm=False):
    Xt, was_t = _as_tensor64(X)
    if axis == 0:
        Xt = Xt.T
    if norm == "l1":
        nrm = Xt.abs().sum(1)
    elif norm == "l2":
        nrm = torch.sqrt((Xt * Xt).sum(1))
    elif norm == "max":
        nrm = Xt.abs().max(1).values
    else:
        raise ValueError(f"'{norm}' is not a supported norm")
    safe = torch.where(nrm == 0, torch.ones_like(nrm), nrm)
    out = Xt / safe[:, None]
    if axis == 0:
        out = out.T
    res = _out(out, was_t, X if was_t else None)
    if return_norm:
        return res, _out(nrm, was_t)
    return res


class Normalizer(TransformerMixin, BaseEstimator):

    def _more_tags(self):
        return {"stateless": True}

    def __init__(self, norm="l2", *, copy=True):
        self.norm = norm
        self.copy = copy

    def fit(self, X, y=None):
        self.n_features_in_ = np.asarray(to_numpy(X)).shape[1] if not isinstance(X, torch.Tensor) \
            else X.shape[1]
        return self

    def transform(self, X, copy=None):
        return normalize(X, self.norm, axis=1)


__all__ = ["StandardScaler", "MinMaxScaler", "Normalizer", "normalize"]


from ._polynomial import PolynomialFeatures, SplineTransformer  # noqa: E402,F401
from ._encoders import (LabelBinarizer, LabelEncoder, MultiLabelBinarizer,  # noqa: E402,F401
                        OneHotEncoder, OrdinalEncoder, label_binarize)
from ._data_extra import (Binarizer, FunctionTransformer, KBinsDiscretizer,  # noqa: E402,F401
                          KernelCenterer, MaxAbsScaler, PowerTransformer, QuantileTransformer,
                          RobustScaler, add_dummy_feature, binarize,
                          maxabs_scale, power_transform, quantile_transform, robust_scale)

__all__ += ["PolynomialFeatures", "SplineTransformer", "LabelBinarizer", "LabelEncoder", "MultiLabelBinarizer",
            "OneHotEncoder", "OrdinalEncoder", "label_binarize", "Binarizer",
            "FunctionTransformer", "KBinsDiscretizer", "KernelCenterer", "MaxAbsScaler",
            "PowerTransformer", "QuantileTransformer", "RobustScaler",
            "add_dummy_feature", "binarize", "maxabs_scale", "power_transform",
            "quantile_transform", "robust_scale"]


def scale(X, *, axis=0, with_mean=True, with_std=True, copy=True):
    """Standardise along an axis (reference ``preprocessing/_data.py``
    ``scale``: NaN-aware, with the two-pass re-centring of large means)."""
    import warnings as _w
    Xa = np.array(to_numpy(X) if hasattr(X, "detach") else X, dtype=np.float64, copy=True)
    Xr = Xa if axis == 0 else Xa.T
    if with_mean:
        mean_ = np.nanmean(Xr, axis=0)
    if with_std:
        scale_ = np.nanstd(Xr, axis=0)
        scale_ = np.where(scale_ < 10 * np.finfo(scale_.dtype).eps, 1.0, scale_)
    if with_mean:
        Xr -= mean_
        m1 = np.nanmean(Xr, axis=0)
        if not np.allclose(m1, 0):
            _w.warn("Numerical issues were encountered when centering the data and might not "
                    "be solved. Dataset may contain too large values. You may need to prescale "
                    "your features.")
            Xr -= m1
    if with_std:
        Xr /= scale_
        if with_mean:
            m2 = np.nanmean(Xr, axis=0)
            if not np.allclose(m2, 0):
                _w.warn("Numerical issues were encountered when scaling the data and might not "
                        "be solved. The standard deviation of the data is probably very close to "
                        "0. ")
                Xr -= m2
    return Xa


def minmax_scale(X, feature_range=(0, 1), *, axis=0, copy=True):
    """Scale every feature (axis=0) or sample (axis=1) to ``feature_range``."""
    Xa = np.array(to_numpy(X) if hasattr(X, "detach") else X, dtype=np.float64, copy=True)
    orig_1d = Xa.ndim == 1
    if orig_1d:
        Xa = Xa.reshape(-1, 1)
    Xr = Xa if axis == 0 else Xa.T
    lo, hi = feature_range
    if lo >= hi:
        raise ValueError("Minimum of desired feature range must be smaller than maximum. Got %s."
                         % str(feature_range))
    dmin, dmax = np.nanmin(Xr, axis=0), np.nanmax(Xr, axis=0)
    rng = dmax - dmin
    rng = np.where(rng < 10 * np.finfo(np.float64).eps, 1.0, rng)
    s = (hi - lo) / rng
    Xr *= s
    Xr += lo - dmin * s
    return Xa.ravel() if orig_1d else Xa

from ..utils._aliases import alias_submodules  # noqa: E402
alias_submodules(__name__, "_data", "_label")

from ..utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
