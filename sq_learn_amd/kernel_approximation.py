"""Kernel feature maps (reference ``sklearn/kernel_approximation.py``:
RBFSampler (random Fourier features), SkewedChi2Sampler,
AdditiveChi2Sampler, Nystroem, PolynomialCountSketch) and
``sklearn/kernel_ridge.py`` (KernelRidge) and ``sklearn/random_projection.py``
(Gaussian / sparse random projections, Johnson-Lindenstrauss bound).

Projections and kernel matrices are device GEMMs (fp64 on the resolved
device); random matrices are drawn with numpy ``RandomState`` so seeds give
the reference's matrices."""

import warnings

import numpy as np
import scipy.sparse as sp
import torch

from .base import BaseEstimator, RegressorMixin, TransformerMixin
from .exceptions import DataDimensionalityWarning
from .runtime.device import resolve_device
from .utils.validation import check_is_fitted, check_random_state


def _dense(X):
    if hasattr(X, "detach"):
        X = X.detach().cpu().numpy()
    if sp.issparse(X):
        X = X.toarray()
    return np.asarray(X, dtype=np.float64)


def _mm(A, B, device=None):
    dev = resolve_device(device)
    if dev.type == "cpu":
        return A @ B
    return (torch.as_tensor(A, device=dev) @ torch.as_tensor(B, device=dev)).cpu().numpy()


def _nf(est, X):
    if X.shape[1] != est.n_features_in_:
        raise ValueError(f"X has {X.shape[1]} features, but {type(est).__name__} is expecting "
                         f"{est.n_features_in_} features as input.")


class RBFSampler(TransformerMixin, BaseEstimator):
    def __init__(self, *, gamma=1.0, n_components=100, random_state=None):
        self.gamma = gamma
        self.n_components = n_components
        self.random_state = random_state

    def fit(self, X, y=None):
        X = _dense(X)
        rs = check_random_state(self.random_state)
        self.n_features_in_ = X.shape[1]
        self.random_weights_ = np.sqrt(2 * self.gamma) * rs.normal(
            size=(X.shape[1], self.n_components))
        self.random_offset_ = rs.uniform(0, 2 * np.pi, size=self.n_components)
        return self

    def transform(self, X):
        check_is_fitted(self)
        X = _dense(X)
        self._check_n_features(X, reset=False)
        _nf(self, X)
        proj = _mm(X, self.random_weights_) + self.random_offset_
        return np.cos(proj) * np.sqrt(2.0) / np.sqrt(self.n_components)


class SkewedChi2Sampler(TransformerMixin, BaseEstimator):

    def _more_tags(self):
        return {"requires_positive_X": True}

    def __init__(self, *, skewedness=1.0, n_components=100, random_state=None):
        self.skewedness = skewedness
        self.n_components = n_components
        self.random_state = random_state

    def fit(self, X, y=None):
        X = _dense(X)
        rs = check_random_state(self.random_state)
        self.n_features_in_ = X.shape[1]
        u = rs.uniform(size=(X.shape[1], self.n_components))
        self.random_weights_ = 1.0 / np.pi * np.log(np.tan(np.pi / 2.0 * u))
        self.random_offset_ = rs.uniform(0, 2 * np.pi, size=self.n_components)
        return self

    def transform(self, X):
        check_is_fitted(self)
        X = _dense(X)
        self._check_n_features(X, reset=False)
        if (X <= -self.skewedness).any():
            raise ValueError("X may not contain entries smaller than -skewedness.")
        proj = _mm(np.log(X + self.skewedness), self.random_weights_) + self.random_offset_
        return np.cos(proj) * np.sqrt(2.0) / np.sqrt(self.n_components)


class AdditiveChi2Sampler(TransformerMixin, BaseEstimator):

    def _more_tags(self):
        return {"requires_positive_X": True, "stateless": True}

    def __init__(self, *, sample_steps=2, sample_interval=None):
        self.sample_steps = sample_steps
        self.sample_interval = sample_interval

    def fit(self, X, y=None):
        X = _dense(X)
        self.n_features_in_ = X.shape[1]
        if self.sample_interval is None:
            if self.sample_steps == 1:
                self.sample_interval_ = 0.8
            elif self.sample_steps == 2:
                self.sample_interval_ = 0.5
            elif self.sample_steps == 3:
                self.sample_interval_ = 0.4
            else:
                raise ValueError("If sample_steps is not in [1, 2, 3], you need to provide "
                                 "sample_interval")
        else:
            self.sample_interval_ = self.sample_interval
        return self

    def transform(self, X):
        check_is_fitted(self)
        X = _dense(X)
        self._check_n_features(X, reset=False)
        if (X < 0).any():
            raise ValueError("Negative values in data passed to X in AdditiveChi2Sampler.fit")
        nz = X > 0
        Xn = np.where(nz, X, 1.0)
        logx = np.log(Xn)
        step = np.sqrt(Xn * self.sample_interval_)
        feats = [np.where(nz, step, 0.0)]
        for j in range(1, self.sample_steps):
            factor = np.sqrt(2.0 * Xn * self.sample_interval_
                             / np.cosh(np.pi * j * self.sample_interval_))
            feats.append(np.where(nz, factor * np.cos(j * logx * self.sample_interval_), 0.0))
            feats.append(np.where(nz, factor * np.sin(j * logx * self.sample_interval_), 0.0))
        return np.hstack(feats)


class Nystroem(TransformerMixin, BaseEstimator):
    def __init__(self, kernel="rbf", *, gamma=None, coef0=None, degree=None,
                 kernel_params=None, n_components=100, random_state=None, n_jobs=None):
        self.kernel = kernel
        self.gamma = gamma
        self.coef0 = coef0
        self.degree = degree
        self.kernel_params = kernel_params
        self.n_components = n_components
        self.random_state = random_state
        self.n_jobs = n_jobs

    def _k(self, A, B):
        from .utils.pairwise import pairwise_kernels
        if callable(self.kernel):
            return np.asarray(self.kernel(A, B))
        kw = dict(self.kernel_params or {})
        for name in ("gamma", "coef0", "degree"):
            v = getattr(self, name)
            if v is not None:
                kw[name] = v
        if self.kernel == "linear":
            kw = {}
        elif self.kernel == "rbf":
            kw = {k: v for k, v in kw.items() if k == "gamma"}
        out = pairwise_kernels(A, B, metric=self.kernel, **kw)
        return out.cpu().numpy() if hasattr(out, "cpu") else np.asarray(out)

    def fit(self, X, y=None):
        X = _dense(X)
        rs = check_random_state(self.random_state)
        n_samples = X.shape[0]
        self.n_features_in_ = X.shape[1]
        if self.n_components > n_samples:
            n_components = n_samples
            warnings.warn("n_components > n_samples. This is not possible.\nn_components was set "
                          "to n_samples, which results in inefficient evaluation of the full "
                          "kernel.")
        else:
            n_components = self.n_components
        inds = rs.permutation(n_samples)
        basis_inds = inds[:n_components]
        basis = X[basis_inds]
        K = self._k(basis, basis)
        U, S, V = np.linalg.svd(K)
        S = np.maximum(S, 1e-12)
        self.normalization_ = (U / np.sqrt(S)) @ V
        self.components_ = basis
        self.component_indices_ = basis_inds
        return self

    def transform(self, X):
        check_is_fitted(self)
        X = _dense(X)
        self._check_n_features(X, reset=False)
        return _mm(self._k(X, self.components_), self.normalization_.T)


class PolynomialCountSketch(TransformerMixin, BaseEstimator):
    def __init__(self, *, gamma=1.0, degree=2, coef0=0, n_components=100, random_state=None):
        self.gamma = gamma
        self.degree = degree
        self.coef0 = coef0
        self.n_components = n_components
        self.random_state = random_state

    def fit(self, X, y=None):
        X = _dense(X)
        rs = check_random_state(self.random_state)
        n_features = X.shape[1] + (1 if self.coef0 != 0 else 0)
        self.n_features_in_ = X.shape[1]
        self.indexHash_ = rs.randint(0, high=self.n_components, size=(self.degree, n_features))
        self.bitHash_ = rs.choice(a=[-1, 1], size=(self.degree, n_features))
        return self

    def transform(self, X):
        check_is_fitted(self)
        X = _dense(X) * np.sqrt(self.gamma)
        self._check_n_features(X, reset=False)
        if self.coef0 != 0:
            X = np.hstack([X, np.full((X.shape[0], 1), np.sqrt(self.coef0))])
        count_sketches = np.zeros((X.shape[0], self.degree, self.n_components), dtype=np.complex128)
        for d in range(self.degree):
            for j in range(X.shape[1]):
                count_sketches[:, d, self.indexHash_[d, j]] += self.bitHash_[d, j] * X[:, j]
        cs_fft = np.fft.fft(count_sketches, axis=2)
        cs_fft = np.prod(cs_fft, axis=1)
        return np.real(np.fft.ifft(cs_fft))


class KernelRidge(RegressorMixin, BaseEstimator):
    """Kernel ridge regression: (K + alpha I) dual_coef = y, solved on the
    device (Cholesky; least squares fallback)."""

    def __init__(self, alpha=1, *, kernel="linear", gamma=None, degree=3, coef0=1,
                 kernel_params=None, device=None):
        self.alpha = alpha
        self.kernel = kernel
        self.gamma = gamma
        self.degree = degree
        self.coef0 = coef0
        self.kernel_params = kernel_params
        self.device = device

    def _get_kernel(self, X, Y=None):
        from .utils.pairwise import pairwise_kernels
        if callable(self.kernel):
            return np.asarray(self.kernel(X, Y if Y is not None else X,
                                          **(self.kernel_params or {})))
        if self.kernel == "precomputed":
            return X
        params = dict(self.kernel_params or {}) if self.kernel_params else \
            {"gamma": self.gamma, "degree": self.degree, "coef0": self.coef0}
        allowed = {"linear": (), "rbf": ("gamma",), "laplacian": ("gamma",),
                   "poly": ("gamma", "degree", "coef0"), "polynomial": ("gamma", "degree",
                                                                         "coef0"),
                   "sigmoid": ("gamma", "coef0"), "chi2": ("gamma",), "cosine": ()}
        params = {k: v for k, v in params.items() if k in allowed.get(self.kernel, params)}
        out = pairwise_kernels(X, Y, metric=self.kernel, device=self.device, **params) \
            if "device" in pairwise_kernels.__code__.co_varnames else \
            pairwise_kernels(X, Y, metric=self.kernel, **params)
        return out.cpu().numpy() if hasattr(out, "cpu") else np.asarray(out)

    def fit(self, X, y, sample_weight=None):
        X = _dense(X)
        y = np.asarray(y, dtype=np.float64)
        self.n_features_in_ = X.shape[1]
        K = self._get_kernel(X)
        alpha = np.atleast_1d(self.alpha)
        ravel = y.ndim == 1
        Y = y.reshape(-1, 1) if ravel else y
        if sample_weight is not None:
            sw = np.sqrt(np.asarray(sample_weight, dtype=np.float64))
            K = K * np.outer(sw, sw)
            Y = Y * sw[:, None]
        dev = resolve_device(self.device)
        Kt = torch.as_tensor(K, dtype=torch.float64, device=dev)
        Yt = torch.as_tensor(Y, dtype=torch.float64, device=dev)
        coefs = []
        for k in range(Y.shape[1]):
            a = float(alpha[k] if alpha.size > 1 else alpha[0])
            A = Kt + a * torch.eye(Kt.shape[0], dtype=Kt.dtype, device=dev)
            L, info = torch.linalg.cholesky_ex(A)
            if int(info) == 0:
                c = torch.cholesky_solve(Yt[:, k:k + 1], L)
            else:
                warnings.warn("Singular matrix in solving dual problem. Using least-squares "
                              "solution instead.")
                c = torch.linalg.lstsq(A.cpu(), Yt[:, k:k + 1].cpu()).solution.to(dev)
            coefs.append(c)
        dual = torch.cat(coefs, dim=1).cpu().numpy()
        if sample_weight is not None:
            dual = dual * sw[:, None]
        self.dual_coef_ = dual.ravel() if ravel else dual
        self.X_fit_ = X
        return self

    def predict(self, X):
        check_is_fitted(self)
        X = _dense(X)
        K = self._get_kernel(X, self.X_fit_)
        return _mm(K, self.dual_coef_, self.device)


# --------------------------------------------------------- random projection
def johnson_lindenstrauss_min_dim(n_samples, *, eps=0.1):
    eps = np.asarray(eps)
    n_samples = np.asarray(n_samples)
    if np.any(eps <= 0.0) or np.any(eps >= 1):
        raise ValueError("The JL bound is defined for eps in ]0, 1[, got %r" % eps)
    if np.any(n_samples <= 0):
        raise ValueError("The JL bound is defined for n_samples greater than zero, got %r"
                         % n_samples)
    denominator = (eps ** 2 / 2) - (eps ** 3 / 3)
    return (4 * np.log(n_samples) / denominator).astype(np.int64)


class _BaseRandomProjection(TransformerMixin, BaseEstimator):
    def fit(self, X, y=None):
        Xd = X if sp.issparse(X) else _dense(X)
        n_samples, n_features = Xd.shape
        self.n_features_in_ = n_features
        if self.n_components == "auto":
            self.n_components_ = int(johnson_lindenstrauss_min_dim(n_samples, eps=self.eps))
            if self.n_components_ <= 0:
                raise ValueError("eps=%f and n_samples=%d lead to a target dimension of %d "
                                 "which is invalid" % (self.eps, n_samples, self.n_components_))
            if self.n_components_ > n_features:
                raise ValueError("eps=%f and n_samples=%d lead to a target dimension of %d which "
                                 "is larger than the original space with n_features=%d"
                                 % (self.eps, n_samples, self.n_components_, n_features))
        else:
            if self.n_components <= 0:
                raise ValueError("n_components must be greater than 0, got %s"
                                 % self.n_components)
            if self.n_components > n_features:
                warnings.warn("The number of components is higher than the number of features: "
                              "n_features < n_components (%s < %s).The dimensionality of the "
                              "problem will not be reduced." % (n_features, self.n_components),
                              DataDimensionalityWarning)
            self.n_components_ = self.n_components
        self.components_ = self._make_random_matrix(self.n_components_, n_features)
        return self

    def transform(self, X):
        check_is_fitted(self)
        if sp.issparse(X):
            out = X @ self.components_.T
        else:
            X = _dense(X)
            if X.shape[1] != self.components_.shape[1]:
                raise ValueError("Impossible to perform projection:X at fit stage had a "
                                 "different number of features. (%s != %s)"
                                 % (X.shape[1], self.components_.shape[1]))
            C = self.components_.toarray() if sp.issparse(self.components_) else self.components_
            out = _mm(X, C.T)
        if sp.issparse(out) and not getattr(self, "dense_output", True):
            return out
        return out.toarray() if sp.issparse(out) else out


class GaussianRandomProjection(_BaseRandomProjection):
    def __init__(self, n_components="auto", *, eps=0.1, random_state=None):
        self.n_components = n_components
        self.eps = eps
        self.random_state = random_state

    def _make_random_matrix(self, n_components, n_features):
        rs = check_random_state(self.random_state)
        return rs.normal(loc=0.0, scale=1.0 / np.sqrt(n_components),
                         size=(n_components, n_features))


class SparseRandomProjection(_BaseRandomProjection):
    def __init__(self, n_components="auto", *, density="auto", eps=0.1, dense_output=False,
                 random_state=None):
        self.n_components = n_components
        self.density = density
        self.eps = eps
        self.dense_output = dense_output
        self.random_state = random_state

    def _make_random_matrix(self, n_components, n_features):
        rs = check_random_state(self.random_state)
        density = 1 / np.sqrt(n_features) if self.density == "auto" else self.density
        if density <= 0 or density > 1:
            raise ValueError("Expected density in range ]0, 1], got: %r" % density)
        self.density_ = density
        if density == 1:
            comps = rs.binomial(1, 0.5, (n_components, n_features)) * 2 - 1
            return 1 / np.sqrt(n_components) * comps
        from .utils.random import sample_without_replacement
        indices, offset = [], 0
        indptr = [offset]
        for _ in range(n_components):
            n_nonzero_i = rs.binomial(n_features, density)
            idx = sample_without_replacement(n_features, n_nonzero_i, random_state=rs)
            indices.append(idx)
            offset += n_nonzero_i
            indptr.append(offset)
        indices = np.concatenate(indices)
        data = rs.binomial(1, 0.5, size=np.size(indices)) * 2 - 1
        comps = sp.csr_matrix((data, indices, indptr), shape=(n_components, n_features))
        return np.sqrt(1 / density) / np.sqrt(n_components) * comps


__all__ = ["RBFSampler", "SkewedChi2Sampler", "AdditiveChi2Sampler", "Nystroem",
           "PolynomialCountSketch", "KernelRidge", "GaussianRandomProjection",
           "SparseRandomProjection", "johnson_lindenstrauss_min_dim"]
