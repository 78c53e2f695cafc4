"""Pairwise distances and kernels on device tensors (reference
``sklearn/metrics/pairwise.py``: ``euclidean_distances`` :203, kernels
:1011-1139, ``pairwise_distances_chunked`` :1503).

Kernel matrices are one library GEMM (hipBLASLt via torch.matmul) plus an
elementwise epilogue; distance matrices are chunked by the configured
``working_memory`` so 10^5 x 10^5 problems never materialise at once.
"""

import numpy as np
import torch

from .._config import get_config
from ..runtime.device import to_tensor, to_numpy, resolve_device


def _pair(X, Y, device=None):
    dev = X.device if isinstance(X, torch.Tensor) else resolve_device(device)
    X = to_tensor(X, dev)
    if not X.is_floating_point() or X.dtype == torch.bfloat16:
        X = X.double() if dev.type == "cpu" else X.float()
    Y = X if Y is None else to_tensor(Y, dev).to(X.dtype)
    return X, Y


def euclidean_distances(X, Y=None, *, squared=False, X_norm_squared=None, Y_norm_squared=None,
                        device=None):
    numpy_in = not isinstance(X, torch.Tensor)
    X, Y = _pair(X, Y, device)
    xn = (X * X).sum(1) if X_norm_squared is None else to_tensor(X_norm_squared, X.device).reshape(-1).to(X.dtype)
    yn = (Y * Y).sum(1) if Y_norm_squared is None else to_tensor(Y_norm_squared, X.device).reshape(-1).to(X.dtype)
    D = (xn[:, None] + yn[None, :] - 2.0 * (X @ Y.T)).clamp_(min=0.0)
    if X is Y:
        D.fill_diagonal_(0.0)
    if not squared:
        D = torch.sqrt(D)
    return to_numpy(D) if numpy_in else D


def linear_kernel(X, Y=None, dense_output=True, device=None):
    numpy_in = not isinstance(X, torch.Tensor)
    X, Y = _pair(X, Y, device)
    K = X @ Y.T
    return to_numpy(K) if numpy_in else K


def polynomial_kernel(X, Y=None, degree=3, gamma=None, coef0=1, device=None):
    numpy_in = not isinstance(X, torch.Tensor)
    X, Y = _pair(X, Y, device)
    if gamma is None:
        gamma = 1.0 / X.shape[1]
    K = (gamma * (X @ Y.T) + coef0) ** degree
    return to_numpy(K) if numpy_in else K


def sigmoid_kernel(X, Y=None, gamma=None, coef0=1, device=None):
    numpy_in = not isinstance(X, torch.Tensor)
    X, Y = _pair(X, Y, device)
    if gamma is None:
        gamma = 1.0 / X.shape[1]
    K = torch.tanh(gamma * (X @ Y.T) + coef0)
    return to_numpy(K) if numpy_in else K


def rbf_kernel(X, Y=None, gamma=None, device=None):
    numpy_in = not isinstance(X, torch.Tensor)
    X, Y = _pair(X, Y, device)
    if gamma is None:
        gamma = 1.0 / X.shape[1]
    D = euclidean_distances(X, Y, squared=True)
    K = torch.exp(-gamma * D)
    return to_numpy(K) if numpy_in else K


PAIRWISE_KERNEL_FUNCTIONS = {"linear": linear_kernel, "poly": polynomial_kernel,
                             "polynomial": polynomial_kernel, "rbf": rbf_kernel,
                             "sigmoid": sigmoid_kernel}


def pairwise_kernels(X, Y=None, metric="linear", **kw):
    return PAIRWISE_KERNEL_FUNCTIONS[metric](X, Y, **kw)


def get_chunk_n_rows(row_bytes, *, max_n_rows=None, working_memory=None):
    """Rows that fit in ``working_memory`` MiB (reference ``utils/__init__.py:918``)."""
    if working_memory is None:
        working_memory = get_config()["working_memory"]
    n = int(working_memory * (2 ** 20) // row_bytes)
    if max_n_rows is not None:
        n = min(n, max_n_rows)
    return max(n, 1)


def pairwise_distances_chunked(X, Y=None, *, reduce_func=None, working_memory=None, device=None):
    """Yield distance blocks of at most ``working_memory`` MiB."""
    X, Y = _pair(X, Y, device)
    rows = get_chunk_n_rows(Y.shape[0] * X.element_size(), working_memory=working_memory)
    yn = (Y * Y).sum(1)
    for s in range(0, X.shape[0], rows):
        xb = X[s:s + rows]
        D = torch.sqrt(((xb * xb).sum(1)[:, None] + yn[None, :] - 2.0 * (xb @ Y.T)).clamp_(min=0))
        yield reduce_func(D, s) if reduce_func is not None else D


def gen_batches(n, batch_size, *, min_batch_size=0):
    start = 0
    for _ in range(int(n // batch_size)):
        end = start + batch_size
        if end + min_batch_size > n:
            continue
        yield slice(start, end)
        start = end
    if start < n:
        yield slice(start, n)


def gen_even_slices(n, n_packs, *, n_samples=None):
    start = 0
    for pack_num in range(n_packs):
        this_n = n // n_packs
        if pack_num < n % n_packs:
            this_n += 1
        if this_n > 0:
            end = start + this_n
            if n_samples is not None:
                end = min(n_samples, end)
            yield slice(start, end, None)
            start = end


# ------------------------------------------------------------ non-GEMM metrics
_OPS = {"l1": 0, "chi2": 1, "chebyshev": 2, "minkowski": 3}


def _torch_reduce(X, Y, op, p):
    rows = get_chunk_n_rows(max(Y.shape[0] * X.shape[1], 1) * X.element_size())
    out = torch.empty((X.shape[0], Y.shape[0]), dtype=X.dtype, device=X.device)
    for s in range(0, X.shape[0], rows):
        xb = X[s:s + rows, None, :]
        yb = Y[None, :, :]
        if op == "chi2":
            num = (xb - yb) ** 2
            den = xb + yb
            out[s:s + rows] = -torch.where(den != 0, num / torch.where(den != 0, den, 1), 0).sum(2)
        else:
            out[s:s + rows] = torch.cdist(X[s:s + rows], Y, p={"l1": 1.0, "chebyshev": float("inf"),
                                                               "minkowski": p}[op])
    return out


def pairwise_reduce(X, Y, op, p=2.0):
    """Dense (n, d) x (m, d) -> (n, m) for op in l1 | chi2 | chebyshev |
    minkowski: HIP tile kernel (``csrc/pairwise_fast.hip``) on the GPU,
    torch on the CPU."""
    if X.is_cuda:
        from ..ops import _native as nat
        X = X.contiguous()
        Y = Y.contiguous()
        if X.dtype not in (torch.float32, torch.float64):
            X, Y = X.float(), Y.float()
        out = torch.empty((X.shape[0], Y.shape[0]), dtype=X.dtype, device=X.device)
        nat.native().pairwise_reduce(X.data_ptr(), Y.data_ptr(), out.data_ptr(), X.shape[0],
                                     Y.shape[0], X.shape[1], _OPS[op], float(p),
                                     0 if X.dtype == torch.float32 else 1,
                                     nat.stream_handle(X.device))
        return out
    return _torch_reduce(X, Y, op, p)


def _is_sparse(a):
    try:
        import scipy.sparse as sp
        return sp.issparse(a)
    except ImportError:  # pragma: no cover
        return False


def manhattan_distances(X, Y=None, *, sum_over_features=True, device=None):
    """L1 distances; CSR inputs use the host-native sorted-index merge
    (reference ``_sparse_manhattan``), dense ones the tile kernel."""
    if _is_sparse(X) or _is_sparse(Y):
        import scipy.sparse as sp
        from ..ops import _host
        if not sum_over_features:
            raise TypeError("sum_over_features=False not supported for sparse matrices")
        Xs = sp.csr_matrix(X, dtype=np.float64)
        Ys = Xs if Y is None else sp.csr_matrix(Y, dtype=np.float64)
        Xs.sum_duplicates()
        Ys.sum_duplicates()
        D = np.zeros((Xs.shape[0], Ys.shape[0]))
        a = [np.ascontiguousarray(v) for v in (Xs.data, Xs.indices.astype(np.int32),
                                                Xs.indptr.astype(np.int64), Ys.data,
                                                Ys.indices.astype(np.int32),
                                                Ys.indptr.astype(np.int64))]
        _host.lib().sqh_sparse_manhattan(*[_host.ptr(v) for v in a], Xs.shape[0], Ys.shape[0],
                                         _host.ptr(D))
        return D
    numpy_in = not isinstance(X, torch.Tensor)
    X, Y = _pair(X, Y, device)
    if not sum_over_features:
        D = (X[:, None, :] - Y[None, :, :]).abs().reshape(-1, X.shape[1])
    else:
        D = pairwise_reduce(X, Y, "l1")
    return to_numpy(D) if numpy_in else D


def cosine_similarity(X, Y=None, dense_output=True, device=None):
    numpy_in = not isinstance(X, torch.Tensor)
    X, Y = _pair(X, Y, device)
    Xn = X / torch.linalg.vector_norm(X, dim=1, keepdim=True).clamp(min=torch.finfo(X.dtype).tiny)
    Yn = Xn if Y is X else Y / torch.linalg.vector_norm(Y, dim=1, keepdim=True).clamp(
        min=torch.finfo(Y.dtype).tiny)
    K = Xn @ Yn.T
    return to_numpy(K) if numpy_in else K


def cosine_distances(X, Y=None, device=None):
    numpy_in = not isinstance(X, torch.Tensor)
    S = cosine_similarity(X if not numpy_in else to_tensor(X, resolve_device(device)),
                          None if Y is None else (Y if not numpy_in else
                                                  to_tensor(Y, resolve_device(device))))
    D = (1.0 - S).clamp_(0.0, 2.0)
    if Y is None:
        D.fill_diagonal_(0.0)
    return to_numpy(D) if numpy_in else D


def additive_chi2_kernel(X, Y=None, device=None):
    """k(x, y) = -sum (x - y)^2 / (x + y) (non-negative inputs)."""
    numpy_in = not isinstance(X, torch.Tensor)
    X, Y = _pair(X, Y, device)
    if bool((X < 0).any()):
        raise ValueError("X contains negative values.")
    if Y is not X and bool((Y < 0).any()):
        raise ValueError("Y contains negative values.")
    K = pairwise_reduce(X, Y, "chi2")
    return to_numpy(K) if numpy_in else K


def chi2_kernel(X, Y=None, gamma=1.0, device=None):
    numpy_in = not isinstance(X, torch.Tensor)
    K = additive_chi2_kernel(X if not numpy_in else to_tensor(X, resolve_device(device)),
                             None if Y is None else (Y if not numpy_in else
                                                     to_tensor(Y, resolve_device(device))))
    K = torch.exp(gamma * K)
    return to_numpy(K) if numpy_in else K


def laplacian_kernel(X, Y=None, gamma=None, device=None):
    numpy_in = not isinstance(X, torch.Tensor)
    X, Y = _pair(X, Y, device)
    if gamma is None:
        gamma = 1.0 / X.shape[1]
    K = torch.exp(-gamma * pairwise_reduce(X, Y, "l1"))
    return to_numpy(K) if numpy_in else K


def haversine_distances(X, Y=None, device=None):
    numpy_in = not isinstance(X, torch.Tensor)
    X, Y = _pair(X, Y, device)
    if X.shape[1] != 2 or Y.shape[1] != 2:
        raise ValueError("Haversine distance only valid in 2 dimensions")
    lat1, lon1 = X[:, 0:1], X[:, 1:2]
    lat2, lon2 = Y[:, 0][None, :], Y[:, 1][None, :]
    a = (torch.sin((lat2 - lat1) / 2) ** 2
         + torch.cos(lat1) * torch.cos(lat2) * torch.sin((lon2 - lon1) / 2) ** 2)
    D = 2 * torch.arcsin(torch.sqrt(a.clamp(0, 1)))
    return to_numpy(D) if numpy_in else D


def _euclid(X, Y=None, **kw):
    return euclidean_distances(X, Y, **kw)


def _sqeuclid(X, Y=None, **kw):
    return euclidean_distances(X, Y, squared=True, **kw)


def _minkowski(X, Y=None, p=2, w=None, device=None):
    numpy_in = not isinstance(X, torch.Tensor)
    X, Y = _pair(X, Y, device)
    if w is not None:
        wt = to_tensor(np.asarray(w), X.device).to(X.dtype) ** (1.0 / p)
        X, Y = X * wt, Y * wt
    D = pairwise_reduce(X, Y, "minkowski", p=float(p)) if p not in (1, 2) else (
        pairwise_reduce(X, Y, "l1") if p == 1 else euclidean_distances(X, Y))
    return to_numpy(D) if numpy_in else D


def _chebyshev(X, Y=None, device=None):
    numpy_in = not isinstance(X, torch.Tensor)
    X, Y = _pair(X, Y, device)
    D = pairwise_reduce(X, Y, "chebyshev")
    return to_numpy(D) if numpy_in else D


PAIRWISE_DISTANCE_FUNCTIONS = {
    "cityblock": manhattan_distances, "cosine": cosine_distances, "euclidean": _euclid,
    "haversine": haversine_distances, "l2": _euclid, "l1": manhattan_distances,
    "manhattan": manhattan_distances, "sqeuclidean": _sqeuclid, "chebyshev": _chebyshev,
    "minkowski": _minkowski,
}
PAIRWISE_KERNEL_FUNCTIONS.update({"additive_chi2": additive_chi2_kernel, "chi2": chi2_kernel,
                                  "cosine": cosine_similarity, "laplacian": laplacian_kernel})


def pairwise_distances(X, Y=None, metric="euclidean", *, n_jobs=None, force_all_finite=True,
                       **kwds):
    """Distance matrix for a named metric, 'precomputed' or a callable
    (reference ``metrics/pairwise.py: pairwise_distances``)."""
    if metric == "precomputed":
        return np.asarray(X) if not isinstance(X, torch.Tensor) else X
    if callable(metric):
        Xa = np.asarray(X)
        Ya = Xa if Y is None else np.asarray(Y)
        out = np.zeros((Xa.shape[0], Ya.shape[0]))
        for i in range(Xa.shape[0]):
            for j in range(Ya.shape[0]):
                out[i, j] = metric(Xa[i], Ya[j], **kwds)
        return out
    if metric not in PAIRWISE_DISTANCE_FUNCTIONS:
        from scipy.spatial.distance import cdist
        Xa = np.asarray(X, dtype=np.float64)
        return cdist(Xa, Xa if Y is None else np.asarray(Y, dtype=np.float64), metric=metric,
                     **kwds)
    return PAIRWISE_DISTANCE_FUNCTIONS[metric](X, Y, **kwds)


def pairwise_distances_argmin_min(X, Y, *, axis=1, metric="euclidean", metric_kwargs=None,
                                  device=None):
    """(argmin, min) over Y for every row of X, in device chunks."""
    if axis == 0:
        X, Y = Y, X
    numpy_in = not isinstance(X, torch.Tensor)
    X, Y = _pair(X, Y, device)
    rows = get_chunk_n_rows(max(Y.shape[0], 1) * X.element_size())
    idx = torch.empty(X.shape[0], dtype=torch.int64, device=X.device)
    val = torch.empty(X.shape[0], dtype=X.dtype, device=X.device)
    for s in range(0, X.shape[0], rows):
        D = pairwise_distances(X[s:s + rows], Y, metric=metric, **(metric_kwargs or {}))
        D = torch.as_tensor(D, device=X.device)
        m = D.min(1)
        idx[s:s + rows] = m.indices
        val[s:s + rows] = m.values.to(val.dtype)
    if numpy_in:
        return to_numpy(idx), to_numpy(val)
    return idx, val


def pairwise_distances_argmin(X, Y, *, axis=1, metric="euclidean", metric_kwargs=None):
    return pairwise_distances_argmin_min(X, Y, axis=axis, metric=metric,
                                         metric_kwargs=metric_kwargs)[0]


def paired_distances(X, Y, *, metric="euclidean", **kwds):
    """Row-wise distances d(X[i], Y[i])."""
    numpy_in = not isinstance(X, torch.Tensor)
    Xt, Yt = _pair(X, Y)
    if Xt.shape != Yt.shape:
        raise ValueError("X and Y should be of same shape. They were respectively %r and %r long."
                         % (tuple(Xt.shape), tuple(Yt.shape)))
    if metric in ("euclidean", "l2"):
        D = torch.linalg.vector_norm(Xt - Yt, dim=1)
    elif metric in ("manhattan", "l1", "cityblock"):
        D = (Xt - Yt).abs().sum(1)
    elif metric == "cosine":
        Xn = Xt / torch.linalg.vector_norm(Xt, dim=1, keepdim=True)
        Yn = Yt / torch.linalg.vector_norm(Yt, dim=1, keepdim=True)
        D = 0.5 * ((Xn - Yn) ** 2).sum(1)
    elif callable(metric):
        Xa, Ya = np.asarray(X), np.asarray(Y)
        return np.array([metric(Xa[i], Ya[i]) for i in range(len(Xa))])
    else:
        raise ValueError("Unknown distance %s" % metric)
    return to_numpy(D) if numpy_in else D


def paired_euclidean_distances(X, Y):
    return paired_distances(X, Y, metric="euclidean")


def paired_manhattan_distances(X, Y):
    return paired_distances(X, Y, metric="manhattan")


def paired_cosine_distances(X, Y):
    return paired_distances(X, Y, metric="cosine")
