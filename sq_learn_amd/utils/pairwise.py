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
