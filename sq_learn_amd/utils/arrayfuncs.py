"""Small array kernels (reference ``utils/arrayfuncs.pyx``,
``utils/_logistic_sigmoid.pyx``): ``min_pos``, ``cholesky_delete`` (host
Givens downdate, ``csrc/host/pairwise_host.cpp``) and the numerically
stable log-sigmoid."""

import numpy as np
import torch

from ..ops import _host


def min_pos(X):
    """Smallest strictly positive entry (dtype max if there is none)."""
    X = np.asarray(X)
    if X.dtype not in (np.float32, np.float64):
        raise ValueError("Unsupported dtype for array X")
    pos = X[X > 0]
    return X.dtype.type(pos.min()) if pos.size else np.finfo(X.dtype).max


def cholesky_delete(L, go_out):
    """Remove variable ``go_out`` from the lower Cholesky factor ``L``
    (n x n view, modified in place): row deletion + Givens re-triangulation."""
    n = L.shape[0]
    if L.dtype == np.float64 and L.flags["C_CONTIGUOUS"]:
        _host.lib().sqh_cholesky_delete(_host.ptr(L), n, L.shape[1], int(go_out))
        return L
    work = np.ascontiguousarray(L, dtype=np.float64)
    _host.lib().sqh_cholesky_delete(_host.ptr(work), n, work.shape[1], int(go_out))
    L[...] = work.astype(L.dtype)
    return L


def log_logistic(X, out=None):
    """log(1 / (1 + exp(-x))) computed stably (reference
    ``utils/extmath.py: log_logistic`` over ``_log_logistic_sigmoid``);
    numpy arrays or device tensors."""
    if isinstance(X, torch.Tensor):
        r = torch.nn.functional.logsigmoid(X)
        if out is not None:
            out.copy_(r)
            return out
        return r
    X = np.asarray(X, dtype=np.float64) if np.asarray(X).dtype.kind != "f" else np.asarray(X)
    is_1d = X.ndim == 1
    X = np.atleast_2d(X)
    res = np.where(X > 0, -np.log1p(np.exp(-np.abs(X))), X - np.log1p(np.exp(-np.abs(X))))
    if out is not None:
        out[...] = res.reshape(out.shape)
        res = out
    return np.squeeze(res) if is_1d else res
