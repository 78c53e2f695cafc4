"""Shared input handling for the estimators: numpy / tensor / ShardedArray
-> (local device tensor, global geometry, communicator), plus the global
(cross-rank) statistics every estimator needs."""

import numpy as np
import torch

from ..parallel.comm import Comm
from ..parallel.sharding import ShardedArray
from ..runtime.device import resolve_device
from ..utils.validation import check_array
from ..ops import linalg as L


class Data:
    """Local rows of a (possibly sharded) dataset on the compute device."""

    def __init__(self, local, n_global, row_offset, comm, source_kind):
        self.X = local
        self.n_global = int(n_global)
        self.row_offset = int(row_offset)
        self.comm = comm
        self.source_kind = source_kind   # 'numpy' | 'tensor' | 'sharded'

    @property
    def n_local(self):
        return self.X.shape[0]

    @property
    def d(self):
        return self.X.shape[1]

    @property
    def device(self):
        return self.X.device


def as_data(X, device=None, dtype=None, copy=False, comm=None):
    """Validate and place X.  ``dtype=None``: float64 on CPU, float32 on GPU
    (bf16 tensors are kept as given - they are the data)."""
    dev = resolve_device(device)
    if isinstance(X, ShardedArray):
        loc = X.local
        if loc.device != dev:
            loc = loc.to(dev)
        loc = _cast(loc, dev, dtype)
        check_array(loc, dtype=None, ensure_min_samples=0)
        return Data(loc.contiguous(), X.n_global, X.row_offset, X.comm, "sharded")
    comm = comm if comm is not None else Comm(None)
    if isinstance(X, torch.Tensor):
        t = check_array(X, dtype=None)
        if not t.is_floating_point():
            t = t.double()
        t = t.to(dev) if t.device != dev else (t.clone() if copy else t)
        t = _cast(t, dev, dtype)
        return Data(t.contiguous(), t.shape[0], 0, comm, "tensor")
    arr = check_array(X, dtype=[np.float64, np.float32])
    t = torch.as_tensor(np.ascontiguousarray(arr))
    t = _cast(t, dev, dtype)
    t = t.to(dev)
    return Data(t.contiguous(), t.shape[0], 0, comm, "numpy")


def _cast(t, dev, dtype):
    if dtype is not None:
        return t.to(dtype)
    if t.dtype == torch.bfloat16:
        return t
    if dev.type == "cuda" and t.dtype == torch.float64:
        return t.to(torch.float32)
    if not t.is_floating_point():
        return t.to(torch.float64 if dev.type == "cpu" else torch.float32)
    return t


def global_sum(data: Data, t):
    data.comm.all_reduce_(t)
    return t


def global_mean_var(data: Data):
    """Column mean and (population) variance over all ranks in one collective."""
    X = data.X
    s, ss = L.col_moments_local(X)
    buf = torch.cat([s, ss])
    data.comm.all_reduce_(buf)
    d = X.shape[1]
    mean = buf[:d] / data.n_global
    var = (buf[d:] / data.n_global - mean ** 2).clamp(min=0.0)
    return mean, var


def gather_rows(data: Data, global_idx):
    """Rows with the given global indices, replicated on every rank (one
    all-reduce: owners contribute their rows, others zeros)."""
    idx = torch.as_tensor(np.asarray(global_idx, dtype=np.int64), device=data.device)
    out = torch.zeros((idx.numel(), data.d), dtype=torch.float64 if data.device.type == "cpu"
                      else torch.float32, device=data.device)
    lo, hi = data.row_offset, data.row_offset + data.n_local
    mine = (idx >= lo) & (idx < hi)
    if bool(mine.any()):
        out[mine] = data.X[idx[mine] - lo].to(out.dtype)
    data.comm.all_reduce_(out)
    return out


def prelude_stats(data: Data, mu_start=0.0, mu_end=1.0, mu_step=0.1, condition=True):
    """eta = max ||x||^2, mu(A) p-grid search and 1/sigma_min on the raw data
    (reference ``_dmeans.py:1242-1245``, ``_qPCA.py:634-636``), all ranks."""
    X = data.X
    rn = L.row_norms_sq(X).double()
    eta = torch.tensor([float(rn.max()) if rn.numel() else 0.0], dtype=torch.float64, device=X.device)
    data.comm.all_reduce_(eta, op="max")
    eta = float(eta.item())
    label, mu = best_mu_distributed(data, mu_start, mu_end, mu_step, fro_sq=float(rn.sum()))
    cond = None
    if condition:
        smin = sigma_min(data)
        cond = float("inf") if smin == 0 else 1.0 / smin
    return eta, label, mu, cond


def best_mu_distributed(data: Data, start=0.0, end=1.0, step=0.05, fro_sq=None, fro_sq_global=None,
                        mean=None):
    """``best_mu`` (``Utility.py:196-231``) over a row-sharded matrix: one
    fused power-sum pass (row-max and column sums for every exponent of the
    p-grid), then MAX / SUM all-reduces.  ``mean``: mu of the centred matrix
    X - mean, subtracted inside the pass."""
    domain = [i for i in np.arange(start, end, step)] + [end]
    exps = sorted(set([round(float(2 * p), 12) for p in domain] +
                      [round(float(2 * (1 - p)), 12) for p in domain]))
    rowmax, colsum = L.mu_power_sums_local(data.X, exps, mean=mean)
    data.comm.all_reduce_(rowmax, op="max")
    data.comm.all_reduce_(colsum, op="sum")
    colmax = colsum.max(dim=1).values
    pos = {e: i for i, e in enumerate(exps)}
    vals = []
    for p in domain:
        s1 = float(rowmax[pos[round(float(2 * p), 12)]])
        s2 = float(colmax[pos[round(float(2 * (1 - p)), 12)]])
        vals.append(float(np.sqrt(s1 * s2)))
    best = int(np.argmin(vals))
    if fro_sq_global is not None:
        fro = float(np.sqrt(fro_sq_global))
    else:
        if fro_sq is None:
            Xd = data.X.double() if mean is None else data.X.double() - mean.double().to(data.device)
            fro_sq = float((Xd ** 2).sum())
        t = torch.tensor([fro_sq], dtype=torch.float64, device=data.device)
        data.comm.all_reduce_(t)
        fro = float(np.sqrt(t.item()))
    if vals[best] <= fro:
        return f"p={domain[best]}", vals[best]
    return "Frobenius", fro


def sigma_min(data: Data, mean=None):
    """Smallest singular value of the (optionally centred) global matrix.

    The reference takes it from an fp64 LAPACK SVD of X
    (``_dmeans.py:1244-1245``).  Here: sharded CholeskyQR2 in fp64
    (:func:`ops.linalg.cholqr2_r`, two passes over X, two d x d
    all-reduces) and the singular values of the d x d R - accurate to
    ~eps64 * cond(X) relative.  Rank-deficient / cond >~ 1e8 matrices fall
    back to the square roots of the fp64 Gram eigenvalues."""
    n, d = data.n_global, data.d
    if n < d:
        full = gather_full(data).double()
        if mean is not None:
            full = full - mean.double().to(full.device)
        s = torch.linalg.svdvals(full)
        return float(s.min()) if s.numel() else 0.0
    R = L.cholqr2_r(data.X, data.comm, mean)
    if R is not None:
        return float(torch.linalg.svdvals(R.cpu()).min())      # d x d, host LAPACK
    G = data.comm.all_reduce_(L.gram64_local(data.X, mean)).cpu()
    ev = torch.linalg.eigvalsh(0.5 * (G + G.T))
    return float(torch.sqrt(ev.clamp(min=0.0)).min())


def gather_full(data: Data):
    if data.comm.world_size == 1:
        return data.X
    return torch.cat(data.comm.all_gather_varlen(data.X), 0)


def check_n_features(est, data):
    """Raise like the reference's ``_check_n_features(reset=False)``."""
    n_in = getattr(est, "n_features_in_", None)
    if n_in is not None and data.d != n_in:
        raise ValueError(f"X has {data.d} features, but {type(est).__name__} is expecting "
                         f"{n_in} features as input.")
    return data
