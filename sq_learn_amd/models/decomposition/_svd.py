"""SVD back-ends for the PCA family over (possibly row-sharded) data.

* ``exact``: for small single-process data, ``torch.linalg.svd`` of the
  centred matrix in fp64 - bit-for-bit the reference's ``scipy.linalg.svd``
  semantics (``_qPCA.py:581``, ``_pca.py:437-502``).
* ``gram``: the MI355X path for tall matrices (n >> d): the d x d Gram
  (X-mu)^T (X-mu) by the fp64-MFMA kernel (one pass over X), one
  all-reduce, host ``eigh`` in fp64 -> S, V; left singular vectors
  U = (X-mu) V S^-1 are materialised only for the retained columns, on the
  shard that owns the rows.
* ``cholqr2`` (default for tall matrices): sharded CholeskyQR2 in fp64
  (two passes over X, two d x d all-reduces), then the SVD of the d x d R:
  singular values and right vectors to ~eps64 * cond relative, like the
  reference's fp64 LAPACK (the ``gram`` eigenvalues lose eps * cond^2);
  falls back to ``gram`` when cond(X) >~ 1e8 or X is rank deficient.
* ``randomized``: :func:`utils.extmath.randomized_svd_distributed`
  (fp64-MFMA power iterations and CholeskyQR2, K14, C6/C7).
"""

import numpy as np
import torch

from ...utils.extmath import svd_flip, svd_flip_distributed, randomized_svd_distributed
from ...ops import linalg as L


class SVDResult:
    def __init__(self, S, Vt, U_local=None, method="exact"):
        self.S = S              # numpy [r]
        self.Vt = Vt            # numpy [r, d]
        self.U_local = U_local  # tensor [n_loc, k] or None
        self.method = method


def _small(data):
    return data.comm.world_size == 1 and data.n_global * data.d <= 4e7 and \
        (data.device.type == "cpu" or data.n_global <= 200_000)


def full_svd(data, mean, k_left, method="auto"):
    """Thin SVD of (X - mean); U computed for the first ``k_left`` columns."""
    if method == "auto":
        method = "exact" if (_small(data) or data.n_global < data.d) else "cholqr2"
    X = data.X
    if method == "cholqr2":
        R = L.cholqr2_r(X, data.comm, mean)
        if R is None:
            method = "gram"
        else:
            _, S, Vt = torch.linalg.svd(R.cpu())       # d x d, host LAPACK fp64
            return _finish(data, mean, S, Vt, k_left, "cholqr2")
    if method == "exact":
        full = X if data.comm.world_size == 1 else torch.cat(data.comm.all_gather_varlen(X), 0)
        Xc = full.to(torch.float64) - mean.to(torch.float64).to(full.device)
        U, S, Vt = torch.linalg.svd(Xc, full_matrices=False)
        U, Vt = svd_flip(U, Vt)
        if data.comm.world_size > 1:
            U = U[data.row_offset:data.row_offset + data.n_local]
        return SVDResult(S.cpu().numpy(), Vt.cpu().numpy(), U[:, :k_left], "exact")
    # Gram path
    G = L.gram_local(X, mean)                      # fp64 (fp64-MFMA kernel on the GPU)
    data.comm.all_reduce_(G)
    G = G.cpu()
    G = 0.5 * (G + G.T)
    ev, V = torch.linalg.eigh(G)                   # d x d, host LAPACK fp64
    ev = ev.flip(0).clamp(min=0.0)
    V = V.flip(1)
    S = torch.sqrt(ev)
    Vt = V.T.contiguous()
    return _finish(data, mean, S, Vt, k_left, "gram")


def _finish(data, mean, S, Vt, k_left, method):
    """Left vectors U = (X - mean) V S^-1 for the retained columns on the
    row shard, deterministic signs."""
    X = data.X
    r = min(data.n_global, data.d)
    S, Vt = S[:r], Vt[:r]
    k = min(k_left, int((S > S[0] * 1e-12).sum()) if S.numel() else 0) if r else 0
    dt = torch.float64 if X.device.type == "cpu" else torch.float32
    Vk = Vt[:k].T.to(torch.float64).contiguous()
    Uk = torch.empty((data.n_local, k), dtype=dt, device=X.device)
    if k and data.n_local:
        # U = (X - mean) V_k in one fp64-accumulated pass (csrc/tsgemm64.hip xw)
        L.xw(X if X.stride(1) == 1 else X.contiguous(), Vk.to(X.device), mean=mean, out=Uk)
    if k:
        Uk /= S[:k].to(dt).to(X.device)
    # u-based signs for the retained columns, v-based for the rest
    Vt_dev = Vt.to(X.device)
    if k:
        Uk, Vk_t = svd_flip_distributed(Uk, Vt_dev[:k].to(dt), data.comm)
        Vt_dev = torch.cat([Vk_t.to(torch.float64), Vt_dev[k:]], 0)
    if Vt_dev.shape[0] > k:
        rest = Vt_dev[k:]
        idx = torch.argmax(rest.abs(), dim=1)
        sg = torch.sign(rest[torch.arange(rest.shape[0], device=rest.device), idx])
        sg = torch.where(sg == 0, torch.ones_like(sg), sg)
        Vt_dev = torch.cat([Vt_dev[:k], rest * sg[:, None]], 0)
    return SVDResult(S.cpu().numpy(), Vt_dev.to(torch.float64).cpu().numpy(), Uk, method)


def truncated_svd(data, mean, n_components, n_iter="auto", seed=0, n_oversamples=10):
    U, s, Vt = randomized_svd_distributed(data.X, mean, n_components, data.comm,
                                          n_oversamples=n_oversamples, n_iter=n_iter, seed=seed,
                                          n_rows=data.n_global, d=data.d)
    return SVDResult(s.cpu().numpy(), Vt.cpu().numpy(), U, "randomized")
