"""Row-sharded linear algebra ops: row norms, Gram (X-mu)^T(X-mu), fused
power iteration (X-mu)^T((X-mu) Q) and the mu(A) power sums.

GPU tensors use the MFMA kernels of ``csrc/linalg.hip``; CPU tensors use
torch.  All functions return *local* (per-shard) partial results; callers
reduce them across ranks with one collective.
"""

import torch

from . import _native as nat

# exponents of the mu(A) p-grid: s_{2p} (rows) and s_{2(1-p)} (columns) for
# p in {0, 0.1, ..., 1.0} need |a|^q for q in {0, 0.2, ..., 2.0}
MU_EXPONENTS_STEP01 = [round(0.2 * i, 10) for i in range(11)]


def row_norms_sq(X, out=None):
    """||x_i||^2 (fp32 on GPU, X dtype on CPU). Reference ``utils/extmath.py:49``."""
    if nat.use_native(X) and X.dtype in (torch.float32, torch.bfloat16):
        X = X.contiguous()
        out = torch.empty(X.shape[0], dtype=torch.float32, device=X.device) if out is None else out
        nat.native().row_norms(X.data_ptr(), nat.dtype_code(X), out.data_ptr(), X.shape[0],
                               X.shape[1], nat.stream_handle(X.device))
        return out
    Xf = X if X.dtype in (torch.float32, torch.float64) else X.float()
    r = (Xf * Xf).sum(1)
    if out is not None:
        out.copy_(r)
        return out
    return r


def gram_local(X, mean):
    """Local partial of G = (X - mean)^T (X - mean) (fp32 on GPU, f64 on CPU)."""
    n, d = X.shape
    if nat.use_native(X) and X.dtype in (torch.float32, torch.bfloat16):
        X = X.contiguous()
        G = torch.zeros((d, d), dtype=torch.float32, device=X.device)
        m = mean.to(torch.float32).contiguous()
        # per-split partial tiles, reduced in a fixed order (deterministic)
        side = (d + 63) // 64
        cap = max(1, 2048 // (side * (side + 1) // 2)) * (side * (side + 1) // 2) * 64 * 64
        part = torch.empty(cap, dtype=torch.float32, device=X.device)
        nat.native().gram(X.data_ptr(), nat.dtype_code(X), G.data_ptr(), m.data_ptr(), n, d,
                          part.data_ptr(), cap, nat.stream_handle(X.device))
        # kernel fills the upper triangle tiles; mirror
        iu = torch.triu_indices(d, d, 1, device=X.device)
        G[iu[1], iu[0]] = G[iu[0], iu[1]]
        return G
    Xc = X.to(torch.float64) - mean.to(torch.float64)
    return Xc.T @ Xc


def power_iter_local(X, Q, mean):
    """Local partial of Z = (X - mean)^T ((X - mean) Q)  (one pass over X)."""
    n, d = X.shape
    l = Q.shape[1]
    if nat.use_native(X) and X.dtype in (torch.float32, torch.bfloat16) and d <= 256 and l <= 64:
        X = X.contiguous()
        Z = torch.zeros((d, l), dtype=torch.float32, device=X.device)
        Qc = Q.to(torch.float32).contiguous()
        m = mean.to(torch.float32).contiguous()
        wgs = 256   # per-WG partials summed in a fixed order (deterministic)
        part = torch.empty((wgs, d, l), dtype=torch.float32, device=X.device)
        nat.native().power_iter(X.data_ptr(), nat.dtype_code(X), Qc.data_ptr(), Z.data_ptr(),
                                m.data_ptr(), n, d, l, part.data_ptr(), wgs,
                                nat.stream_handle(X.device))
        return Z
    acc = torch.float64 if X.device.type == "cpu" else torch.float32
    Z = torch.zeros((d, l), dtype=acc, device=X.device)
    Qa = Q.to(acc)
    ma = mean.to(acc)
    step = 1 << 20
    for s in range(0, n, step):
        Xc = X[s:s + step].to(acc) - ma
        Z += Xc.T @ (Xc @ Qa)
    return Z


def mu_power_sums_local(X, exponents):
    """(row_max [nq], col_sums [nq, d]) local partials for mu(A).

    row_max[i] = max_rows sum_j |x_rj|^q_i   (q=0: nonzero count)
    col_sums[i, j] = sum_rows |x_rj|^q_i
    """
    n, d = X.shape
    q = torch.tensor(exponents, dtype=torch.float32)
    nq = len(exponents)
    if nat.use_native(X) and X.dtype in (torch.float32, torch.bfloat16) and d <= 256 and nq <= 12:
        X = X.contiguous()
        qd = q.to(X.device)
        rowmax = torch.zeros(nq, dtype=torch.float32, device=X.device)
        colsum = torch.zeros((nq, d), dtype=torch.float32, device=X.device)
        wgs = 1024   # per-WG partials, summed in a fixed order (deterministic)
        part = torch.empty((wgs, nq, d), dtype=torch.float32, device=X.device)
        nat.native().mu_sums(X.data_ptr(), nat.dtype_code(X), qd.data_ptr(), nq, rowmax.data_ptr(),
                             colsum.data_ptr(), part.data_ptr(), wgs, n, d,
                             nat.stream_handle(X.device))
        return rowmax.double(), colsum.double()
    A = X.abs().to(torch.float64)
    rowmax = torch.zeros(nq, dtype=torch.float64, device=X.device)
    colsum = torch.zeros((nq, d), dtype=torch.float64, device=X.device)
    nz = A != 0
    logA = torch.log(torch.where(nz, A, torch.ones_like(A)))
    for i, qq in enumerate(exponents):
        if qq == 0:
            P = nz.to(torch.float64)
        else:
            P = torch.where(nz, torch.exp(qq * logA), torch.zeros_like(A))
        if n:
            rowmax[i] = P.sum(1).max()
        colsum[i] = P.sum(0)
    return rowmax, colsum
