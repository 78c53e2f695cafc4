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


def gram64_native(X, mean=None):
    """G = (X - mean)^T (X - mean) in fp64 on the matrix cores
    (csrc/gram64.hip, v_mfma_f64_16x16x4_f64): per-workgroup partial upper
    blocks summed in a fixed order (deterministic); X fp32 or fp64, d <= 256."""
    n, d = X.shape
    assert X.dtype in (torch.float32, torch.float64, torch.bfloat16) and X.stride(1) == 1 and d <= 256
    code = {torch.float32: 0, torch.float64: 1, torch.bfloat16: 2}[X.dtype]
    if n == 0:   # an empty shard contributes an exact zero (the kernel writes nothing)
        return torch.zeros((d, d), dtype=torch.float64, device=X.device)
    nb = (d + 15) // 16
    nblk = nb * (nb + 1) // 2
    grid = int(max(1, min(256, (n + 255) // 256)))
    part = torch.empty((grid, nblk, 16, 16), dtype=torch.float64, device=X.device)
    mu = None if mean is None else mean.to(torch.float64).to(X.device).contiguous()
    rc = nat.native().gram64(X.data_ptr(), code, X.stride(0),
                             0 if mu is None else mu.data_ptr(), n, d, part.data_ptr(), grid,
                             nat.stream_handle(X.device))
    if rc:
        raise RuntimeError(f"gram64 failed (hip error {rc})")
    blocks = part.sum(0)                                   # [nblk, 16, 16], fixed order
    # scatter the upper blocks and their transposes in two indexed copies
    # (was one tiny copy per block: ~270 launches per call)
    iu = torch.triu_indices(nb, nb, device=X.device)
    G4 = torch.zeros((nb, nb, 16, 16), dtype=torch.float64, device=X.device)
    G4[iu[1], iu[0]] = blocks.transpose(1, 2)
    G4[iu[0], iu[1]] = blocks                              # diagonal blocks: the upper copy
    return G4.permute(0, 2, 1, 3).reshape(nb * 16, nb * 16)[:d, :d].contiguous()


def gram64_local(X, mean=None, W=None, chunk_rows=1 << 19):
    """Local partial of G = ((X - mean) W)^T ((X - mean) W) accumulated in
    fp64.  GPU: the fp64-MFMA kernel (:func:`gram64_native`) on X (pass 1)
    or on row chunks of (X - mean) W formed by library DGEMM (pass 2); CPU:
    torch fp64.  The building block of the fp64-faithful sharded
    CholeskyQR2 (:func:`cholqr2_r`)."""
    n, d = X.shape
    dw = d if W is None else W.shape[1]
    native = (nat.use_native(X) and X.dtype in (torch.float32, torch.float64, torch.bfloat16)
              and d <= 256 and dw <= 256 and X.stride(1) == 1)
    if native and W is None:
        return gram64_native(X, mean)
    G = torch.zeros((dw, dw), dtype=torch.float64, device=X.device)
    m = None if mean is None else mean.to(torch.float64).to(X.device)
    Wd = None if W is None else W.to(torch.float64).to(X.device)
    for s in range(0, n, chunk_rows):
        Xc = X[s:s + chunk_rows].to(torch.float64)
        if m is not None:
            Xc = Xc - m
        if Wd is not None:
            Xc = Xc @ Wd
        if native:
            G += gram64_native(Xc.contiguous())
        else:
            G.addmm_(Xc.T, Xc)
    return G


def cholqr2_r(X, comm, mean=None):
    """R factor of the thin QR of the row-sharded matrix X - mean by
    CholeskyQR2 in fp64 (two passes over X, one d x d all-reduce each):
    R1 = chol(X^T X), R2 = chol((X R1^-1)^T (X R1^-1)), R = R2 R1.  The
    singular values of R are those of X to ~eps64 * cond(X) relative (the
    Gram eigenvalues alone: eps * cond^2).  Returns None when the first
    Cholesky fails (cond(X) >~ 1e8 or rank deficient): callers fall back to
    the Gram eigenvalues."""
    G1 = comm.all_reduce_(gram64_local(X, mean))
    G1 = 0.5 * (G1 + G1.T)
    R1, info = torch.linalg.cholesky_ex(G1, upper=True)
    if int(info) != 0:
        return None
    eye = torch.eye(G1.shape[0], dtype=torch.float64, device=G1.device)
    W1 = torch.linalg.solve_triangular(R1, eye, upper=True)
    G2 = comm.all_reduce_(gram64_local(X, mean, W1))
    G2 = 0.5 * (G2 + G2.T)
    R2, info = torch.linalg.cholesky_ex(G2, upper=True)
    if int(info) != 0:
        return None
    return R2 @ R1


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
