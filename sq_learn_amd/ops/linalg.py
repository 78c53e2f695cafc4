"""Row-sharded linear algebra ops: row norms, the fp64 tall-skinny GEMMs
(A - mu_a)^T (B - mu_b) and (A - mu) W (Gram, CholeskyQR2, power iteration,
randomized range finder) and the mu(A) power sums.

GPU tensors use the MFMA kernels of ``csrc/tsgemm64.hip`` (fp64) and
``csrc/linalg.hip`` (row norms, mu sums); CPU tensors use torch.  All
functions return *local* (per-shard) partial results; callers reduce them
across ranks with one collective.
"""

import os

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


# ------------------------------------------------ fp64-MFMA tall-skinny GEMMs
_XTX_TARGET_WGS = 1024        # 2-3 resident workgroups per CU (LDS-bound), 256 CUs
_XTX_MAX_SPLITS = 512
# fp64 row-chunk buffers of the two-kernel passes (X W into a chunk, then the
# chunk's Gram): 128 MiB chunks stay in the 256 MB Infinity Cache between the
# producing and the consuming kernel instead of a round trip through HBM
_CHUNK_BYTES = int(os.environ.get("SQ_CHUNK_MB", "128")) << 20


def _part(device, numel):
    """fp64 workspace for the xtx split partials, from torch's caching
    allocator on the current stream (reused block, no allocation cost after
    the first call; stream-ordered, so concurrent calls on different streams
    never share partials)."""
    return torch.empty(max(numel, 1), dtype=torch.float64, device=device)


def _mean64(m, device):
    return None if m is None else m.to(device=device, dtype=torch.float64).contiguous()


def xtx(A, B=None, mean_a=None, mean_b=None, out=None, accumulate=False):
    """C = (A - mean_a)^T (B - mean_b) in fp64 (``B=None``: the symmetric Gram
    of A).  GPU: csrc/tsgemm64.hip (fp64 MFMA, split-K over row ranges,
    fixed-order partial sums: deterministic; any feature count, fp32 / bf16 /
    fp64 inputs with row stride).  ``out`` (+= when ``accumulate``) lets
    chunked callers sum several row blocks.  Returns the LOCAL partial."""
    sym = B is None
    n, da = A.shape
    db = da if sym else B.shape[1]
    if not sym:
        assert B.shape[0] == n
    dev = A.device
    if out is None:
        out = torch.zeros((da, db), dtype=torch.float64, device=dev)
        accumulate = False
    if not nat.use_native(A):
        Ac = A.to(torch.float64)
        if mean_a is not None:
            Ac = Ac - mean_a.to(torch.float64)
        if sym:
            Bc = Ac
        else:
            Bc = B.to(torch.float64)
            if mean_b is not None:
                Bc = Bc - mean_b.to(torch.float64)
        r = Ac.T @ Bc
        if accumulate:
            out += r
        else:
            out.copy_(r)
        return out
    assert A.stride(1) == 1 and (sym or B.stride(1) == 1)
    TM, TN, npairs = nat.native().xtx_geometry(da, db, int(sym))
    splits = max(8, min(-(-_XTX_TARGET_WGS // npairs), -(-max(n, 1) // 256), _XTX_MAX_SPLITS))
    splits = -(-splits // 8) * 8
    part = _part(dev, splits * npairs * TM * TN)
    ma, mb = _mean64(mean_a, dev), (None if sym else _mean64(mean_b, dev))
    Bt = A if sym else B
    rc = nat.native().xtx(A.data_ptr(), nat.dtype_code(A), A.stride(0), nat.ptr(ma), da,
                          Bt.data_ptr(), nat.dtype_code(Bt), Bt.stride(0), nat.ptr(mb), db, n,
                          int(sym), splits, part.data_ptr(), out.data_ptr(), int(accumulate),
                          nat.stream_handle(dev))
    if rc:
        raise RuntimeError(f"xtx failed (hip error {rc})")
    return out


def xw(A, W, mean=None, upper=False, out_dtype=torch.float64, out=None):
    """Y = (A - mean) W, W (d x l) applied in fp64 (csrc/tsgemm64.hip on the
    GPU; ``upper``: W is upper triangular and its zero block is skipped)."""
    n, d = A.shape
    l = W.shape[1]
    dev = A.device
    if out is None:
        out = torch.empty((n, l), dtype=out_dtype, device=dev)
    if not nat.use_native(A):
        Ac = A.to(torch.float64)
        if mean is not None:
            Ac = Ac - mean.to(torch.float64)
        out.copy_(Ac @ W.to(torch.float64))
        return out
    assert A.stride(1) == 1 and out.stride(1) == 1 and out.dtype in (torch.float32, torch.float64)
    Wd = W.to(device=dev, dtype=torch.float64).contiguous()
    m = _mean64(mean, dev)
    rc = nat.native().xw(A.data_ptr(), nat.dtype_code(A), A.stride(0), nat.ptr(m), n, d,
                         Wd.data_ptr(), Wd.stride(0), l, int(bool(upper)), out.data_ptr(),
                         1 if out.dtype == torch.float64 else 0, out.stride(0),
                         nat.stream_handle(dev))
    if rc:
        raise RuntimeError(f"xw failed (hip error {rc})")
    return out


def gram_local(X, mean):
    """Local partial of G = (X - mean)^T (X - mean) in fp64 (:func:`xtx`)."""
    return xtx(X, mean_a=mean)


def _chunk(cols, chunk_rows):
    return chunk_rows if chunk_rows else max(1 << 16, _CHUNK_BYTES // (8 * max(cols, 1)))


def gram64_local(X, mean=None, W=None, chunk_rows=None):
    """Local partial of G = ((X - mean) W)^T ((X - mean) W) accumulated in
    fp64: pass 1 of CholeskyQR2 (W = None) is one :func:`xtx` over X; pass 2
    forms Y = (X - mean) W1 (W1 = R1^-1 upper triangular) chunk by chunk with
    :func:`xw` into an fp64 buffer and accumulates Y^T Y (no library GEMM, no
    fp64 copy of X)."""
    n, d = X.shape
    if W is None:
        return xtx(X, mean_a=mean)
    dw = W.shape[1]
    chunk_rows = _chunk(dw, chunk_rows)
    G = torch.zeros((dw, dw), dtype=torch.float64, device=X.device)
    if n == 0:
        return G
    if X.stride(1) != 1:
        X = X.contiguous()
    buf = torch.empty((min(n, chunk_rows), dw), dtype=torch.float64, device=X.device)
    for s in range(0, n, chunk_rows):
        e = min(n, s + chunk_rows)
        Y = xw(X[s:e], W, mean=mean, upper=True, out=buf[:e - s])
        xtx(Y, out=G, accumulate=True)
    return G


def gram64_native(X, mean=None):
    """G = (X - mean)^T (X - mean) in fp64 on the matrix cores (any d)."""
    return xtx(X, mean_a=mean)


def cholqr2_r(X, comm, mean=None):
    """R factor of the thin QR of the row-sharded matrix X - mean by
    CholeskyQR2 in fp64 (two passes over X, one d x d all-reduce each; the
    second pass only when cond(R1) > 100):
    R1 = chol(X^T X), R2 = chol((X R1^-1)^T (X R1^-1)), R = R2 R1.  The
    singular values of R are those of X to ~eps64 * cond(X) relative (the
    Gram eigenvalues alone: eps * cond^2).  Returns None when the first
    Cholesky fails (cond(X) >~ 1e8 or rank deficient): callers fall back to
    the Gram eigenvalues.  The d x d factorisations run on the host (LAPACK
    fp64)."""
    G1 = comm.all_reduce_(gram64_local(X, mean)).cpu()
    G1 = 0.5 * (G1 + G1.T)
    R1, info = torch.linalg.cholesky_ex(G1, upper=True)
    if int(info) != 0:
        return None
    # well-conditioned X (cond(R1) <= 100, estimated from the d x d R1 on the
    # host): the singular values of R1 are already accurate to
    # ~eps64 * cond^2 <= 2e-12 relative - the second pass over X (which
    # brings that to eps64 * cond) is skipped
    sv = torch.linalg.svdvals(R1)
    if sv.numel() and float(sv[-1]) > 0.0 and float(sv[0]) <= 100.0 * float(sv[-1]):
        return R1.to(X.device)
    eye = torch.eye(G1.shape[0], dtype=torch.float64)
    W1 = torch.linalg.solve_triangular(R1, eye, upper=True)
    G2 = comm.all_reduce_(gram64_local(X, mean, W1.to(X.device))).cpu()
    G2 = 0.5 * (G2 + G2.T)
    R2, info = torch.linalg.cholesky_ex(G2, upper=True)
    if int(info) != 0:
        return None
    return (R2 @ R1).to(X.device)


def power_iter_local(X, Q, mean, chunk_rows=None):
    """Local partial of Z = (X - mean)^T ((X - mean) Q) in fp64: per row
    chunk Y = (X - mean) Q by :func:`xw` (fp64, stays in a reused buffer),
    then Z += (X - mean)^T Y by :func:`xtx`."""
    n, d = X.shape
    l = Q.shape[1]
    chunk_rows = _chunk(l, chunk_rows)
    Z = torch.zeros((d, l), dtype=torch.float64, device=X.device)
    if n == 0:
        return Z
    if not nat.use_native(X):
        Qd = Q.to(torch.float64)
        md = mean.to(torch.float64)
        for s in range(0, n, chunk_rows):
            Xc = X[s:s + chunk_rows].to(torch.float64) - md
            Z += Xc.T @ (Xc @ Qd)
        return Z
    if X.stride(1) != 1:
        X = X.contiguous()
    buf = torch.empty((min(n, chunk_rows), l), dtype=torch.float64, device=X.device)
    for s in range(0, n, chunk_rows):
        e = min(n, s + chunk_rows)
        Y = xw(X[s:e], Q, mean=mean, out=buf[:e - s])
        xtx(X[s:e], Y, mean_a=mean, out=Z, accumulate=True)
    return Z


def col_moments_local(X):
    """(sum over rows, sum of squares over rows) of every column, fp64 [d]
    each - one pass over X on the GPU (csrc/linalg.hip col_moments, fixed
    row partition, fixed-order partial sums: deterministic); no fp64 copy
    of X."""
    n, d = X.shape
    if nat.use_native(X) and X.dtype in (torch.float32, torch.bfloat16) and n > 0:
        # the launcher's own partition (sq_col_moments): every one of its
        # wgs blocks writes its row of partials, so no zero-fill and no rows
        # beyond the ones used (2048 x 2d was ~2 GiB at d = 65k)
        wgs = min(2048, max(1, -(-n // 256)))
        rpw = -(-n // wgs)
        wgs = -(-n // rpw)
        part = torch.empty((wgs, 2 * d), dtype=torch.float64, device=X.device)
        rc = nat.native().col_moments(X.data_ptr(), nat.dtype_code(X), X.stride(0), n, d,
                                      part.data_ptr(), wgs, nat.stream_handle(X.device))
        if rc:
            raise RuntimeError(f"col_moments failed (hip error {rc})")
        tot = part.sum(0)
        return tot[:d], tot[d:]
    Xd = X.to(torch.float64)
    return Xd.sum(0), (Xd * Xd).sum(0)


def mu_power_sums_local(X, exponents, mean=None):
    """(row_max [nq], col_sums [nq, d]) local partials for mu(A).

    row_max[i] = max_rows sum_j |a_rj|^q_i   (q=0: nonzero count)
    col_sums[i, j] = sum_rows |a_rj|^q_i
    with a = x - mean (``mean`` [d], optional: fused into the pass, no
    centred copy of X).
    """
    n, d = X.shape
    q = torch.tensor(exponents, dtype=torch.float32)
    nq = len(exponents)
    if nat.use_native(X) and X.dtype in (torch.float32, torch.bfloat16) and nq <= 12:
        if X.stride(1) != 1:
            X = X.contiguous()
        qd = q.to(X.device)
        rowmax = torch.zeros(nq, dtype=torch.float32, device=X.device)
        colsum = torch.zeros((nq, d), dtype=torch.float32, device=X.device)
        wgs = 1024   # per-WG partials, summed in a fixed order (deterministic)
        part = torch.empty((wgs, nq, d), dtype=torch.float32, device=X.device)
        # d > 512: row power sums carried across the 512-column blocks
        racc = torch.zeros((nq, n), dtype=torch.float32, device=X.device) if d > 512 else None
        mu = None if mean is None else mean.to(device=X.device, dtype=torch.float32).contiguous()
        # an arithmetic grid 0, b, 2b, ... (the p-grid's 2p): one exp2 per element,
        # the other powers by products
        qstep = 0.0
        if nq >= 2 and exponents[0] == 0.0 and exponents[1] > 0.0:
            b = float(exponents[1])
            if all(abs(float(e) - i * b) <= 1e-9 * max(1.0, i * b) for i, e in enumerate(exponents)):
                qstep = b
        rc = nat.native().mu_sums(X.data_ptr(), nat.dtype_code(X), X.stride(0), qd.data_ptr(), nq,
                                  rowmax.data_ptr(), colsum.data_ptr(), part.data_ptr(), wgs,
                                  nat.ptr(racc), n, d, nat.ptr(mu), qstep,
                                  nat.stream_handle(X.device))
        if rc:
            raise RuntimeError(f"mu_sums failed (hip error {rc})")
        return rowmax.double(), colsum.double()
    A = X.to(torch.float64)
    if mean is not None:
        A = A - mean.to(device=X.device, dtype=torch.float64)
    A = A.abs()
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
