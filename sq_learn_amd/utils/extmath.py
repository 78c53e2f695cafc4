"""Extended math (reference ``sklearn/utils/extmath.py``): ``row_norms`` (:49),
``squared_norm`` (:26), ``safe_sparse_dot`` (:119), ``randomized_range_finder``
(:161), ``randomized_svd`` (:246), ``svd_flip`` (:522), ``stable_cumsum``
(:829), ``fast_logdet`` (:81); plus the PPCA dimension MLE of
``decomposition/_pca.py`` (``_assess_dimension`` / ``_infer_dimension``).

``randomized_svd_distributed`` is the MI355X version of the randomized range
finder over a row-sharded matrix: the Gaussian test matrix is replicated
(Philox, same on every rank), each power iteration is ONE fused pass over
the local rows (``(X-mu)^T ((X-mu) Q)``, csrc/linalg.hip) plus ONE d x l
all-reduce, and the final orthonormalisation is CholeskyQR2 (two l x l
all-reduces) instead of a tall-skinny LU/QR.  Normalising the d x l iterate
every step spans the same subspace as sklearn's LU-normalised n x l iterate.
"""

import math
import warnings

import numpy as np
import torch
from scipy import linalg
from scipy.special import gammaln

from .validation import check_random_state


def squared_norm(x):
    x = np.ravel(x, order="K")
    return float(np.dot(x, x))


def row_norms(X, squared=False):
    if isinstance(X, torch.Tensor):
        Xf = X if X.dtype in (torch.float32, torch.float64) else X.float()
        r = (Xf * Xf).sum(1)
        return r if squared else torch.sqrt(r)
    X = np.asarray(X)
    norms = np.einsum("ij,ij->i", X, X)
    return norms if squared else np.sqrt(norms)


def safe_sparse_dot(a, b, *, dense_output=False):
    out = a @ b
    if dense_output and hasattr(out, "toarray"):
        return out.toarray()
    return out


def fast_logdet(A):
    sign, ld = np.linalg.slogdet(A)
    return ld if sign > 0 else -np.inf


def stable_cumsum(arr, axis=None, rtol=1e-05, atol=1e-08):
    out = np.cumsum(arr, axis=axis, dtype=np.float64)
    expected = np.sum(arr, axis=axis, dtype=np.float64)
    if not np.all(np.isclose(out.take(-1, axis=axis), expected, rtol=rtol, atol=atol, equal_nan=True)):
        warnings.warn("cumsum was found to be unstable: its last element does not correspond to sum",
                      RuntimeWarning)
    return out


def svd_flip(u, v, u_based_decision=True):
    """Deterministic signs (numpy or torch)."""
    if isinstance(u, torch.Tensor):
        if u_based_decision:
            idx = torch.argmax(u.abs(), dim=0)
            signs = torch.sign(u[idx, torch.arange(u.shape[1], device=u.device)])
        else:
            idx = torch.argmax(v.abs(), dim=1)
            signs = torch.sign(v[torch.arange(v.shape[0], device=v.device), idx])
        signs = torch.where(signs == 0, torch.ones_like(signs), signs)
        return u * signs, v * signs[:, None]
    if u_based_decision:
        max_abs_cols = np.argmax(np.abs(u), axis=0)
        signs = np.sign(u[max_abs_cols, range(u.shape[1])])
    else:
        max_abs_rows = np.argmax(np.abs(v), axis=1)
        signs = np.sign(v[range(v.shape[0]), max_abs_rows])
    signs[signs == 0] = 1
    return u * signs, v * signs[:, np.newaxis]


def svd_flip_distributed(U_local, Vt, comm):
    """u-based svd_flip where U's rows are sharded: the sign of column j is
    that of its global max-|.| entry (one gather of 2*r values per rank)."""
    r = U_local.shape[1]
    if U_local.shape[0]:
        a = U_local.abs()
        idx = torch.argmax(a, dim=0)
        val = U_local[idx, torch.arange(r, device=U_local.device)]
        mx = a[idx, torch.arange(r, device=U_local.device)]
    else:
        val = torch.zeros(r, dtype=U_local.dtype, device=U_local.device)
        mx = torch.full((r,), -1.0, dtype=U_local.dtype, device=U_local.device)
    both = torch.stack([mx.double(), val.double()])
    got = comm.all_gather(both)
    allmx = torch.stack([g[0] for g in got])   # [world, r]
    allv = torch.stack([g[1] for g in got])
    w = torch.argmax(allmx, dim=0)
    signs = torch.sign(allv[w, torch.arange(r, device=allv.device)])
    signs = torch.where(signs == 0, torch.ones_like(signs), signs)
    s = signs.to(U_local.dtype)
    return U_local * s, Vt * s.to(Vt.dtype)[:, None]


# --------------------------------------------------------------- numpy path
def randomized_range_finder(A, *, size, n_iter, power_iteration_normalizer="auto",
                            random_state=None):
    random_state = check_random_state(random_state)
    Q = random_state.normal(size=(A.shape[1], size))
    if hasattr(A, "dtype") and A.dtype.kind == "f":
        Q = Q.astype(A.dtype, copy=False)
    if power_iteration_normalizer == "auto":
        power_iteration_normalizer = "none" if n_iter <= 2 else "LU"
    for _ in range(n_iter):
        if power_iteration_normalizer == "none":
            Q = A @ Q
            Q = A.T @ Q
        elif power_iteration_normalizer == "LU":
            Q, _ = linalg.lu(A @ Q, permute_l=True)
            Q, _ = linalg.lu(A.T @ Q, permute_l=True)
        elif power_iteration_normalizer == "QR":
            Q, _ = linalg.qr(A @ Q, mode="economic")
            Q, _ = linalg.qr(A.T @ Q, mode="economic")
    Q, _ = linalg.qr(A @ Q, mode="economic")
    return Q


def randomized_svd(M, n_components, *, n_oversamples=10, n_iter="auto",
                   power_iteration_normalizer="auto", transpose="auto", flip_sign=True,
                   random_state=0):
    random_state = check_random_state(random_state)
    n_random = n_components + n_oversamples
    n_samples, n_features = M.shape
    if n_iter == "auto":
        n_iter = 7 if n_components < 0.1 * min(M.shape) else 4
    if transpose == "auto":
        transpose = n_samples < n_features
    if transpose:
        M = M.T
    Q = randomized_range_finder(M, size=n_random, n_iter=n_iter,
                                power_iteration_normalizer=power_iteration_normalizer,
                                random_state=random_state)
    B = Q.T @ M
    Uhat, s, Vt = linalg.svd(B, full_matrices=False)
    U = Q @ Uhat
    if flip_sign:
        if not transpose:
            U, Vt = svd_flip(U, Vt)
        else:
            U, Vt = svd_flip(U, Vt, u_based_decision=False)
    if transpose:
        return Vt[:n_components, :].T, s[:n_components], U[:, :n_components].T
    return U[:, :n_components], s[:n_components], Vt[:n_components, :]


# ------------------------------------------------------- distributed path
def _rsvd_gram(X_local, mean, G, Z, k, n_iter, dev):
    """The range finder run in the feature domain on the d x d Gram
    G = (X-mu)^T (X-mu) (all-reduced, on the host): Z <- qr(G Z) n_iter
    times is the same subspace iteration as the streamed
    qr((X-mu)^T ((X-mu) Z)).  The range basis Q = (X-mu) Z E lam^-1/2
    (M = Z^T G Z = E lam E^T, the Gram of (X-mu) Z) is never formed:
    B = Q^T (X-mu) = lam^-1/2 E^T Z^T G, and U = Q Uhat is ONE xw pass over
    X with the d x k matrix Z E lam^-1/2 Uhat.  Directions of (X-mu) Z with
    lam < 1e-6 lam_max (sigma ratio 1e-3, where Q's orthogonality error
    ~eps64 lam_max / lam would pass 1e-10) are dropped; None when the
    k-th one is among them (the caller streams instead)."""
    from ..ops import linalg as L
    for _ in range(n_iter):
        Z, _ = torch.linalg.qr(G @ Z)
    M = Z.T @ G @ Z
    lam, E = torch.linalg.eigh(0.5 * (M + M.T))
    lam, E = lam.flip(0), E.flip(1)
    lmax = float(lam[0]) if lam.numel() else 0.0
    if not lmax > 0.0 or not float(lam[k - 1]) >= 1e-6 * lmax:
        return None
    m = int((lam >= 1e-6 * lmax).sum())
    T = Z @ (E[:, :m] / torch.sqrt(lam[:m]))          # Q = (X - mu) T
    Uhat, sv, Vt = torch.linalg.svd(T.T @ G, full_matrices=False)
    U = L.xw(X_local, (T @ Uhat[:, :k]).contiguous().to(dev), mean=mean)
    return U, sv, Vt


def randomized_svd_distributed(X_local, mean, n_components, comm, *, n_oversamples=10,
                               n_iter="auto", seed=0, flip_sign=True, n_rows=None, d=None,
                               method="auto"):
    """Randomized SVD of the centred row-sharded matrix (X - mean)
    (``utils/extmath.py:161-242`` of the reference, Halko et al.).

    Every pass over the n rows is an fp64-MFMA tall-skinny kernel
    (ops/linalg.py xw / xtx -> csrc/tsgemm64.hip on the GPU).
    ``method="gram"`` (auto for d <= max(512, 4 l (n_iter + 2)), the
    flop crossover with margin): one xtx pass forms the d x d Gram, the
    power iterations and B run on it (:func:`_rsvd_gram`), one xw pass
    forms U - two reads of X instead of 2 n_iter + 4.  ``"stream"``: power
    iterations Z <- qr((X-mu)^T ((X-mu) Z)), Y = (X-mu) Z, two CholeskyQR
    passes Y <- Y R^-1, B^T = (X-mu)^T Y, U = Y Uhat.  The small d x l / l x l
    factorisations (QR, Cholesky, SVD) run on the host in fp64 LAPACK; one
    all-reduce per pass.  Returns (U_local [n_loc, k] fp64, s [k], Vt [k, d])."""
    from ..ops import linalg as L
    from ..ops.random import philox_normal
    from ..runtime.rng import RngKey
    n_loc, dd = X_local.shape
    d = dd if d is None else d
    k = int(n_components)
    l = min(k + n_oversamples, d)
    n_glob = n_rows if n_rows is not None else n_loc
    if n_iter == "auto":
        n_iter = 7 if k < 0.1 * min(n_glob, d) else 4
    dev = X_local.device
    if X_local.stride(1) != 1:
        X_local = X_local.contiguous()
    Z = philox_normal((d, l), RngKey(seed, "gaussian", 0), dtype=torch.float64, device="cpu")
    if method == "auto":
        method = "gram" if d <= 4096 and d <= max(512, 4 * l * (n_iter + 2)) else "stream"
    if method == "gram":
        G = comm.all_reduce_(L.xtx(X_local, mean_a=mean)).cpu()
        got = _rsvd_gram(X_local, mean, 0.5 * (G + G.T), Z, k, n_iter, dev)
        if got is not None:
            U, sv, Vt = got
            Vt = Vt[:k].to(dev)
            if flip_sign:
                U, Vt = svd_flip_distributed(U, Vt, comm)
            return U, sv[:k].to(dev), Vt
    elif method != "stream":
        raise ValueError(f"method must be 'auto', 'gram' or 'stream', got {method!r}")
    for _ in range(n_iter):
        Zn = comm.all_reduce_(L.power_iter_local(X_local, Z.to(dev), mean)).cpu()
        Z, _ = torch.linalg.qr(Zn)
    # Y = (X - mu) Z, then CholeskyQR2: Y <- Y R^-1 twice (fp64 throughout)
    Y = L.xw(X_local, Z.to(dev), mean=mean)
    Y2 = torch.empty_like(Y)
    for _ in range(2):
        G = comm.all_reduce_(L.xtx(Y)).cpu()
        G = 0.5 * (G + G.T)
        jitter = 0.0
        for _try in range(5):
            R, info = torch.linalg.cholesky_ex(G + jitter * torch.eye(l, dtype=G.dtype), upper=True)
            if int(info) == 0:
                break
            jitter = max(jitter * 10, 1e-12 * float(G.diagonal().max()))
        Rinv = torch.linalg.solve_triangular(R, torch.eye(l, dtype=R.dtype), upper=True)
        L.xw(Y, Rinv.to(dev), upper=True, out=Y2)
        Y, Y2 = Y2, Y
    # B = Q^T (X - mu) (l x d), as (X - mu)^T Q (d x l: the tall side on the tile rows)
    B = comm.all_reduce_(L.xtx(X_local, Y, mean_a=mean)).cpu().T
    Uhat, sv, Vt = torch.linalg.svd(B, full_matrices=False)
    U = L.xw(Y, Uhat[:, :k].contiguous().to(dev))
    Vt = Vt[:k].to(dev)
    if flip_sign:
        U, Vt = svd_flip_distributed(U, Vt, comm)
    return U, sv[:k].to(dev), Vt


# --------------------------------------------------------- PPCA dimension
def _assess_dimension(spectrum, rank, n_samples):
    """Log-likelihood of a rank ``rank`` PPCA model (Minka 2000)."""
    n_features = spectrum.shape[0]
    if not 1 <= rank < n_features:
        raise ValueError("the tested rank should be in [1, n_features - 1]")
    eps = 1e-15
    if spectrum[rank - 1] < eps:
        return -np.inf
    pu = -rank * np.log(2.0)
    for i in range(1, rank + 1):
        pu += gammaln((n_features - i + 1) / 2.0) - np.log(np.pi) * (n_features - i + 1) / 2.0
    pl = np.sum(np.log(spectrum[:rank]))
    pl = -pl * n_samples / 2.0
    v = max(eps, np.sum(spectrum[rank:]) / (n_features - rank))
    pv = -np.log(v) * n_samples * (n_features - rank) / 2.0
    m = n_features * rank - rank * (rank + 1.0) / 2.0
    pp = np.log(2.0 * np.pi) * (m + rank) / 2.0
    pa = 0.0
    spectrum_ = spectrum.copy()
    spectrum_[rank:n_features] = v
    for i in range(rank):
        for j in range(i + 1, len(spectrum)):
            pa += np.log((spectrum[i] - spectrum[j]) * (1.0 / spectrum_[j] - 1.0 / spectrum_[i])) + np.log(n_samples)
    return pu + pl + pv + pp - pa / 2.0 - rank * np.log(n_samples) / 2.0


def _infer_dimension(spectrum, n_samples):
    ll = np.empty_like(spectrum)
    ll[0] = -np.inf
    for rank in range(1, spectrum.shape[0]):
        ll[rank] = _assess_dimension(spectrum, rank, n_samples)
    return int(ll.argmax())


def density(w, **kwargs):
    """Fraction of non-zero entries of a vector / (sparse) matrix."""
    import scipy.sparse as _sp
    if hasattr(w, "toarray") and _sp.issparse(w):
        return float(w.nnz) / (w.shape[0] * w.shape[1])
    w = np.asarray(w)
    return 0.0 if w.size == 0 else float((w != 0).sum()) / w.size


def weighted_mode(a, w, *, axis=0):
    """Most frequent value along ``axis`` with weights ``w`` (ties: the
    smallest value; no positive weight at all: 0).  Returns (mode, score)
    with the reduced axis kept as size 1, like scipy.stats.mode."""
    if axis is None:
        a, w, axis = np.ravel(a), np.ravel(w), 0
    else:
        a, w = np.asarray(a), np.asarray(w)
    if a.shape != w.shape:
        w = np.broadcast_to(w, a.shape)
    values = np.unique(a)                                   # ascending
    totals = np.stack([np.where(a == v, w, 0).sum(axis=axis) for v in values])
    first_max = np.argmax(totals, axis=0)                   # first = smallest value
    best = np.take_along_axis(totals, first_max[None], 0)[0]
    mode = np.where(best > 0, values[first_max], 0).astype(float)
    return np.expand_dims(mode, axis), np.expand_dims(np.maximum(best, 0).astype(float), axis)


def cartesian(arrays, out=None):
    """All combinations of the input 1-D arrays as rows (first array varies
    slowest)."""
    arrays = [np.asarray(x) for x in arrays]
    dtype = np.result_type(*arrays)
    grids = np.meshgrid(*arrays, indexing="ij")
    res = np.stack([g.reshape(-1) for g in grids], axis=1).astype(dtype, copy=False)
    if out is not None:
        out[...] = res
        return out
    return res


def log_logistic(X, out=None):
    """log(1 / (1 + exp(-x))) computed stably elementwise (2-D input, as the
    reference)."""
    X = np.asarray(X, dtype=np.float64)
    is_1d = X.ndim == 1
    X = np.atleast_2d(X)
    res = -np.logaddexp(0.0, -X)
    if out is not None:
        out[...] = res.reshape(out.shape)
        return out
    return res[0] if is_1d else res


def softmax(X, copy=True):
    """Row-wise softmax (in place unless ``copy``)."""
    X = np.array(X, dtype=np.float64, copy=True) if copy else X
    X -= X.max(axis=1)[:, None]
    np.exp(X, X)
    X /= X.sum(axis=1)[:, None]
    return X


def make_nonnegative(X, min_value=0):
    """X shifted so that its minimum is at least ``min_value``."""
    X = np.asarray(X)
    min_ = X.min()
    if min_ < min_value:
        import scipy.sparse as _sp
        if _sp.issparse(X):
            raise ValueError("Cannot make the data matrix nonnegative because it is sparse."
                             " Adding a value to every entry would make it dense.")
        X = X + (min_value - min_)
    return X
