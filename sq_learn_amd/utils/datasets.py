"""Synthetic data generators (reference ``datasets/_samples_generator.py``:
``make_blobs`` :751, ``make_low_rank_matrix`` :1105, ``make_classification``
:38).

Two flavours:

* NumPy (``make_blobs`` etc.): sklearn-compatible signatures and RandomState
  semantics, for small data and CPU tests;
* device / sharded (``make_blobs_device``, ``make_low_rank_device``): rows
  generated directly in HBM (bf16 or fp32) by the Philox kernels, keyed by
  *global* row index - rank r of a G-GPU job generates exactly rows
  [start_r, stop_r) of the same global dataset, so 10M-50M-row benchmarks
  never touch the host.
"""

import numbers

import numpy as np
import torch

from .validation import check_random_state
from ..runtime.rng import RngKey, philox4x32, uniform_from_u32, MASK32
from ..ops.random import philox_normal, philox_uniform


# ------------------------------------------------------------------ NumPy
def make_blobs(n_samples=100, n_features=2, *, centers=None, cluster_std=1.0,
               center_box=(-10.0, 10.0), shuffle=True, random_state=None, return_centers=False):
    generator = check_random_state(random_state)
    if isinstance(n_samples, numbers.Integral):
        if centers is None:
            centers = 3
        if isinstance(centers, numbers.Integral):
            n_centers = centers
            centers = generator.uniform(center_box[0], center_box[1], size=(n_centers, n_features))
        else:
            centers = np.asarray(centers, dtype=float)
            n_features = centers.shape[1]
            n_centers = centers.shape[0]
    else:
        n_centers = len(n_samples)
        if centers is None:
            centers = generator.uniform(center_box[0], center_box[1], size=(n_centers, n_features))
        centers = np.asarray(centers, dtype=float)
        n_features = centers.shape[1]
    if hasattr(cluster_std, "__len__") and len(cluster_std) != len(centers):
        raise ValueError("Length of `clusters_std` not consistent with number of centers.")
    if isinstance(cluster_std, numbers.Real):
        cluster_std = np.full(len(centers), cluster_std)
    if isinstance(n_samples, numbers.Integral):
        per = [n_samples // n_centers] * n_centers
        for i in range(n_samples % n_centers):
            per[i] += 1
    else:
        per = list(n_samples)
    X, y = [], []
    for i, (n, std) in enumerate(zip(per, cluster_std)):
        X.append(generator.normal(loc=centers[i], scale=std, size=(n, n_features)))
        y += [i] * n
    X = np.concatenate(X)
    y = np.array(y)
    if shuffle:
        idx = np.arange(X.shape[0])
        generator.shuffle(idx)
        X, y = X[idx], y[idx]
    if return_centers:
        return X, y, centers
    return X, y


def make_low_rank_matrix(n_samples=100, n_features=100, *, effective_rank=10, tail_strength=0.5,
                         random_state=None):
    generator = check_random_state(random_state)
    n = min(n_samples, n_features)
    u, _ = np.linalg.qr(generator.randn(n_samples, n), mode="reduced")
    v, _ = np.linalg.qr(generator.randn(n_features, n), mode="reduced")
    singular_ind = np.arange(n, dtype=np.float64)
    low_rank = (1 - tail_strength) * np.exp(-1.0 * (singular_ind / effective_rank) ** 2)
    tail = tail_strength * np.exp(-0.1 * singular_ind / effective_rank)
    s = np.identity(n) * (low_rank + tail)
    return np.dot(np.dot(u, s), v.T)


def make_classification(n_samples=100, n_features=20, *, n_informative=2, n_redundant=2,
                        n_classes=2, class_sep=1.0, flip_y=0.01, random_state=None, shuffle=True):
    """Simplified make_classification: Gaussian clusters on hypercube
    vertices in the informative subspace + linear redundant features + noise."""
    rs = check_random_state(random_state)
    n_useless = n_features - n_informative - n_redundant
    if n_useless < 0:
        raise ValueError("n_features must be >= n_informative + n_redundant")
    y = np.arange(n_samples) % n_classes
    verts = rs.randint(0, 2, size=(n_classes, n_informative)) * 2 - 1
    Xi = verts[y] * class_sep + rs.randn(n_samples, n_informative)
    B = 2 * rs.rand(n_informative, n_redundant) - 1
    Xr = Xi @ B
    Xu = rs.randn(n_samples, n_useless)
    X = np.hstack([Xi, Xr, Xu])
    flip = rs.rand(n_samples) < flip_y
    y = y.copy()
    y[flip] = rs.randint(n_classes, size=int(flip.sum()))
    if shuffle:
        p = rs.permutation(n_samples)
        X, y = X[p], y[p]
    return X, y


# ---------------------------------------------------------------- device
def _centers_device(k, d, center_box, seed, device):
    key = RngKey(seed, "data", 0)
    u = philox_uniform((k, d), key, device=device)
    lo, hi = center_box
    return (lo + (hi - lo) * u.double()).to(torch.float32)


def blob_labels(row_start, row_stop, k, seed, device):
    """Cluster id of global rows [row_start, row_stop) (uniform over k)."""
    key = RngKey(seed, "data", 1)
    idx = torch.arange(row_start, row_stop, dtype=torch.int64, device=device)
    w = philox4x32(idx & MASK32, (idx >> 32) & MASK32, key.s0, key.s1, key.k0, key.k1)[0]
    return ((w * k) >> 32).to(torch.int64)


def make_blobs_device(n_samples, n_features, centers=8, cluster_std=1.0, center_box=(-10.0, 10.0),
                      seed=0, device="cuda", dtype=torch.bfloat16, row_range=None,
                      chunk_rows=1 << 20, return_centers=False):
    """Rows [start, stop) of a global make_blobs dataset generated in HBM.

    Returns (X_local [stop-start, d] dtype, y_local int64[, centers])."""
    device = torch.device(device)
    start, stop = row_range if row_range is not None else (0, n_samples)
    k = int(centers)
    C = _centers_device(k, n_features, center_box, seed, device)
    X = torch.empty((stop - start, n_features), dtype=dtype, device=device)
    y = blob_labels(start, stop, k, seed, device)
    nkey = RngKey(seed, "data", 2)
    for s in range(start, stop, chunk_rows):
        e = min(stop, s + chunk_rows)
        z = philox_normal((e - s, n_features), nkey, 0.0, cluster_std, dtype=torch.float32,
                          device=device, offset=s * n_features)
        z += C[y[s - start:e - start]]
        X[s - start:e - start] = z.to(dtype)
    if return_centers:
        return X, y, C
    return X, y


def make_low_rank_device(n_samples, n_features, effective_rank=10, tail_strength=0.5, seed=0,
                         device="cuda", dtype=torch.float32, row_range=None, chunk_rows=1 << 20):
    """Low-rank-plus-tail matrix A = G diag(s) V^T with G iid N(0, 1/n)
    (rows generated independently -> shardable); singular spectrum follows
    make_low_rank_matrix's bell + tail profile."""
    device = torch.device(device)
    start, stop = row_range if row_range is not None else (0, n_samples)
    n = min(n_samples, n_features)
    idx = torch.arange(n, dtype=torch.float64)
    s = ((1 - tail_strength) * torch.exp(-(idx / effective_rank) ** 2)
         + tail_strength * torch.exp(-0.1 * idx / effective_rank))
    vkey = RngKey(seed, "data", 3)
    Vg = philox_normal((n_features, n), vkey, dtype=torch.float64, device="cpu")
    V, _ = torch.linalg.qr(Vg)
    M = (torch.diag(s) @ V.T).to(torch.float32).to(device)          # [n, d]
    X = torch.empty((stop - start, n_features), dtype=dtype, device=device)
    gkey = RngKey(seed, "data", 4)
    scale = 1.0 / np.sqrt(n_samples)
    for r0 in range(start, stop, chunk_rows):
        r1 = min(stop, r0 + chunk_rows)
        G = philox_normal((r1 - r0, n), gkey, 0.0, scale, dtype=torch.float32, device=device,
                          offset=r0 * n)
        X[r0 - start:r1 - start] = (G @ M).to(dtype)
    return X
