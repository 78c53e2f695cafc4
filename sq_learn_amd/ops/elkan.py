"""Elkan bounded k-means assignment.

Reference: ``cluster/_k_means_elkan.pyx`` - ``init_bounds_dense`` (:33-101),
``elkan_iter_chunked_dense`` (:184-333, bound update :282-317),
``_update_chunk_dense`` (:336-409); centre geometry from
``cluster/_kmeans.py:_kmeans_single_elkan`` (half centre-centre distances and
the distance to the nearest other centre).

State per row: ``upper`` (>= distance to the assigned centre) and
``lower[j]`` (<= distance to centre j).  One call = the reference's bound
update with the previous centre shifts, followed by the assignment pass;
``init=True`` computes the initial bounds.

Device path: ``csrc/elkan.hip`` (one wave per row, lower bounds staged in
LDS, ballot over 64 centres, cooperative distance dot products); it follows
the reference's sequential per-row recurrence exactly.  The torch twin
(CPU, and GPU rows with d > 1024) keeps the same bound invariants with a
vectorised rule: a row that fails Elkan's skip test gets all k distances
(tight bounds) - the resulting labels are the exact argmin either way.
"""

import torch

from . import _native as nat


def centre_geometry(C):
    """(hcc, snext): half centre-centre distances (k x k, zero diagonal) and
    half the distance to each centre's nearest other centre (k,), computed
    in fp64 without the norm expansion, returned in ``C.dtype``."""
    Cd = C.double()
    D = torch.cdist(Cd, Cd, compute_mode="donot_use_mm_for_euclid_dist") * 0.5
    k = C.shape[0]
    if k > 1:
        off = D + torch.diag(torch.full((k,), float("inf"), dtype=D.dtype, device=D.device))
        snext = off.min(1).values
    else:
        snext = torch.full((1,), float("inf"), dtype=D.dtype, device=D.device)
    D.fill_diagonal_(0.0)
    return D.to(C.dtype).contiguous(), snext.to(C.dtype).contiguous()


def centre_shift(C_old, C_new):
    """Per-centre Euclidean displacement (k,), fp64 math, ``C_new.dtype``."""
    return torch.linalg.vector_norm(C_new.double() - C_old.double(), dim=1).to(C_new.dtype)


def _native_ok(X, k):
    if not nat.use_native(X) or X.dtype not in (torch.float32, torch.float64):
        return False
    return X.shape[1] <= 1024 and k * X.element_size() <= 65536


def elkan_step(X, C, hcc, snext, shift, labels, upper, lower, init=False):
    """In place on int32 ``labels``, ``upper`` (n,), ``lower`` (n, k).

    ``X`` (n, d) and ``C`` (k, d) share a float dtype with the bounds."""
    n, d = X.shape
    k = C.shape[0]
    if n == 0:
        return labels
    if _native_ok(X, k):
        dt = 0 if X.dtype == torch.float32 else 1
        nat.native().elkan_step(X.data_ptr(), C.data_ptr(), hcc.data_ptr(), snext.data_ptr(),
                                shift.data_ptr(), labels.data_ptr(), upper.data_ptr(),
                                lower.data_ptr(), n, d, k, dt, int(bool(init)),
                                nat.stream_handle(X.device))
        return labels
    return elkan_step_torch(X, C, hcc, snext, shift, labels, upper, lower, init)


def _distances(Xs, C):
    return torch.cdist(Xs, C, compute_mode="donot_use_mm_for_euclid_dist")


def elkan_step_torch(X, C, hcc, snext, shift, labels, upper, lower, init=False,
                     chunk_rows=1 << 14):
    n = X.shape[0]
    for s in range(0, n, chunk_rows):
        e = min(n, s + chunk_rows)
        Xs = X[s:e]
        if init:
            D = _distances(Xs, C)
            lower[s:e] = D
            m = D.min(1)
            labels[s:e] = m.indices.to(labels.dtype)
            upper[s:e] = m.values
            continue
        lab = labels[s:e].long()
        u = upper[s:e] + shift[lab]
        lo = (lower[s:e] - shift[None, :]).clamp_(min=0)
        act = u > snext[lab]
        if bool(act.any()):
            idx = act.nonzero()[:, 0]
            D = _distances(Xs[idx], C)
            lo[idx] = D
            m = D.min(1)
            lab = lab.clone()
            lab[idx] = m.indices
            u[idx] = m.values
        lower[s:e] = lo
        upper[s:e] = u
        labels[s:e] = lab.to(labels.dtype)
    return labels
