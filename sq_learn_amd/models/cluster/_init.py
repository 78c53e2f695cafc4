"""Centroid initialisation over row-sharded data.

``kmeans_plusplus`` is the greedy k-means++ of the reference
(``_dmeans.py:153-247`` / ``cluster/_kmeans.py:153-247``): 2 + ln(k) local
trials per centre, candidates sampled proportionally to the current
potential (searchsorted in the fp64 cumulative sum), the trial with the
lowest resulting potential kept.  The random stream is the reference's
RandomState draws (``randint(n)`` then ``random_sample(n_local_trials)`` per
centre), generated for all centres up front and shared by every rank.

Every centre is enqueued on the device with NO host synchronisation: the
current potential, the candidate ids, the argmin over trials and the
closest-distance column are device tensors; the data-dependent parts are
three small collectives per centre on a multi-rank run (all-gather of the
shard totals of the potential, owner-contributes all-reduce of the t
candidate rows, all-reduce of the t trial potentials).  The per-centre
work is one pass over the shard: on the GPU the fused trial kernel
(``csrc/kmpp.hip``: direct-form fp32 distances to the t candidates, the
t potentials as fixed-order fp64 block partials, distances written
transposed so the winner's column is contiguous); elsewhere ``X C^T``
(library GEMM) with the min / sum epilogue in torch.

``kmeans_parallel`` is k-means|| (Bahmani et al. 2012), an option the
reference does not have: O(log phi) oversampling rounds of ~l = 2k rows
each, drawn independently with p = min(1, l d^2(x) / phi) from a counter-
based Philox stream (shard invariant), distances to the growing candidate
set by the device E-step (exact fp32 minimum distances), then the weighted
candidates (weight = rows closest to each) reduced to k centres by the same
greedy k-means++ on the small weighted set.
"""

import math

import numpy as np
import torch

from .._data import Data, gather_rows
from ...ops import linalg as L
from ...ops import kmeans as K
from ...runtime.rng import RngKey


def _sq_dist(X, C, xn=None):
    Xf = X if X.dtype in (torch.float32, torch.float64) else X.float()
    Cf = C.to(Xf.dtype)
    if xn is None:
        xn = (Xf * Xf).sum(1)
    cn = (Cf * Cf).sum(1)
    return (xn[:, None] + cn[None, :] - 2.0 * (Xf @ Cf.T)).clamp_(min=0.0)


def _gather_rows_device(data: Data, ids):
    """Rows of the global indices ``ids`` (device int64 tensor) on every
    rank: the owner contributes, one all-reduce, no host sync."""
    X = data.X
    lo = data.row_offset
    loc = (ids - lo).clamp(0, max(data.n_local - 1, 0))
    mine = (ids >= lo) & (ids < lo + data.n_local)
    rows = X[loc].to(torch.float64 if X.device.type == "cpu" else torch.float32)
    rows = torch.where(mine[:, None], rows, torch.zeros_like(rows))
    data.comm.all_reduce_(rows)
    return rows


def _search_device(data: Data, cs, total_local, vals):
    """Global row of each value of ``vals`` (device, replicated) in the
    cumulative potential: shard totals all-gathered, each trial resolved by
    the rank whose prefix range holds it (searchsorted in its local fp64
    cumulative sum ``cs``), ids combined by a sum all-reduce."""
    comm = data.comm
    if comm.world_size > 1:
        tot = torch.cat(comm.all_gather(total_local.reshape(1)))
        prefix = torch.cat([torch.zeros(1, dtype=tot.dtype, device=tot.device), torch.cumsum(tot, 0)])
        owner = torch.searchsorted(prefix[1:].contiguous(), vals).clamp(max=comm.world_size - 1)
        local_vals = vals - prefix[comm.rank]
    else:
        owner = torch.zeros_like(vals, dtype=torch.int64)
        local_vals = vals
    pos = torch.searchsorted(cs, local_vals.contiguous()).clamp(max=max(cs.numel() - 1, 0))
    ids = torch.where(owner == comm.rank, pos + data.row_offset, torch.zeros_like(pos))
    if comm.world_size > 1:
        comm.all_reduce_(ids)
    return ids.clamp(max=data.n_global - 1)


def kmeans_plusplus(data: Data, n_clusters, random_state, x_squared_norms=None,
                    n_local_trials=None, sample_weight=None):
    """Returns (centers [k, d] tensor on the data device, global indices).

    ``sample_weight`` (framework extension, used by k-means||): the potential
    of a row is w * d^2."""
    X = data.X
    comm = data.comm
    n = data.n_global
    k = int(n_clusters)
    dev = X.device
    if n_local_trials is None:
        n_local_trials = 2 + int(np.log(k))
    t = int(n_local_trials)
    Xf = X if X.dtype in (torch.float32, torch.float64) else X.float()
    if x_squared_norms is None:
        x_squared_norms = L.row_norms_sq(X)
    xn = x_squared_norms.to(Xf.dtype)
    rs = random_state
    center_id = int(rs.randint(n))
    draws = torch.as_tensor(rs.random_sample((max(k - 1, 0), t)), dtype=torch.float64, device=dev)
    w = None if sample_weight is None else sample_weight.to(torch.float64).to(dev).contiguous()
    ids = torch.empty(k, dtype=torch.int64, device=dev)
    ids[0] = center_id
    c0 = gather_rows(data, [center_id]).to(Xf.dtype)
    centers = torch.empty((k, data.d), dtype=Xf.dtype, device=dev)
    centers[0] = c0[0]
    closest = _sq_dist(Xf, c0, xn)[:, 0].double()
    pot_rows = closest if w is None else closest * w
    total = pot_rows.sum()
    current_pot = comm.all_reduce_(total.clone().reshape(1))[0]
    # fused HIP trial pass (csrc/kmpp.hip): one HBM pass over the shard per
    # centre, no [n, t] temporaries; the torch path below is the CPU / odd-
    # shape fallback
    native = (dev.type == "cuda" and Xf.dtype == torch.float32 and Xf.dim() == 2
              and Xf.stride(1) == 1 and Xf.stride(0) == data.d and data.d % 4 == 0
              and Xf.data_ptr() % 16 == 0 and 1 <= t <= 16)
    D = part = None
    for c in range(1, k):
        vals = draws[c - 1] * current_pot
        cs = torch.cumsum(pot_rows, 0)
        cand_ids = _search_device(data, cs, total, vals)
        cands = _gather_rows_device(data, cand_ids).to(Xf.dtype)
        if native:
            D, pots = K.kmpp_trials_native(Xf, cands.contiguous(), closest, w, D, part)
            comm.all_reduce_(pots)
            best = torch.argmin(pots)
            current_pot = pots[best]
            closest = torch.minimum(closest, D.index_select(0, best.reshape(1))[0].double())
            pot_rows = closest if w is None else closest * w
            total = pot_rows.sum()
            centers[c] = cands.index_select(0, best.reshape(1))[0]
            ids[c] = cand_ids.index_select(0, best.reshape(1))[0]
            continue
        newd = torch.minimum(closest[:, None], _sq_dist(Xf, cands, xn).double())   # [n_loc, t]
        pots = (newd if w is None else newd * w[:, None]).sum(0)
        comm.all_reduce_(pots)
        best = torch.argmin(pots)
        current_pot = pots[best]
        closest = newd.index_select(1, best.reshape(1))[:, 0].contiguous()
        pot_rows = closest if w is None else closest * w
        total = pot_rows.sum()
        centers[c] = cands.index_select(0, best.reshape(1))[0]
        ids[c] = cand_ids.index_select(0, best.reshape(1))[0]
    return centers, ids.cpu().numpy()


def kmeans_parallel(data: Data, n_clusters, random_state, x_squared_norms=None, seed=0,
                    oversampling=2.0, rounds=5):
    """k-means|| initialisation (see the module docstring).  Returns
    (centers [k, d] tensor, None).  Each round's new candidates go through
    one device E-step (``LloydEngine.estep``, exact minimum distances) and
    are merged into the running (min distance, closest candidate)."""
    from ._lloyd import LloydEngine
    from ...ops.random import philox_uniform
    X = data.X
    comm = data.comm
    dev = X.device
    k = int(n_clusters)
    ell = oversampling * k
    rs = random_state
    first = int(rs.randint(data.n_global))
    wd = torch.float32 if dev.type == "cuda" else torch.float64
    C = gather_rows(data, [first]).to(wd)
    xn = x_squared_norms if x_squared_norms is not None else L.row_norms_sq(X)

    def nearest(Cnew):
        eng = LloydEngine(X, Cnew.shape[0], delta=0.0, seed=seed, comm=comm,
                          row_offset=data.row_offset, gemm_precision="fp32", xn=xn)
        lab, mind, _ = eng.estep(Cnew)
        return lab.long(), mind.double().clamp(min=0.0)

    label, d2 = nearest(C)
    phi = comm.all_reduce_(d2.sum().reshape(1))[0]
    key = RngKey(seed, "init", 0xC0FFEE)
    for r in range(int(rounds)):
        u = philox_uniform((data.n_local,), key.derive(sub=r), device=dev, offset=data.row_offset)
        p = (ell * d2 / phi).clamp(max=1.0)
        pick = torch.nonzero(u.double() < p)[:, 0]
        new = X[pick].to(wd)
        allnew = torch.cat(comm.all_gather_varlen(new), 0) if comm.world_size > 1 else new
        if allnew.shape[0] == 0:
            break
        lab_n, d2_n = nearest(allnew)
        closer = d2_n < d2
        label = torch.where(closer, lab_n + C.shape[0], label)
        d2 = torch.where(closer, d2_n, d2)
        C = torch.cat([C, allnew], 0)
        phi = comm.all_reduce_(d2.sum().reshape(1))[0]
    # candidate weights: rows closest to each candidate (all ranks)
    wts = torch.bincount(label, minlength=C.shape[0]).double()
    comm.all_reduce_(wts)
    if C.shape[0] <= k:
        extra = k - C.shape[0]
        if extra:
            more, _ = kmeans_plusplus(data, extra + 1, rs, xn)
            C = torch.cat([C, more[1:].to(C.dtype)], 0)
        return C[:k], None
    cand = Data(C, C.shape[0], 0, type(comm)(None), "tensor")
    centers, _ = kmeans_plusplus(cand, k, rs, sample_weight=wts)
    return centers, None


def random_init(data: Data, n_clusters, random_state):
    seeds = random_state.permutation(data.n_global)[:n_clusters]
    return gather_rows(data, seeds), seeds
