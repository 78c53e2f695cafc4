"""Centroid initialisation over row-sharded data.

``kmeans_plusplus`` follows the greedy k-means++ of the reference
(``_dmeans.py:153-247`` / ``cluster/_kmeans.py:153-247``): 2 + ln(k) local
trials per centre, candidates sampled proportionally to the current
potential, the trial with the lowest resulting potential kept.  The random
stream is a numpy RandomState shared (same seed) by every rank, so ranks
agree on every draw; the data-dependent parts are three collectives per
centre: the gather of shard potentials, the candidate rows (owner
contributes, others zeros) and the per-candidate potentials.
"""

import numpy as np
import torch

from .._data import Data, gather_rows
from ...ops import linalg as L


def _sq_dist(X, C, xn=None):
    Xf = X if X.dtype in (torch.float32, torch.float64) else X.float()
    Cf = C.to(Xf.dtype)
    if xn is None:
        xn = (Xf * Xf).sum(1)
    cn = (Cf * Cf).sum(1)
    return (xn[:, None] + cn[None, :] - 2.0 * (Xf @ Cf.T)).clamp_(min=0.0)


def kmeans_plusplus(data: Data, n_clusters, random_state, x_squared_norms=None,
                    n_local_trials=None):
    """Returns (centers [k, d] tensor on the data device, global indices)."""
    X = data.X
    comm = data.comm
    n = data.n_global
    k = int(n_clusters)
    if n_local_trials is None:
        n_local_trials = 2 + int(np.log(k))
    if x_squared_norms is None:
        x_squared_norms = L.row_norms_sq(X)
    xn = x_squared_norms.to(torch.float64 if X.device.type == "cpu" else torch.float32)
    rs = random_state
    indices = np.full(k, -1, dtype=np.int64)
    center_id = int(rs.randint(n))
    centers = torch.empty((k, data.d), dtype=torch.float64 if X.device.type == "cpu" else torch.float32,
                          device=X.device)
    c0 = gather_rows(data, [center_id])
    centers[0] = c0[0]
    indices[0] = center_id
    closest = _sq_dist(X, c0, xn)[:, 0].double()
    pot = closest.sum().reshape(1)
    comm.all_reduce_(pot)
    current_pot = float(pot.item())
    for c in range(1, k):
        rand_vals = rs.random_sample(n_local_trials) * current_pot
        cand_ids = _search_global(data, closest, rand_vals)
        cands = gather_rows(data, cand_ids)
        d_c = _sq_dist(X, cands, xn).double()                 # [n_loc, t]
        newd = torch.minimum(closest[:, None], d_c)
        pots = newd.sum(0)
        comm.all_reduce_(pots)
        best = int(torch.argmin(pots).item())
        current_pot = float(pots[best].item())
        closest = newd[:, best].contiguous()
        centers[c] = cands[best]
        indices[c] = cand_ids[best]
    return centers, indices


def _search_global(data: Data, closest, rand_vals):
    """Global row index of each value of the (replicated) rand_vals in the
    cumulative potential of the row-sharded ``closest``."""
    comm = data.comm
    local_sum = closest.sum().reshape(1)
    sums = torch.cat(comm.all_gather(local_sum)).double().cpu().numpy()
    prefix = np.concatenate([[0.0], np.cumsum(sums)])
    rank = comm.rank
    out = np.zeros(len(rand_vals), dtype=np.int64)
    mine = []
    for t, v in enumerate(rand_vals):
        owner = int(np.searchsorted(prefix[1:], v, side="left"))
        owner = min(owner, comm.world_size - 1)
        if owner == rank:
            mine.append((t, v - prefix[rank]))
    res = torch.zeros(len(rand_vals), dtype=torch.float64, device=closest.device)
    if mine:
        cs = torch.cumsum(closest, 0)
        vals = torch.tensor([m[1] for m in mine], dtype=torch.float64, device=closest.device)
        pos = torch.searchsorted(cs, vals)
        pos = pos.clamp(max=max(closest.numel() - 1, 0))
        for (t, _), p in zip(mine, pos.tolist()):
            res[t] = float(p + data.row_offset)
    comm.all_reduce_(res)
    out[:] = res.cpu().numpy().astype(np.int64)
    return np.minimum(out, data.n_global - 1)


def random_init(data: Data, n_clusters, random_state):
    seeds = random_state.permutation(data.n_global)[:n_clusters]
    return gather_rows(data, seeds), seeds
