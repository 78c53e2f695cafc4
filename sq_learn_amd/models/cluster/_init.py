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
two small collectives per centre on a multi-rank run (owner-contributes
all-reduce of the t packed candidate rows + ids, all-gather of the per-rank
t trial potentials, which also carries the next prefix of shard totals).  On
the GPU each centre reads only the rows a candidate can improve
(``csrc/kmpp.hip``: a triangle-inequality screen against each row's nearest
chosen centre, a certified bound from an int8 copy of the rows, exact
direct-form fp32 distances for the rest; fixed-point potentials so the
result does not depend on the screens or the rank count); elsewhere
``X C^T`` (library GEMM) with the min / sum epilogue in torch.

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


def _pick_candidates(data: Data, cs, prefix, sizes, vals, xdtype):
    """Candidate rows of the values ``vals`` (device, replicated) in the
    global cumulative potential, in ONE collective: the rank whose prefix
    range (prefix[r], prefix[r + 1]] holds a value (first non-empty such rank:
    left-side search, the reference's ``np.searchsorted``) resolves it in its
    local fp64 cumulative sum ``cs`` and contributes the row and its global
    id; one all-reduce of the packed [t, d + 1] block combines them.  An empty
    shard never owns a value (and never indexes its rows)."""
    comm = data.comm
    X = data.X
    t = vals.shape[0]
    d = data.d
    wd = torch.float64
    if comm.world_size > 1:
        ends = prefix[1:]
        ok = (ends[None, :] >= vals[:, None]) & (sizes[None, :] > 0)          # [t, W]
        nz = torch.nonzero(sizes > 0)
        last = nz[-1, 0] if nz.numel() else torch.zeros((), dtype=torch.int64, device=vals.device)
        owner = torch.where(ok.any(1), ok.to(torch.int32).argmax(1).to(torch.int64), last)
        local_vals = vals - prefix[comm.rank]
    else:
        owner = torch.zeros(t, dtype=torch.int64, device=vals.device)
        local_vals = vals
    if comm.world_size == 1:
        pos = torch.searchsorted(cs, local_vals.contiguous()).clamp(0, max(data.n_local - 1, 0))
        return X[pos].to(xdtype), (pos + data.row_offset).clamp(0, data.n_global - 1)
    packed = torch.zeros((t, d + 1), dtype=wd, device=X.device)
    if data.n_local > 0:
        pos = torch.searchsorted(cs, local_vals.contiguous()).clamp(max=data.n_local - 1)
        mine = (owner == comm.rank)
        packed[:, :d] = torch.where(mine[:, None], X[pos].to(wd), torch.zeros((), dtype=wd,
                                                                             device=X.device))
        packed[:, d] = torch.where(mine, (pos + data.row_offset).to(wd),
                                   torch.zeros((), dtype=wd, device=X.device))
    comm.all_reduce_(packed)   # ids < 2^53: exact in fp64
    ids = packed[:, d].round().to(torch.int64).clamp(0, data.n_global - 1)
    return packed[:, :d].to(xdtype), ids


def _pick_candidates_native(data: Data, state, prefix, sizes, vals, xdtype):
    """``_pick_candidates`` with the local search done by the device
    two-level sampler (``KmppState.pick``: fixed-point block totals, then a
    workgroup scan of the block) instead of a cumulative sum over the shard."""
    comm = data.comm
    X = data.X
    t = vals.shape[0]
    d = data.d
    if comm.world_size == 1:
        pos = state.pick(vals).clamp(0, max(data.n_local - 1, 0))
        return X[pos].to(xdtype), (pos + data.row_offset).clamp(0, data.n_global - 1)
    ends = prefix[1:]
    ok = (ends[None, :] >= vals[:, None]) & (sizes[None, :] > 0)          # [t, W]
    nz = torch.nonzero(sizes > 0)
    last = nz[-1, 0] if nz.numel() else torch.zeros((), dtype=torch.int64, device=vals.device)
    owner = torch.where(ok.any(1), ok.to(torch.int32).argmax(1).to(torch.int64), last)
    local_vals = vals - prefix[comm.rank]
    wd = torch.float64
    packed = torch.zeros((t, d + 1), dtype=wd, device=X.device)
    if data.n_local > 0:
        pos = state.pick(local_vals).clamp(0, data.n_local - 1)
        mine = (owner == comm.rank)
        packed[:, :d] = torch.where(mine[:, None], X[pos].to(wd), torch.zeros((), dtype=wd,
                                                                             device=X.device))
        packed[:, d] = torch.where(mine, (pos + data.row_offset).to(wd),
                                   torch.zeros((), dtype=wd, device=X.device))
    comm.all_reduce_(packed)   # ids < 2^53: exact in fp64
    ids = packed[:, d].round().to(torch.int64).clamp(0, data.n_global - 1)
    return packed[:, :d].to(xdtype), ids


def _kmeans_plusplus_native(data: Data, k, rs, t, w, prune, stats=None, Xf=None):
    """The exact accelerated k-means++ on the device (csrc/kmpp.hip, see
    ``ops.kmeans.KmppState``): per centre one pick (two-level sampling of
    the t candidates), one trial pass that reads only the rows a candidate
    can improve, two small collectives on a multi-rank run; potentials in
    exact fixed point (identical results with or without the screens and on
    any number of ranks)."""
    from ...ops.kmeans import KmppState
    X = data.X if Xf is None else Xf     # fp32 rows (a bf16 shard is widened once)
    comm = data.comm
    dev = X.device
    n = data.n_global
    center_id = int(rs.randint(n))
    draws = torch.as_tensor(rs.random_sample((max(k - 1, 0), t)), dtype=torch.float64, device=dev)
    ids = torch.empty(k, dtype=torch.int64, device=dev)
    ids[0] = center_id
    c0 = gather_rows(data, [center_id]).to(torch.float32)
    centers = torch.empty((k, data.d), dtype=torch.float32, device=dev)
    centers[0] = c0[0]
    state = KmppState(X, k, t, w=w, prune=prune)
    mx = state.first_centre(c0[0])
    comm.all_reduce_(mx, op="max")
    P = state.set_scale(mx.item(), n)                                   # local total [1]
    ts = torch.cat([P, torch.tensor([float(data.n_local)], dtype=torch.float64, device=dev)])
    g = torch.stack(comm.all_gather(ts))                                  # [W, 2]
    totals, sizes = g[:, 0].contiguous(), g[:, 1].contiguous()
    W = comm.world_size
    if W == 1 and data.n_local > 0 and X.dtype == torch.float32:
        # one rank: pick (+ row copy), trial pass, one finishing launch per
        # centre - no host-side tensor chain
        Pd = P.clone()
        vals = (draws[0] * Pd) if k > 1 else torch.zeros(t, dtype=torch.float64, device=dev)
        cands = torch.empty((t, data.d), dtype=torch.float32, device=dev)
        cand_ids = torch.empty(t, dtype=torch.int64, device=dev)
        for c in range(1, k):
            state.pick(vals, cands, cand_ids, data.row_offset, n)
            state.trials(cands, centers, c, reduce=False)
            state.finish(Pd, draws[c] if c < k - 1 else None, vals, cands, cand_ids, centers, ids,
                         c)
            if stats is not None:
                stats.append(state.list_counts())
        return centers, ids.cpu().numpy()
    zero = torch.zeros(1, dtype=torch.float64, device=dev)
    for c in range(1, k):
        prefix = torch.cat([zero, torch.cumsum(totals, 0)])
        vals = draws[c - 1] * prefix[-1]
        cands, cand_ids = _pick_candidates_native(data, state, prefix, sizes, vals, torch.float32)
        delta = state.trials(cands, centers, c)
        pots_loc = P - delta                                              # exact integers
        if W > 1:
            allp = torch.stack(comm.all_gather(pots_loc.reshape(t)))     # [W, t]
            pots = allp.sum(0)
        else:
            allp = pots_loc.reshape(1, t)
            pots = pots_loc
        best = torch.argmin(pots)
        totals = allp.index_select(1, best.reshape(1))[:, 0].contiguous()
        P = totals[comm.rank:comm.rank + 1].clone()
        state.apply(best, c)
        centers[c] = cands.index_select(0, best.reshape(1))[0]
        ids[c] = cand_ids.index_select(0, best.reshape(1))[0]
        if stats is not None:
            stats.append(state.list_counts())
    return centers, ids.cpu().numpy()


def kmeans_plusplus(data: Data, n_clusters, random_state, x_squared_norms=None,
                    n_local_trials=None, sample_weight=None, prune=None, stats=None):
    """Returns (centers [k, d] tensor on the data device, global indices).

    ``sample_weight`` (framework extension, used by k-means||): the potential
    of a row is w * d^2.

    GPU (fp32 rows, d % 4 == 0): the exact accelerated k-means++ of
    ``_kmeans_plusplus_native`` (``prune``: the triangle / int8 screens,
    default on; ``SQ_KMPP_PRUNE=0`` turns them off; ``stats``: a list that
    receives per centre [survivor rows, exact rows]).  Elsewhere the torch
    path below.

    Collectives on a multi-rank run: TWO per centre, both tiny and with no
    host synchronisation - the all-reduce of the packed candidate rows + ids
    (``_pick_candidates``) and the all-gather of the per-rank trial
    potentials [W, t].  The gather gives both the global trial potentials
    (summed in rank order, identical on every rank) and, at the winning
    trial, every shard's new potential total - the prefix the next centre's
    search needs (the former separate all-gather of the shard totals)."""
    import os
    X = data.X
    comm = data.comm
    n = data.n_global
    k = int(n_clusters)
    dev = X.device
    if n_local_trials is None:
        n_local_trials = 2 + int(np.log(k))
    t = int(n_local_trials)
    Xf = X if X.dtype in (torch.float32, torch.float64) else X.float()
    rs = random_state
    w = None if sample_weight is None else sample_weight.to(torch.float64).to(dev).contiguous()
    native = (dev.type == "cuda" and Xf.dtype == torch.float32 and Xf.dim() == 2
              and Xf.stride(1) == 1 and Xf.stride(0) % 4 == 0 and data.d % 4 == 0
              and Xf.data_ptr() % 16 == 0 and 1 <= t <= 16 and k >= 1)
    if native:
        if prune is None:
            prune = os.environ.get("SQ_KMPP_PRUNE", "1") != "0"
        return _kmeans_plusplus_native(data, k, rs, t, w, bool(prune), stats, Xf=Xf)
    if x_squared_norms is None:
        x_squared_norms = L.row_norms_sq(X)
    xn = x_squared_norms.to(Xf.dtype)
    center_id = int(rs.randint(n))
    draws = torch.as_tensor(rs.random_sample((max(k - 1, 0), t)), dtype=torch.float64, device=dev)
    ids = torch.empty(k, dtype=torch.int64, device=dev)
    ids[0] = center_id
    c0 = gather_rows(data, [center_id]).to(Xf.dtype)
    centers = torch.empty((k, data.d), dtype=Xf.dtype, device=dev)
    centers[0] = c0[0]
    if data.n_local:
        closest = _sq_dist(Xf, c0, xn)[:, 0].double()
    else:
        closest = torch.zeros(0, dtype=torch.float64, device=dev)
    pot_rows = closest if w is None else closest * w
    W = comm.world_size
    # shard potential totals and sizes (one all-gather for the first centre)
    ts = torch.stack([pot_rows.sum(), torch.tensor(float(data.n_local), dtype=torch.float64,
                                                   device=dev)])
    g = torch.stack(comm.all_gather(ts))                                  # [W, 2]
    totals, sizes = g[:, 0].contiguous(), g[:, 1].contiguous()
    zero = torch.zeros(1, dtype=torch.float64, device=dev)
    for c in range(1, k):
        prefix = torch.cat([zero, torch.cumsum(totals, 0)])
        current_pot = prefix[-1]
        vals = draws[c - 1] * current_pot
        cs = torch.cumsum(pot_rows, 0)
        cands, cand_ids = _pick_candidates(data, cs, prefix, sizes, vals, Xf.dtype)
        newd = torch.minimum(closest[:, None], _sq_dist(Xf, cands, xn).double())   # [n_loc, t]
        pots_loc = (newd if w is None else newd * w[:, None]).sum(0)
        allp = torch.stack(comm.all_gather(pots_loc.reshape(t)))          # [W, t]
        pots = allp[0].clone()
        for r in range(1, W):                                             # rank order: replicated
            pots += allp[r]
        best = torch.argmin(pots)
        totals = allp.index_select(1, best.reshape(1))[:, 0].contiguous()
        closest = newd.index_select(1, best.reshape(1))[:, 0].contiguous()
        pot_rows = closest if w is None else closest * w
        centers[c] = cands.index_select(0, best.reshape(1))[0]
        ids[c] = cand_ids.index_select(0, best.reshape(1))[0]
    return centers, ids.cpu().numpy()


def kmeans_plusplus_restarts(data: Data, n_clusters, random_state, n_restarts,
                             n_local_trials=None, prune=None):
    """The k-means++ initialisations of ``n_restarts`` consecutive restarts
    (reference: ``_dmeans.py:1285-1306`` runs ``_init_centroids`` once per
    restart, and its Lloyd loop never draws from ``random_state``): every
    restart's draws - ``randint(n)`` then ``random_sample((k - 1, t))``
    (``_dmeans.py:153-247``) - are taken up front in that order, then the
    restarts run together on the device (``ops.kmeans.KmppBatch``: one
    launch per phase for all of them, rows shared).  Returns a list of
    [k, d] centre tensors identical to sequential ``kmeans_plusplus`` calls,
    or None where the batched device path does not apply (one rank, fp32
    rows on the GPU, no sample weights)."""
    import os
    from ...ops.kmeans import KmppBatch
    X = data.X
    dev = X.device
    k = int(n_clusters)
    if n_local_trials is None:
        n_local_trials = 2 + int(np.log(k))
    t = int(n_local_trials)
    Xf = X if X.dtype in (torch.float32, torch.float64) else X.float()
    if not (dev.type == "cuda" and data.comm.world_size == 1 and Xf.dtype == torch.float32
            and Xf.dim() == 2 and Xf.stride(1) == 1 and Xf.stride(0) % 4 == 0
            and data.d % 4 == 0 and Xf.data_ptr() % 16 == 0 and 1 <= t <= 16 and k >= 2
            and n_restarts >= 1 and data.n_local > 0):
        return None
    if prune is None:
        prune = os.environ.get("SQ_KMPP_PRUNE", "1") != "0"
    rs = random_state
    n = data.n_global
    # device memory per restart (closest, nearest, 2 masks, 2 x t distances,
    # 2 row lists): restarts run in groups that fit half the free memory
    per = data.n_local * (4 + 4 + 4 + 8 * t + 8) + k * data.d * 4
    free = torch.cuda.mem_get_info(dev)[0]
    group = max(1, min(int(n_restarts), int(0.5 * free // max(per, 1))))
    if prune:
        # the fused screen / bound hold <= 16 restarts and <= 128 trial columns
        tp = 1 << max(0, (t - 1).bit_length())
        group = min(group, 16, max(1, 128 // tp))
    out = []
    for g0 in range(0, int(n_restarts), group):
        nr = min(group, int(n_restarts) - g0)
        ids0, draws = [], []
        for _ in range(nr):
            ids0.append(int(rs.randint(n)))
            draws.append(rs.random_sample((k - 1, t)))
        c0s = torch.stack([gather_rows(data, [i]).to(torch.float32)[0] for i in ids0])
        batch = KmppBatch(Xf, k, t, nr, prune=bool(prune))
        centers, _ = batch.run(c0s, torch.as_tensor(np.stack(draws), dtype=torch.float64),
                               torch.tensor(ids0, dtype=torch.int64, device=dev), n,
                               row_offset=data.row_offset)
        out += [centers[r].clone() for r in range(nr)]
        del batch
    return out


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


def permutation_head(random_state, n, k):
    """``random_state.permutation(n)[:k]`` with the identical draws and the
    identical generator state afterwards (the reference's 'random' init,
    ``_kmeans.py`` ``_init_centroids``), run natively for large n
    (``csrc/host/mt_permutation.cpp``: the legacy MT19937 Fisher-Yates pass
    over int32 instead of numpy's over int64).  Falls back to numpy for
    generators that are not a legacy MT19937 RandomState."""
    n, k = int(n), int(k)
    try:
        st = random_state.get_state()
    except AttributeError:
        st = None
    if (st is None or not isinstance(st, tuple) or st[0] != "MT19937" or n < (1 << 16)
            or n >= (1 << 31)):
        return random_state.permutation(n)[:k]
    from ...ops import _host
    key = np.array(st[1], dtype=np.uint32).copy()
    pos = np.array([int(st[2])], dtype=np.int32)
    out = np.empty(max(k, 1), dtype=np.int64)
    rc = _host.lib().sqh_mt_permutation_head(_host.ptr(key), _host.ptr(pos), n, k,
                                              _host.ptr(out))
    if rc:
        raise RuntimeError("sqh_mt_permutation_head failed")
    random_state.set_state(("MT19937", key, int(pos[0]), st[3], st[4]))
    return out[:k]


def random_init(data: Data, n_clusters, random_state):
    seeds = permutation_head(random_state, data.n_global, n_clusters)
    return gather_rows(data, seeds), seeds
