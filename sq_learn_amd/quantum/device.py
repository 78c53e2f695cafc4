"""Batched, device-capable versions of the QuantumUtility error model.

Same laws as :mod:`.reference` (the NumPy oracle), restructured for tensors:

* :func:`gaussian_tomography` - the ``true_tomography=False`` approximation
  (``Utility.py:88-104``) as one fused Philox truncated-normal add;
* :func:`tomography_rows_torch` - shot-based vector tomography
  (``Utility.py:259-402``) for a batch of rows.  The reference runs up to 100
  geomspace checkpoints *sequentially per row*, each with fresh measurements,
  and stops at the first estimate within delta of the true vector.  Because
  the checkpoints are independent experiments, all of them are sampled at
  once here (multinomials by conditional binomials, vectorised over
  rows x checkpoints) and the stopping rule picks the first passing
  checkpoint - the same distribution in O(d) batched kernel launches instead
  of O(rows * checkpoints * N) Python work.
* :func:`tomography_long` - the same algorithm for LONG vectors (the qPCA
  left singular vectors, length n = 1e6..1e7, ``_qPCA.py:1059-1063``),
  optionally row-sharded over the ranks: multinomials by a segmented
  binomial-splitting tree (``csrc/tomography.hip: mnom_segments_kernel``)
  with the ranks as the top level of the tree.
"""

import math

import numpy as np
import torch

from ..runtime.rng import RngKey
from .reference import check_measure


def gaussian_tomography(A, noise, key: RngKey, offset=0, numel=None, row_stride=None):
    """A + TN(+-noise/sqrt(numel)) per component (Frobenius budget; ``numel``
    defaults to A.numel(), pass the global count for a shard of a matrix).
    Element (i, j) draws Philox element ``offset + i * row_stride + j``
    (``row_stride`` defaults to the row length): a column shard of an
    r x n_global matrix passes row_stride = n_global and offset = its first
    column, so every element draws the value it draws unsharded."""
    from ..ops.random import trunc_normal_add_
    if noise == 0:
        return A
    out = A.clone() if A.dtype in (torch.float32, torch.float64) else A.float()
    out = out.contiguous()
    b = float(noise) / math.sqrt(out.numel() if numel is None else numel)
    if row_stride is None or out.dim() != 2 or row_stride == out.shape[1]:
        trunc_normal_add_(out.view(-1), b, key, offset=offset)
    else:
        for i in range(out.shape[0]):
            trunc_normal_add_(out[i], b, key, offset=offset + i * int(row_stride))
    return out


def _generator_for(key: RngKey, device):
    g = torch.Generator(device=device)
    seed = (key.k0 ^ (key.k1 << 32) ^ (key.stream * 0x9E3779B97F4A7C15)) & ((1 << 63) - 1)
    g.manual_seed(seed)
    return g


def _multinomial_counts(n_shots, probs, gen):
    """Counts of the first ``m`` outcomes of a multinomial over probs[..., :m]
    plus an implicit remainder outcome.  n_shots: [B] float, probs: [B, m]
    (rows may sum to < 1: the rest is the remainder)."""
    B, m = probs.shape
    counts = torch.zeros((B, m), dtype=torch.float64, device=probs.device)
    n_rem = n_shots.to(torch.float64).clone()
    p_rem = torch.ones(B, dtype=torch.float64, device=probs.device)
    for i in range(m):
        p = probs[:, i]
        q = torch.where(p_rem > 0, (p / p_rem).clamp(0.0, 1.0), torch.zeros_like(p))
        c = torch.binomial(n_rem, q, generator=gen)
        counts[:, i] = c
        n_rem = n_rem - c
        p_rem = (p_rem - p).clamp(min=0.0)
    return counts


def tomography_rows_torch(A, delta, key: RngKey, norm="L2", N=None,
                          stop_when_reached_accuracy=True, incremental_measure=True,
                          faster_measure_increment=0, preserve_norm=False, **_ignored):
    """Real tomography of every row of ``A`` (float64 tensor, any device)."""
    A = A.to(torch.float64)
    squeeze = A.ndim == 1
    if squeeze:
        A = A[None, :]
    r, d = A.shape
    dev = A.device
    gen = _generator_for(key, dev)
    nrm = torch.linalg.norm(A, dim=1)
    close = torch.isclose(nrm, torch.ones_like(nrm), rtol=1e-2)
    V = torch.where(close[:, None], A, A / nrm.clamp(min=1e-300)[:, None])
    if N is None:
        N = int((36 * d * np.log(d)) / (delta ** 2)) if norm == "L2" else int((36 * np.log(d)) / (delta ** 2))
    if incremental_measure:
        sched = check_measure(np.geomspace(1, N, num=100, dtype=np.int64), faster_measure_increment)
    else:
        sched = np.array([int(N)], dtype=np.int64)
    T = len(sched)
    if d + 1 > 512:
        out = tomography_long(A, delta, key, norm=norm, N=N,
                              stop_when_reached_accuracy=stop_when_reached_accuracy,
                              incremental_measure=incremental_measure,
                              faster_measure_increment=faster_measure_increment,
                              preserve_norm=preserve_norm)
        return out[0] if squeeze else out
    if dev.type == "cuda" and d + 1 <= 512:
        out = _tomography_rows_native(V.contiguous(), sched, delta, key, norm,
                                      incremental_measure and stop_when_reached_accuracy)
        if preserve_norm:
            out = out * nrm[:, None]
        return out[0] if squeeze else out
    shots = torch.as_tensor(sched, dtype=torch.float64, device=dev)
    # batch = rows x checkpoints
    Vb = V[:, None, :].expand(r, T, d).reshape(r * T, d)
    nb = shots[None, :].expand(r, T).reshape(-1)
    pv = Vb ** 2
    pv = pv / pv.sum(1, keepdim=True)
    cnt = _multinomial_counts(nb, pv, gen)
    P = torch.sqrt(cnt / nb[:, None])
    amp_p = 0.5 * (Vb + P)
    amp_m = 0.5 * (Vb - P)
    Z = (amp_p ** 2).sum(1) + (amp_m ** 2).sum(1)
    p_plus = amp_p ** 2 / Z[:, None]
    plus = _multinomial_counts(nb, p_plus, gen)
    est = torch.where(plus > 0.4 * P ** 2 * nb[:, None], P, -P).reshape(r, T, d)
    if incremental_measure and stop_when_reached_accuracy:
        diff = V[:, None, :] - est
        err = diff.norm(dim=2) if norm == "L2" else diff.abs().amax(dim=2)
        ok = err <= delta
        first = torch.where(ok.any(1), ok.float().argmax(1), torch.full((r,), T - 1, device=dev))
    else:
        first = torch.full((r,), T - 1, dtype=torch.int64, device=dev)
    out = est[torch.arange(r, device=dev), first.long()]
    if preserve_norm:
        out = out * nrm[:, None]
    return out[0] if squeeze else out


_SEG = 2048   # outcomes per segment of mnom_segments_kernel (kSegP)


def multinomial_long(N, W, wrow, key: RngKey, sid, level=0):
    """Counts ``[B, m]`` with row b ~ Multinomial(N[b], W[wrow[b]] / sum)
    (fp64 weights >= 0, any length m) on the device: segment totals are drawn
    one level up from the segment masses (recursively), then one workgroup per
    segment splits its total down an LDS binomial tree.  Deterministic in
    (key, sid[b], level)."""
    from ..ops import _native as nat
    W = W.to(torch.float64).contiguous()
    Wr, m = W.shape
    B = int(N.numel())
    dev = W.device
    wrow = wrow.to(device=dev, dtype=torch.int64).contiguous()
    sid = sid.to(device=dev, dtype=torch.int64).contiguous()
    if bool((wrow < 0).any()) or bool((wrow >= Wr).any()):
        raise IndexError("multinomial_long: weight row index out of range")
    if m <= _SEG:
        Nseg = N.to(device=dev, dtype=torch.float64).contiguous()
    else:
        nfull = m // _SEG
        nseg = -(-m // _SEG)
        Wb = torch.zeros((Wr, nseg), dtype=torch.float64, device=dev)
        Wb[:, :nfull] = W[:, : nfull * _SEG].reshape(Wr, nfull, _SEG).clamp(min=0).sum(-1)
        if nseg > nfull:
            Wb[:, nfull] = W[:, nfull * _SEG:].clamp(min=0).sum(-1)
        Nseg = multinomial_long(N, Wb, wrow, key, sid, level + 1).reshape(-1).contiguous()
    cnt = torch.empty((B, m), dtype=torch.float64, device=dev)
    rc = nat.native().mnom_segments(W.data_ptr(), W.stride(0), wrow.data_ptr(), m, B,
                                    Nseg.data_ptr(), cnt.data_ptr(), cnt.stride(0), key.k0,
                                    key.k1, key.s0, key.s1, sid.data_ptr(), int(level),
                                    nat.stream_handle(dev))
    if rc:
        raise RuntimeError(f"mnom_segments failed (hip error {rc})")
    return cnt


def _multinomial_np(N, W, wrow, rng):
    """CPU twin of :func:`multinomial_long` (same law, numpy stream)."""
    W = np.asarray(W, dtype=np.float64)
    out = np.zeros((len(N), W.shape[1]), dtype=np.float64)
    for b, (n, r) in enumerate(zip(np.asarray(N), np.asarray(wrow))):
        w = np.clip(W[r], 0, None)
        tot = w.sum()
        if n > 0 and tot > 0:
            out[b] = rng.multinomial(int(n), w / tot)
    return out


def tomography_long(A, delta, key: RngKey, norm="L2", N=None, stop_when_reached_accuracy=True,
                    incremental_measure=True, faster_measure_increment=0, preserve_norm=False,
                    comm=None, n_global=None, max_batch_elems=1 << 27):
    """Real tomography (``Utility.py:259-402``) of the rows of ``A`` for long
    vectors, optionally row-SHARDED: ``A`` is ``[r, m_local]``, this rank's
    slice of r vectors of global length ``n_global``; ``comm`` spans the
    ranks that hold the other slices.  Returns this rank's slice of the r
    estimates.

    Per checkpoint (N_t shots) and vector: magnitudes P_i = sqrt(c_i / N_t)
    with c ~ Multinomial(N_t, v^2); signs from plus ~ Multinomial(N_t,
    {((v_i + P_i)/2)^2} + remainder).  Both multinomials are split first over
    the ranks (their masses are all-gathered; every rank draws the same
    split), then over this rank's coordinates by :func:`multinomial_long`.
    With the reference's stopping rule the checkpoints are swept in chunks
    and a vector stops at its first checkpoint with ||v - est|| <= delta;
    without it only the last checkpoint is drawn (the reference returns that
    one, ``Utility.py:169-178``).  The draws of (vector, checkpoint) do not
    depend on the chunking.
    """
    from ..parallel.comm import Comm
    comm = comm if comm is not None else Comm(None)
    A = A.to(torch.float64)
    squeeze = A.ndim == 1
    if squeeze:
        A = A[None, :]
    r, m = A.shape
    dev = A.device
    d = int(n_global) if n_global is not None else m
    R, rank = comm.world_size, comm.rank
    nrm2 = comm.all_reduce_((A * A).sum(1))
    nrm = torch.sqrt(nrm2)
    close = torch.isclose(nrm, torch.ones_like(nrm), rtol=1e-2)
    V = torch.where(close[:, None], A, A / nrm.clamp(min=1e-300)[:, None]).contiguous()
    if N is None:
        N = int((36 * d * np.log(d)) / (delta ** 2)) if norm == "L2" else int((36 * np.log(d)) / (delta ** 2))
    if incremental_measure:
        sched = check_measure(np.geomspace(1, N, num=100, dtype=np.int64), faster_measure_increment)
    else:
        sched = np.array([int(N)], dtype=np.int64)
    T = len(sched)
    stop = incremental_measure and stop_when_reached_accuracy
    gpu = dev.type == "cuda"
    W1 = V * V
    S1 = torch.stack(comm.all_gather(W1.sum(1)), 0) if R > 1 else W1.sum(1)[None]   # [R, r]
    if not gpu:
        seed = int(key.k0) | (int(key.k1) << 32)
        rng_shared = np.random.default_rng([seed, int(key.stream) & 0xFFFFFFFF, 7])
        rng_local = np.random.default_rng([seed, int(key.stream) & 0xFFFFFFFF, 11, rank])

    def mnom(Nb, Wt, wr, sidb, level):
        if gpu:
            return multinomial_long(Nb, Wt, wr, key, sidb, level)
        rng = rng_shared if level in (4, 9) else rng_local   # top levels: same draw on every rank
        return torch.as_tensor(_multinomial_np(Nb.cpu().numpy(), Wt.cpu().numpy(),
                                               wr.cpu().numpy(), rng))

    out = torch.empty_like(V)
    active = list(range(r))
    t_list = list(range(T)) if stop else [T - 1]
    per = max(1, int(max_batch_elems) // max(m, 1))
    pos = 0
    while active and pos < len(t_list):
        ts = t_list[pos: pos + max(1, per // max(len(active), 1))]
        pos += len(ts)
        vec = torch.tensor([v for v in active for _ in ts], dtype=torch.int64, device=dev)
        tt = torch.tensor([t for _ in active for t in ts], dtype=torch.int64, device=dev)
        B = vec.numel()
        Nb = torch.as_tensor(sched, dtype=torch.float64, device=dev)[tt]
        sid = vec * T + tt
        ar = torch.arange(B, device=dev)
        # ---- round 1: magnitudes
        if R > 1:
            top = mnom(Nb, S1[:, vec].T.contiguous(), ar, sid, 4)
            Nloc = top[:, rank].to(dev)
        else:
            Nloc = Nb
        c1 = mnom(Nloc, W1, vec, sid, 0).to(dev)
        P = torch.sqrt(c1 / Nb[:, None])
        del c1
        Vb = V[vec]
        w2 = (0.5 * (Vb + P)) ** 2
        s2 = w2.sum(1)
        z = comm.all_reduce_(s2 + ((0.5 * (Vb - P)) ** 2).sum(1))
        S2 = torch.stack(comm.all_gather(s2), 1) if R > 1 else s2[:, None]          # [B, R]
        rem = (z - S2.sum(1)).clamp(min=0)
        top2 = mnom(Nb, torch.cat([S2, rem[:, None]], 1).contiguous(), ar, sid, 9)
        N2 = top2[:, rank].to(dev)
        # ---- round 2: signs
        c2 = mnom(N2, w2.contiguous(), ar, sid, 5).to(dev)
        est = torch.where(c2 > 0.4 * P * P * Nb[:, None], P, -P)
        del c2, w2
        if stop:
            diff = Vb - est
            if norm == "L2":
                err = torch.sqrt(comm.all_reduce_((diff * diff).sum(1)))
            else:
                err = comm.all_reduce_(diff.abs().amax(1), op="max")
            ok = (err <= float(delta)).cpu().numpy()
        else:
            ok = np.zeros(B, dtype=bool)
        vec_h = vec.cpu().numpy()
        tt_h = tt.cpu().numpy()
        done = set()
        for b in range(B):
            v = int(vec_h[b])
            if v in done:
                continue
            if ok[b] or int(tt_h[b]) == T - 1:
                out[v] = est[b]
                done.add(v)
        active = [v for v in active if v not in done]
    if preserve_norm:
        out = out * nrm[:, None]
    return out[0] if squeeze else out


def _tomography_rows_native(V, sched, delta, key: RngKey, norm, stop):
    """HIP path (csrc/tomography.hip): with the stop rule, one wave per row
    walks its checkpoints in order and keeps the first passing estimate
    (mode 2: only the checkpoints up to it are drawn); SQ_TOMO_ALLPAIRS=1:
    every checkpoint's error in one launch, then the chosen estimates
    regenerated (same Philox words, same result) in a second."""
    from ..ops import _native as nat
    r, d = V.shape
    T = len(sched)
    dev = V.device
    sch = torch.as_tensor(np.asarray(sched, dtype=np.int64), device=dev)
    err = torch.empty((r, T), dtype=torch.float64, device=dev)
    out = torch.empty((r, d), dtype=torch.float64, device=dev)
    st = nat.stream_handle(dev)
    ninf = 0 if norm == "L2" else 1
    m = nat.native()
    import os
    if stop and T > 1 and os.environ.get("SQ_TOMO_ALLPAIRS", "0") != "1":
        m.tomography(V.data_ptr(), r, d, sch.data_ptr(), T, 2, 0, 0, out.data_ptr(), ninf,
                     key.k0, key.k1, key.s0, key.s1, 0, st, float(delta))
        return out
    if stop and T > 1:
        m.tomography(V.data_ptr(), r, d, sch.data_ptr(), T, 0, 0, err.data_ptr(), 0, ninf,
                     key.k0, key.k1, key.s0, key.s1, 0, st)
        ok = err <= float(delta)
        first = torch.where(ok.any(1), ok.to(torch.int8).argmax(1),
                            torch.full((r,), T - 1, device=dev)).to(torch.int32).contiguous()
    else:
        first = torch.full((r,), T - 1, dtype=torch.int32, device=dev)
    m.tomography(V.data_ptr(), r, d, sch.data_ptr(), T, 1, first.data_ptr(), 0, out.data_ptr(),
                 ninf, key.k0, key.k1, key.s0, key.s1, 0, st)
    return out


def consistent_phase_estimation_device(omega, epsilon, gamma, key: RngKey, offset=0):
    """Consistent phase estimation (``Utility.py:740-792``) of every element
    of ``omega`` (float64 tensor, any device): one phase-estimation draw per
    element by ``csrc/qrand.hip: pe_batch_kernel`` (M = 2^m, m from
    delta' = eps C / 2 as in the reference), then the midpoint of the shifted
    eps-grid interval containing it, computed in closed form on the device
    (same values as the reference's ``bisect`` over ``np.arange``)."""
    from ..ops.random import phase_estimation_batch
    from .fejer import pe_qubits
    from .reference import _cpe_params
    omega = omega.to(torch.float64)
    _, dp, shift = _cpe_params(epsilon, gamma)
    m = int(pe_qubits(dp, gamma))
    pe = phase_estimation_batch(omega, torch.full(omega.shape, m, dtype=torch.int32,
                                                  device=omega.device), key, offset=offset)
    start = -1 - shift * dp
    stop = 1 + epsilon - shift * dp
    n_ar = int(np.ceil((stop - start) / epsilon))
    i = torch.floor((pe - start) / epsilon).to(torch.int64) + 1
    for _ in range(2):   # exact np.arange grid values are start + i eps
        i = torch.where((i > 0) & (start + (i - 1) * epsilon > pe), i - 1, i)
        i = torch.where((i < n_ar) & (start + i * epsilon <= pe), i + 1, i)
    i = i.clamp(1, n_ar)

    def val(t):
        return torch.where(t < n_ar, start + t.to(torch.float64) * epsilon,
                           torch.full_like(pe, stop))
    est = (val(i - 1) + val(i)) / 2
    return est.clamp(min=0.0)


def tomography(A, noise, key: RngKey, true_tomography=True, preserve_norm=False, **kw):
    """Device dispatcher with the reference's signature semantics."""
    if noise == 0:
        return A
    if not true_tomography:
        return gaussian_tomography(A, noise, key)
    return tomography_rows_torch(A, noise, key, preserve_norm=preserve_norm, **kw)
