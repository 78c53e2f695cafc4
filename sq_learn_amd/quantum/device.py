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
"""

import math

import numpy as np
import torch

from ..runtime.rng import RngKey
from .reference import check_measure


def gaussian_tomography(A, noise, key: RngKey, offset=0):
    """A + TN(+-noise/sqrt(A.numel())) per component (Frobenius budget)."""
    from ..ops.random import trunc_normal_add_
    if noise == 0:
        return A
    out = A.clone() if A.dtype in (torch.float32, torch.float64) else A.float()
    out = out.contiguous()
    b = float(noise) / math.sqrt(out.numel())
    trunc_normal_add_(out.view(-1), b, key, offset=offset)
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


def _tomography_rows_native(V, sched, delta, key: RngKey, norm, stop):
    """HIP path (csrc/tomography.hip): errors of every checkpoint in one
    launch, first passing checkpoint per row on the device, then the chosen
    estimates regenerated (same Philox words) in a second launch."""
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


def tomography(A, noise, key: RngKey, true_tomography=True, preserve_norm=False, **kw):
    """Device dispatcher with the reference's signature semantics."""
    if noise == 0:
        return A
    if not true_tomography:
        return gaussian_tomography(A, noise, key)
    return tomography_rows_torch(A, noise, key, preserve_norm=preserve_norm, **kw)
