"""Stochastic-layer ops with a HIP path on GPU
tensors and a torch path on CPU tensors; both draw from the same Philox
streams (``runtime/rng.py`` <-> ``csrc/common.h``) keyed by global element id.
"""

import math

import torch

from ..runtime.rng import Philox, RngKey, philox4x32, uniform_from_u32, MASK32
from ..quantum.fejer import WALK, SMALL_M
from . import _native as nat


def _key_args(key: RngKey):
    return key.k0, key.k1, key.s0, key.s1


# ------------------------------------------------------------ truncated normal
def trunc_normal_add_(x, bound, key: RngKey, offset=0):
    """In place ``x += TN(-bound, bound)`` (one draw per element, flat ids
    ``offset + i``).  Reference: ``Utility.py:68-104`` (truncnorm.rvs)."""
    if bound <= 0 or x.numel() == 0:
        return x
    if nat.use_native(x):
        assert x.is_contiguous() and x.dtype in (torch.float32, torch.float64)
        nat.native().trunc_normal_add(x.data_ptr(), nat.dtype_code(x), x.numel(), float(bound),
                                      *_key_args(key), int(offset), nat.stream_handle(x.device))
        return x
    u = Philox(key).uniform_flat(x.numel(), offset=offset, device=x.device, dtype=torch.float64)
    e = math.erf(bound / math.sqrt(2.0))
    z = math.sqrt(2.0) * torch.erfinv((2.0 * u - 1.0) * e)
    z = z.clamp_(-bound, bound)
    x.view(-1).add_(z.to(x.dtype))
    return x


def philox_normal(shape, key: RngKey, mean=0.0, std=1.0, dtype=torch.float32, device="cpu",
                  offset=0):
    """Tensor of ``mean + std * N(0,1)`` keyed by flat element ids."""
    device = torch.device(device)
    n = 1
    for s in shape:
        n *= int(s)
    if device.type == "cuda":
        out = torch.empty(shape, dtype=dtype, device=device)
        nat.native().philox_normal(out.data_ptr(), nat.dtype_code(out), n, float(mean), float(std),
                                   *_key_args(key), int(offset), nat.stream_handle(device))
        return out
    z = Philox(key).normal_flat(n, offset=offset, device=device, dtype=torch.float64)
    return (mean + std * z).to(dtype).reshape(shape)


def philox_uniform(shape, key: RngKey, device="cpu", offset=0):
    device = torch.device(device)
    n = 1
    for s in shape:
        n *= int(s)
    if device.type == "cuda":
        out = torch.empty(shape, dtype=torch.float32, device=device)
        nat.native().philox_uniform(out.data_ptr(), n, *_key_args(key), int(offset),
                                    nat.stream_handle(device))
        return out
    return Philox(key).uniform_flat(n, offset=offset, device=device).reshape(shape)


# ------------------------------------------------------------ Fejer samplers
def _ws_words(key: RngKey, s, w):
    """Word ``w`` of the per-sample word stream of sample ids ``s`` (int64)."""
    blk = w // 4
    c0 = s & MASK32
    c1 = ((s >> 32) & 0xFFFF) | (blk << 16)
    x = philox4x32(c0, c1, key.s0, key.s1, key.k0, key.k1)
    sel = w % 4
    return torch.where(sel == 0, x[0], torch.where(sel == 1, x[1], torch.where(sel == 2, x[2], x[3])))


def _u_ws(key, s, w):
    return uniform_from_u32(_ws_words(key, s, torch.as_tensor(w, dtype=torch.int64)), torch.float64)


def fejer_sample_torch(omega, M, key: RngKey, sample_ids):
    """torch twin of ``csrc/fejer.h::fejer_sample`` (CPU path)."""
    omega = omega.to(torch.float64)
    M = M.to(torch.int64)
    s_ids = sample_ids.to(torch.int64)
    Md = M.to(torch.float64)
    fl = torch.floor(omega)
    phi = omega - fl
    base = fl.to(torch.int64)
    out = torch.empty_like(base)
    w = torch.zeros_like(s_ids)
    u0 = _u_ws(key, s_ids, w)
    sval = torch.sin(math.pi * phi) ** 2

    exact = phi == 0
    small = (~exact) & (M <= SMALL_M)
    big = (~exact) & (M > SMALL_M)
    out[exact] = torch.remainder(base[exact], M[exact])
    if small.any():
        idx = torch.nonzero(small).reshape(-1)
        for i in idx.tolist():
            Mi = int(M[i])
            j = torch.arange(Mi, dtype=torch.float64)
            sn = torch.sin(math.pi * (j - omega[i]) / Mi)
            p = torch.where(sn == 0, torch.ones_like(sn), sval[i] / (Mi * Mi * sn * sn))
            cdf = torch.cumsum(p, 0)
            u = u0[i] * cdf[-1]
            k = int((cdf < u).sum())
            out[i] = min(k, Mi - 1)
    if big.any():
        idx = torch.nonzero(big).reshape(-1)
        ph = phi[idx]
        Mb = Md[idx]
        offs = [0]
        for t in range(1, WALK + 1):
            offs += [t, -t]
        offs_t = torch.tensor(offs, dtype=torch.float64)
        x = offs_t[None, :] - ph[:, None]
        den = torch.sin(math.pi * x / Mb[:, None])
        p = sval[idx][:, None] / (Mb[:, None] ** 2 * den ** 2)
        cdf = torch.cumsum(p, 1)
        k = (cdf < u0[idx][:, None]).sum(1)
        ell = torch.where(k < len(offs), offs_t[k.clamp(max=len(offs) - 1)].to(torch.int64),
                          torch.zeros_like(k))
        tail = k >= len(offs)
        if tail.any():
            ti = torch.nonzero(tail).reshape(-1)
            ell[ti] = _tail_torch(ph[ti], Mb[ti], key, s_ids[idx][ti])
        out[idx] = torch.remainder(base[idx] + ell, M[idx])
    return out


def _tail_torch(phi, M, key, s_ids):
    n = phi.shape[0]
    res = torch.zeros(n, dtype=torch.int64)
    lR = torch.floor(phi + M / 2.0)
    lL = lR - M + 1.0
    zR0 = WALK + 1 - phi
    nR = torch.clamp(lR - WALK, min=0.0)
    zL0 = WALK + 1 + phi
    nL = torch.clamp(-WALK - lL, min=0.0)
    SR = torch.where(nR > 0, 1.0 / (zR0 - 0.5) - 1.0 / (zR0 + nR - 0.5), torch.zeros_like(nR))
    SL = torch.where(nL > 0, 1.0 / (zL0 - 0.5) - 1.0 / (zL0 + nL - 0.5), torch.zeros_like(nL))
    pending = torch.ones(n, dtype=torch.bool)
    for it in range(4096):
        if not pending.any():
            break
        w0 = 1 + 3 * it
        us = _u_ws(key, s_ids, w0)
        right = us * (SR + SL) < SR
        z0 = torch.where(right, zR0, zL0)
        S = torch.where(right, SR, SL)
        cnt = torch.where(right, nR, nL)
        R = 1.0 / (z0 - 0.5) - _u_ws(key, s_ids, w0 + 1) * S
        i = torch.ceil(1.0 / R - 0.5 - z0)
        i = torch.minimum(torch.clamp(i, min=0.0), torch.clamp(cnt - 1.0, min=0.0))
        z = z0 + i
        acc = 4.0 * (z * z - 0.25) / (M * M * torch.sin(math.pi * z / M) ** 2)
        ok = pending & (_u_ws(key, s_ids, w0 + 2) < acc)
        ell = torch.where(right, torch.round(z + phi), torch.round(phi - z)).to(torch.int64)
        res = torch.where(ok, ell, res)
        pending = pending & ~ok
    return res


def ae_bins_torch(eps):
    return torch.ceil((math.pi / (2 * eps)) * (1 + torch.sqrt(1 + 4 * eps))).to(torch.int64)


def amplitude_estimation_batch(a, eps, key: RngKey, Q=1, offset=0):
    """Median-of-Q amplitude estimation of every element of ``a`` (float64).

    Sample id of repetition q of element i is (offset+i)*Q + q - the same
    mapping as ``csrc/qrand.hip::ae_batch_kernel``.
    """
    a = a.to(torch.float64).contiguous()
    eps = torch.broadcast_to(eps.to(torch.float64), a.shape).contiguous()
    if nat.use_native(a):
        out = torch.empty_like(a)
        nat.native().ae_batch(a.data_ptr(), eps.data_ptr(), out.data_ptr(), a.numel(), int(Q),
                              *_key_args(key), int(offset), nat.stream_handle(a.device))
        return out
    flat_a = a.reshape(-1)
    M = ae_bins_torch(eps.reshape(-1))
    omega = M.to(torch.float64) * torch.asin(torch.sqrt(flat_a.clamp(0, 1))) / math.pi
    base = (torch.arange(flat_a.numel(), dtype=torch.int64) + offset) * Q
    reps = []
    for q in range(Q):
        j = fejer_sample_torch(omega, M, key, base + q)
        reps.append(torch.sin(math.pi * j.to(torch.float64) / M.to(torch.float64)) ** 2)
    st = torch.stack(reps, 0)
    res = st[0] if Q == 1 else torch.sort(st, 0).values[Q // 2] if Q % 2 == 1 else torch.median(st, 0).values
    return res.reshape(a.shape)


def phase_estimation_batch(omega, m, key: RngKey, offset=0):
    """k/M samples, M = 2^m (per element), centred at omega in [0,1)."""
    omega = omega.to(torch.float64).contiguous()
    m = torch.broadcast_to(m.to(torch.int32), omega.shape).contiguous()
    if nat.use_native(omega):
        out = torch.empty_like(omega)
        nat.native().pe_batch(omega.data_ptr(), m.data_ptr(), out.data_ptr(), omega.numel(),
                              *_key_args(key), int(offset), nat.stream_handle(omega.device))
        return out
    flat = omega.reshape(-1)
    M = torch.pow(2, m.reshape(-1).to(torch.int64))
    ids = torch.arange(flat.numel(), dtype=torch.int64) + offset
    k = fejer_sample_torch(M.to(torch.float64) * flat, M, key, ids)
    out = k.to(torch.float64) / M.to(torch.float64)
    near1 = (flat == 1) | torch.isclose(flat, torch.ones_like(flat))
    out = torch.where(near1, (M - 1).to(torch.float64) / M.to(torch.float64), out)
    return out.reshape(omega.shape)
