"""q-means / k-means ops: fused E-step, delta-band selection, segmented
centroid reduction, centroid finalisation and the IPE distance path.

GPU tensors run the HIP kernels of ``csrc/kmeans.hip``; CPU tensors run the
torch twins below, which implement the same semantics and draw the same
Philox keys (reference ``_dmeans.py:732-830``).
"""

import math
import os

import numpy as np

import torch

from ..runtime.rng import RngKey, philox4x32, MASK32
from . import _native as nat
from .random import amplitude_estimation_batch

FAST_D = (16, 32, 64, 128, 256)
# d_pad of the certified filter (csrc/estep_f32.hip estep_x64_kernel): the
# power-of-two ladder to 256, then steps of 128 to 1024 (sub-staged tiles)
X64_D = FAST_D + (384, 512, 640, 768, 896, 1024)
X64_MAX_K = 16384   # k_pad of the filter (the segmented reduce's LDS histogram)
BIG = 3.0e38


def pad_features(d):
    """Padded feature count used by the MFMA kernels (zero columns)."""
    for f in X64_D:
        if d <= f:
            return f
    return ((d + 15) // 16) * 16


def pad_clusters(k):
    return ((k + 63) // 64) * 64


def idx_bits(k_pad):
    b = 1
    while (1 << b) < k_pad:
        b += 1
    return b


def band_keys(key: RngKey, grows, cols, k_pad):
    """Selection key of (global row, centroid): philox word of block
    (row << 16 | j), low idx_bits replaced by j (same as band_key() in HIP)."""
    ib = idx_bits(k_pad)
    keep = MASK32 & ~((1 << ib) - 1)
    idx = (grows.to(torch.int64) << 16) | cols.to(torch.int64)
    w = philox4x32(idx & MASK32, (idx >> 32) & MASK32, key.s0, key.s1, key.k0, key.k1)[0]
    return (w & keep) | cols.to(torch.int64)


def band_u(key: RngKey, grows):
    """Per-row uniform of the band rule: u01(Philox word g) (fp32, exact twin
    of ``band_u`` in csrc/kmeans.hip)."""
    g = grows.to(torch.int64)
    w = philox4x32((g >> 2) & MASK32, (g >> 34) & MASK32, key.s0, key.s1, key.k0, key.k1)
    word = torch.stack(w, 1).gather(1, (g & 3)[:, None])[:, 0]
    return ((word >> 8).to(torch.float32) + 0.5) * (1.0 / 16777216.0)


def band_select_torch(D, grows, delta, key: RngKey, k_pad, tie_only=False):
    """Exact delta-band selection over distance rows D [m, k] (torch twin of
    the HIP kernels; csrc/kmeans.hip ``band_pick_wave``).

    members M = {j : D_j <= min + delta}; ordered by kappa(j) = (j mod 32,
    j div 32); label = member of rank floor(u * |M|) with one Philox uniform
    per row -> a uniform choice among the qualifying indices, like the
    reference's ``random.choice`` (``_dmeans.py:742-751, 771-772``)."""
    if tie_only:
        return _band_select_minkey_torch(D, grows, delta, key, k_pad, tie_only=True)
    mn, am = torch.min(D, dim=1)
    thr = mn + float(delta)
    cand = D <= thr[:, None]
    cnt = cand.sum(1)
    labels = am.clone()
    multi = torch.nonzero(cnt > 1).reshape(-1)
    if multi.numel():
        k = D.shape[1]
        j = torch.arange(k, dtype=torch.int64, device=D.device)
        kappa = ((j & 31) << 20) | (j >> 5)
        sub = cand[multi]
        kap = torch.where(sub, kappa[None, :], torch.full_like(kappa, 1 << 40)[None, :])
        srt = torch.sort(kap, dim=1).values
        c = cnt[multi]
        u = band_u(key, grows[multi].to(D.device))
        r = torch.floor(u * c.to(torch.float32)).to(torch.int64)
        r = torch.minimum(r, c - 1)
        ch = srt.gather(1, r[:, None])[:, 0]
        labels[multi] = ((ch & 0xFFFFF) << 5) | (ch >> 20)
    return labels, mn


def _band_select_minkey_torch(D, grows, delta, key: RngKey, k_pad, tie_only=False):
    """Tie-break by the smallest per-(row, centroid) Philox key (the IPE
    kernel's rule, ``ipe_estep_kernel``)."""
    mn, am = torch.min(D, dim=1)
    thr = mn + (0.0 if tie_only else float(delta))
    cand = D <= thr[:, None]
    cnt = cand.sum(1)
    labels = am.clone()
    multi = torch.nonzero(cnt > 1).reshape(-1)
    if multi.numel():
        sub = cand[multi]
        rr, cc = torch.nonzero(sub, as_tuple=True)
        keys = band_keys(key, grows[multi][rr], cc, k_pad)
        best = torch.full((multi.numel(),), 1 << 40, dtype=torch.int64, device=D.device)
        best = best.scatter_reduce(0, rr, keys, reduce="amin")
        ib = idx_bits(k_pad)
        labels[multi] = best & ((1 << ib) - 1)
    return labels, mn


def distances_torch(X, C, xn=None, cn=None):
    """Squared euclidean distances ||x||^2 + ||c||^2 - 2 x.c, clamped >= 0."""
    if xn is None:
        xn = (X * X).sum(1)
    if cn is None:
        cn = (C * C).sum(1)
    D = xn[:, None] + cn[None, :] - 2.0 * (X @ C.T)
    return D.clamp_(min=0.0)


def estep_torch(X, C, delta, key, row_offset, k_pad, chunk_rows=65536, xn=None):
    """CPU E-step (labels, min distances) over row chunks."""
    n = X.shape[0]
    labels = torch.empty(n, dtype=torch.int64, device=X.device)
    mind = torch.empty(n, dtype=X.dtype, device=X.device)
    cn = (C * C).sum(1)
    for s in range(0, n, chunk_rows):
        e = min(n, s + chunk_rows)
        xb = X[s:e]
        xnb = (xb * xb).sum(1) if xn is None else xn[s:e]
        D = distances_torch(xb, C, xnb, cn)
        g = torch.arange(s, e, dtype=torch.int64, device=X.device) + row_offset
        lab, mn = band_select_torch(D, g, delta, key, k_pad)
        labels[s:e] = lab
        mind[s:e] = mn
    return labels, mind


def ipe_estep_torch(X, C, eps, key, row_offset, k_pad, Q=13, chunk_rows=256):
    """CPU IPE E-step: D~ = |x|^2 + |c|^2 - 2 IPE(x, c) (``_dmeans.py:753-772``)."""
    n, k = X.shape[0], C.shape[0]
    labels = torch.empty(n, dtype=torch.int64)
    mind = torch.empty(n, dtype=torch.float64)
    cn = (C.double() ** 2).sum(1)
    for s in range(0, n, chunk_rows):
        e = min(n, s + chunk_rows)
        xb = X[s:e].double()
        xn = (xb * xb).sum(1)
        G = xb @ C.double().T
        S = xn[:, None] + cn[None, :]
        a = (S - 2 * G) / (2 * S)
        a = torch.where(a.abs() <= 1e-15, torch.zeros_like(a), a)
        eps_a = eps * torch.clamp(G.abs(), min=1.0) / S
        at = amplitude_estimation_batch(a.clamp(0, 1), eps_a, key, Q=Q,
                                        offset=(row_offset + s) * k)
        sv = S * (1 - 2 * at) / 2
        Dt = xn[:, None] + cn[None, :] - 2 * sv
        g = torch.arange(s, e, dtype=torch.int64) + row_offset
        lab, mn = band_select_torch(Dt, g, 0.0, key, k_pad, tie_only=True)
        labels[s:e] = lab
        mind[s:e] = mn
    return labels, mind


# ----------------------------------------------------------------- native
class EStepBuffers:
    """Device workspace of the fused E-step (allocated once per fit)."""

    def __init__(self, n, device, ovf_cap=None):
        self.labels = torch.empty(n, dtype=torch.int32, device=device)
        self.mind = torch.empty(n, dtype=torch.float32, device=device)
        # every row may overflow (wide bands): the list holds all n rows, so no
        # row is ever dropped; the fallback kernel strides over the live count
        self.ovf_cap = int(ovf_cap if ovf_cap is not None else max(n, 1))
        self.ovf_rows = torch.empty(self.ovf_cap, dtype=torch.int64, device=device)
        self.ovf_thr = torch.empty(self.ovf_cap, dtype=torch.float32, device=device)
        # (int32; ovf_count is a view of slot 0)
        # [3-pass overflow rows, dense rows, multi rows, kept rows (filter),
        #  list-B rows resolved by the gap screen, list-B rows (filter),
        #  overflow rows of the second (3 members per lane) 3-pass,
        #  the filter's own multi-list rows (the list's head)]
        self.counts = torch.zeros(8, dtype=torch.int32, device=device)
        self.ovf2_rows = None
        self.exact_flag = None   # the fp32 screen's hand-off flags (per multi entry)
        self.ovf_count = self.counts[0:1]
        self.dense_rows = None   # allocated by the certified E-step on first use
        self.multi_rows = None   # certified E-step: rows sent to the fp64 re-check kernel
        self.multi_cand = None   # ... and their candidate lists [n][1 + 16], by ROW
        # Hamerly pruning: 1 for the rows whose candidate list (kept per row in
        # multi_cand) is current, 0 otherwise
        self.mflag = None
        # per-row (min distance - distance to the label) of the rows whose
        # label is not their argmin (fp64 re-check / dense / overflow rows):
        # the incremental M-step's inertia correction; None = not produced
        self.corr = None
        # True while ovf_count is known to be zero (fresh, or reset on the
        # device by the iteration-scalars launch): the E-step skips its memset
        self.ovf_clean = True
        self.inertia = torch.zeros(1, dtype=torch.float64, device=device)
        # per-wave inertia partials (summed in a fixed order: reproducible)
        self.part_cap = n // 32 + 64
        self.inertia_part = torch.zeros(self.part_cap, dtype=torch.float64, device=device)


def estep_native(Xb, C_bf16, cn, xn, k, delta, key: RngKey, row_offset, buf: EStepBuffers,
                 stream=None):
    """Fused MFMA E-step + device-driven overflow fallback (no host sync)."""
    n, d_pad = Xb.shape
    k_pad = C_bf16.shape[0] * 64
    assert Xb.dtype == torch.bfloat16 and C_bf16.dtype == torch.bfloat16
    assert tuple(C_bf16.shape[1:]) == (d_pad // 8 + 2, 64, 8) and d_pad in FAST_D
    assert Xb.is_contiguous() and C_bf16.is_contiguous() and cn.is_contiguous()
    assert buf.labels.numel() >= n and buf.part_cap >= 8
    st = stream if stream is not None else nat.stream_handle(Xb.device)
    m = nat.native()
    if not buf.ovf_clean:
        buf.ovf_count.zero_()
    buf.ovf_clean = False
    m.estep_bf16(Xb.data_ptr(), C_bf16.data_ptr(), buf.inertia_part.data_ptr(), buf.ovf_thr.data_ptr(),
                 xn.data_ptr(), buf.labels.data_ptr(), buf.mind.data_ptr(), buf.ovf_rows.data_ptr(),
                 buf.ovf_count.data_ptr(), buf.inertia.data_ptr(), n, d_pad, k, k_pad,
                 float(delta), int(buf.part_cap), key.k0, key.k1, key.s0, key.s1, int(row_offset),
                 buf.ovf_cap, st)
    m.band_select_rows(Xb.data_ptr(), C_bf16.data_ptr(), buf.ovf_thr.data_ptr(), xn.data_ptr(),
                       buf.ovf_rows.data_ptr(), buf.ovf_count.data_ptr(), buf.labels.data_ptr(),
                       buf.ovf_cap, d_pad, k, k_pad, float(delta), key.k0, key.k1, key.s0, key.s1,
                       int(row_offset), st)
    return buf.labels, buf.mind


def band_select_native(D, xn, delta, key: RngKey, row_offset, labels, mind, k=None, rows=None):
    """Exact selection over fp32 distance rows on the GPU (generic path)."""
    D = D.contiguous()
    m_, kk = D.shape
    k = kk if k is None else k
    nat.native().band_select(D.data_ptr(), 0 if rows is None else rows.data_ptr(),
                             0 if xn is None else xn.data_ptr(), labels.data_ptr(), mind.data_ptr(),
                             m_, k, D.stride(0), float(delta), key.k0, key.k1, key.s0, key.s1,
                             int(row_offset), nat.stream_handle(D.device))


def ipe_estep_native(G, xn, cn, eps, Q, key: RngKey, row_offset, labels, mind):
    G = G.contiguous()
    m_, k = G.shape
    nat.native().ipe_estep(G.data_ptr(), xn.data_ptr(), cn.data_ptr(), labels.data_ptr(),
                           mind.data_ptr(), m_, k, G.stride(0), float(eps), int(Q), key.k0, key.k1,
                           key.s0, key.s1, int(row_offset), nat.stream_handle(G.device))


def ipe_center_fragments(C, k_pad, d_pad):
    """Centroids as 16x16x4 f32 MFMA B fragments (csrc/ipe.hip): tile t,
    k-step s, lane l -> C[16 t + (l & 15)][4 s + (l >> 4)], zero padded."""
    k, d = C.shape
    Cp = torch.zeros((k_pad, d_pad), dtype=torch.float32, device=C.device)
    Cp[:k, :d] = C.float()
    return Cp.view(k_pad // 16, 16, d_pad // 4, 4).permute(0, 2, 3, 1).contiguous()


def ipe_fused_native(X, Cfrag, xn, cn, k, k_pad, d_pad, eps, Q, key: RngKey, tie_key: RngKey,
                     row_offset, labels, mind, prune=True, C=None, hint_labels=None,
                     skip_key: RngKey = None, stats=None, layout=0, rows=None, ext=None):
    """Fused IPE E-step (csrc/ipe.hip): exact fp32 MFMA inner products, the
    median-of-Q amplitude-estimation distance per pair in the epilogue,
    per-row argmin with random ties; G is never materialised.  ``prune``
    (odd Q): each row's hint pair is sampled first - ``hint_labels[row]``
    (int32, e.g. the previous iteration's labels; needs the plain fp32
    centroids ``C``) when valid, else the exact fp32 distance argmin of a
    first MFMA sweep - and its estimate is the row's threshold; every other
    pair is screened by its fp32 hazard against that threshold, spending an
    Exp(1) budget per (row, lane) stream keyed by ``skip_key``; only pairs
    whose budget runs out (thinned to the exact law) or that are competitive
    pay a sampler - same law as prune=False.  ``stats`` (int64[5], optional,
    accumulated): screened pairs, full-sampler pairs, fires, fires reaching
    the exact branch, workgroups that ran the first sweep.  ``layout``
    (tests): 0 auto, 1 / 2 row groups per workgroup, 3 the per-lane-queue
    kernel - all return the same labels bit for bit.  ``rows`` = (rlist
    int64, rcount int32 [1] on the device, list_n >= count on the host) with
    ``ext`` = (thr fp32 [n], hj int32 [n]): list mode over the listed rows,
    with their thresholds / hints given (the dense rows of ``Ipe16``)."""
    n, d = X.shape
    assert X.dtype == torch.float32 and X.stride(1) == 1
    assert xn.dtype == torch.float32 and cn.dtype == torch.float32 and xn.numel() >= n
    assert Cfrag.numel() == k_pad * d_pad and labels.dtype == torch.int32
    if hint_labels is not None:
        assert C is not None and C.dtype == torch.float32 and C.is_contiguous()
        assert tuple(C.shape) == (k, d) and hint_labels.dtype == torch.int32
        assert hint_labels.numel() >= n
    if stats is not None:
        assert stats.dtype == torch.int64 and stats.numel() >= 5 and stats.is_contiguous()
    if skip_key is None:
        skip_key = key.derive(purpose="ipe_skip")
    # the row-group layouts turn label hints into thresholds in a pre-pass
    scratch = None
    if rows is not None:
        assert ext is not None and prune and int(Q) % 2 == 1
        rl, rc, ln = rows
        assert rl.dtype == torch.int64 and rc.dtype == torch.int32
        assert ext[0].dtype == torch.float32 and ext[1].dtype == torch.int32
    elif hint_labels is not None and prune and int(Q) % 2 == 1 and layout != 3:
        scratch = torch.empty(2 * max(n, 1), dtype=torch.int32, device=X.device)
    rc = nat.native().ipe_fused(X.data_ptr(), X.stride(0), Cfrag.data_ptr(),
                                0 if C is None else C.data_ptr(),
                                0 if hint_labels is None else hint_labels.data_ptr(),
                                xn.data_ptr(), cn.data_ptr(), labels.data_ptr(), mind.data_ptr(), n,
                                d, d_pad, k, k_pad, float(eps), int(Q), key.k0, key.k1, key.s0,
                                key.s1, tie_key.k0, tie_key.k1, tie_key.s0, tie_key.s1,
                                skip_key.k0, skip_key.k1, skip_key.s0, skip_key.s1,
                                int(row_offset), int(bool(prune)) | (int(layout) & 3) << 1,
                                0 if stats is None else stats.data_ptr(),
                                0 if scratch is None else scratch.data_ptr(),
                                nat.stream_handle(X.device),
                                *((rows[0].data_ptr(), rows[1].data_ptr(), int(rows[2]),
                                   ext[0].data_ptr(), ext[1].data_ptr()) if rows is not None
                                  else ()))
    if rc:
        raise RuntimeError(f"ipe_fused failed (hip error {rc})")


def centroid_accumulate_native(X, labels, weights, sums, counts, k, chunk=None):
    n, d = X.shape
    if chunk is None:
        chunk = max(256, min(8192, (160 * 1024 // 4) - 2 * k - 64))
        chunk = min(chunk, 8192)
    assert labels.dtype == torch.int32 and sums.dtype == torch.float32 and counts.dtype == torch.float64
    nat.native().centroid_accumulate(X.data_ptr(), nat.dtype_code(X), labels.data_ptr(),
                                     0 if weights is None else weights.data_ptr(), sums.data_ptr(),
                                     counts.data_ptr(), n, d, k, int(chunk),
                                     nat.stream_handle(X.device))


def fixed_point_exp(max_abs, n_rows):
    """Exponent e of the 2^e quantum of the deterministic segmented sums:
    the smallest power of two with max|x| * n / 2^e <= 2^52, so every sum
    is an integer multiple of 2^e below 2^53 quanta (exact in fp64 in any
    addition order); clamped to the kernel's range."""
    bound = float(max_abs) * max(int(n_rows), 1)
    if not math.isfinite(bound):
        raise ValueError("non-finite values in the data: cannot reduce centroids")
    if bound <= 0.0:
        return -120
    e = math.ceil(math.log2(bound)) - 52
    return int(min(max(e, -120), 120))


class ReduceWorkspace:
    """Counting-sort workspace of the segmented centroid reduction, plus the
    fixed-point exponents (``xexp`` for the data, ``wexp`` for the weights;
    0 when unweighted, counts then being exact integers)."""

    def __init__(self, n, k, device, xexp=-30, wexp=0):
        self.hist = torch.zeros(k, dtype=torch.int32, device=device)
        self.cursor = torch.zeros(k, dtype=torch.int32, device=device)
        self.perm = torch.empty(max(n, 1), dtype=torch.int32, device=device)
        self.xexp = int(xexp)
        self.wexp = int(wexp)

    def set_scale(self, max_abs_x, n_rows, max_w=None):
        self.xexp = fixed_point_exp(max_abs_x * (max_w if max_w is not None else 1.0), n_rows)
        self.wexp = 0 if max_w is None else fixed_point_exp(max_w, n_rows)
        return self


def centroid_reduce_native(X, labels, weights, sums, counts, k, ws: ReduceWorkspace, mind=None,
                           C_old=None):
    """sums[l] = sum_{i: label_i = l} w_i x_i, counts[l] = sum w_i (GPU; the
    outputs are overwritten - zeroed inside the histogram launch),
    in units of the quanta 2^ws.xexp / 2^ws.wexp (exact integer-valued fp64,
    order-independent: bit-reproducible).  ``pack_stats_native`` rescales."""
    n, d = X.shape
    assert labels.dtype == torch.int32 and sums.dtype == torch.float64 and counts.dtype == torch.float64
    assert sums.numel() >= k * d and counts.numel() >= k and labels.numel() >= n
    if mind is not None:
        # rows with mind < 0 get |x - C_old[label]|^2 (fp64) from the row pass
        assert X.dtype == torch.float32 and C_old.dtype == torch.float32
        assert tuple(C_old.shape) == (k, d) and C_old.is_contiguous() and d <= 256
    nat.native().centroid_reduce(X.data_ptr(), nat.dtype_code(X), labels.data_ptr(),
                                 0 if weights is None else weights.data_ptr(), sums.data_ptr(),
                                 counts.data_ptr(), n, d, k, ws.xexp,
                                 ws.wexp if weights is not None else 0, ws.hist.data_ptr(),
                                 ws.cursor.data_ptr(), ws.perm.data_ptr(), nat.ptr(mind),
                                 nat.ptr(C_old), nat.stream_handle(X.device))


def bounds_filter_native(labels, ub, lb, shift, smax, delta, rlist, rcount, buf: EStepBuffers,
                         cc=None, nf=0, fidx=None):
    """Hamerly pruning (csrc/estep_f32.hip bounds_filter_kernel): bounds
    moved by the centroid shifts; rows that can no longer be proven to keep
    their candidate set go to ``rlist`` (count in ``rcount``, on the device);
    pruned multi-candidate rows are appended to ``buf``'s multi list (their
    per-row candidate lists stay valid) for the fp64 re-check.
    ``buf.counts`` and ``rcount`` must be zeroed before (the counts
    accumulate; the E-step keeps rcount in ``buf.counts[3]``, so one fill
    clears both).
    ``cc`` [k nf + k] fp32 / ``nf``: the fastest centroids' Elkan distances
    (:func:`fast_centroids_native`; ``smax`` then excludes them).  The
    pass also zeroes ``buf.corr`` (the list-mode E-step that follows skips
    its memset)."""
    n = labels.numel()
    assert ub.dtype == torch.float32 and lb.dtype == torch.float32 and rlist.numel() >= n
    assert shift.dtype == torch.float64 and smax.dtype == torch.float64
    assert buf.mflag is not None and buf.mflag.numel() >= n
    rc = nat.native().bounds_filter(labels.data_ptr(), ub.data_ptr(), lb.data_ptr(),
                                    shift.data_ptr(), smax.data_ptr(), n, float(delta),
                                    rlist.data_ptr(), rcount.data_ptr(), buf.mflag.data_ptr(),
                                    buf.multi_rows.data_ptr(), buf.counts[2:3].data_ptr(),
                                    0 if cc is None else cc.data_ptr(),
                                    0 if cc is None else fidx.data_ptr(),
                                    int(nf if cc is not None else 0), int(shift.numel()),
                                    nat.stream_handle(labels.device),
                                    0 if buf.corr is None else buf.corr.data_ptr(),
                                    buf.counts[7:8].data_ptr())
    if rc:
        raise RuntimeError(f"bounds_filter failed (hip error {rc})")


def fast_centroids_native(shift, C, nf, idx, smax_rest, cc, shift_sq=None):
    """The nf fastest centroids of an update (top-nf shifts) -> ``idx``,
    ``smax_rest`` = the largest shift outside them, ``cc[j][f]`` = |c_j -
    c_idx[f]| rounded down (+inf on j = idx[f]), ``cc[k nf + j]`` = min_f
    cc[j][f]; csrc/estep_f32.hip.  With ``shift_sq`` (the squared
    per-centroid shifts) ``shift`` is first written as sqrt(shift_sq) (1 +
    1e-12) in the same launch."""
    k, d = C.shape
    assert C.dtype == torch.float32 and C.is_contiguous() and shift.dtype == torch.float64
    assert 0 <= nf < k and idx.numel() >= nf and cc.numel() >= k * (nf + 1)
    assert shift.numel() >= k and shift.is_contiguous()
    if shift_sq is not None:
        assert shift_sq.dtype == torch.float64 and shift_sq.is_contiguous() and shift_sq.numel() >= k
    rc = nat.native().fast_centroids(shift.data_ptr(),
                                     0 if shift_sq is None else shift_sq.data_ptr(), C.data_ptr(),
                                     k, d, int(nf), idx.data_ptr(), smax_rest.data_ptr(),
                                     cc.data_ptr(), nat.stream_handle(C.device))
    if rc:
        raise RuntimeError(f"fast_centroids failed (hip error {rc})")


def multi_records(rec=None, mflag=None, it_now=0, it_lo=0, dsh=None, dq=None, rows_b=None,
                  count_b=None, n_done=None):
    """Set (or clear, rec=None) the gap records used by this thread's next
    certified E-steps (csrc/estep_f32.hip): the fp32 screen writes a row's
    record with base ``it_now`` (mflag = 2 + base), the bounds filter lists
    rows whose base is in [it_lo, it_now - 1] in ``rows_b`` / ``count_b``,
    the gap screen moves their records by the shift operand of their base
    (``dsh`` [ring][k][d_pad] fp16 / ``dq`` [ring][k][8], slot base % ring)."""
    if rec is None:
        nat.native().multi_records(0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0)
        return
    assert rec.dtype == torch.float32 and rec.shape[-1] == 8 and mflag.dtype == torch.int32
    assert dsh.dtype == torch.float16 and dq.dtype == torch.float32 and rows_b.dtype == torch.int64
    assert dsh.dim() == 3 and dq.shape[:2] == dsh.shape[:2] and dq.shape[2] == 8
    rc = nat.native().multi_records(rec.data_ptr(), mflag.data_ptr(), int(it_now), int(it_lo),
                                    int(dsh.shape[0]), dsh.data_ptr(), dq.data_ptr(),
                                    int(dsh.stride(0)), rows_b.data_ptr(), count_b.data_ptr(),
                                    0 if n_done is None else n_done.data_ptr())
    if rc:
        raise RuntimeError(f"multi_records failed (hip error {rc})")


def shift_operand_native(C_prev, C_new, alpha, snap, dsh, dq, snew, valid):
    """The gap screen's shift operands of the update C_prev -> C_new (fp32
    [k][d], same layout) for the ring slots in the bitmask ``valid``: slot
    ``snew`` against C_prev (which it snapshots into ``snap[snew]``), the
    others against their snapshots (``snap`` [ring][k][d_pad] fp32)."""
    k, d = C_new.shape[0], C_new.shape[1]
    ring, _, d_pad = dsh.shape
    assert C_prev.dtype == torch.float32 and C_new.dtype == torch.float32
    assert C_prev.stride() == C_new.stride() and C_new.stride(1) == 1
    assert tuple(snap.shape) == (ring, k, d_pad) and tuple(dq.shape) == (ring, k, 8)
    rc = nat.native().shift_operand(C_prev.data_ptr(), C_new.data_ptr(), int(C_new.stride(0)), int(d),
                                    int(d_pad), int(k), float(alpha), snap.data_ptr(), dsh.data_ptr(),
                                    dq.data_ptr(), int(ring), int(snew), int(valid),
                                    nat.stream_handle(C_new.device))
    if rc:
        raise RuntimeError(f"shift_operand failed (hip error {rc})")


def ensure_multi_buffers(buf: EStepBuffers, n, device, bounds=False):
    """Allocate the certified E-step's row lists (and, with ``bounds``, the
    per-row multi flag of the Hamerly pruning)."""
    if buf.dense_rows is None or buf.dense_rows.numel() < n:
        buf.dense_rows = torch.empty(max(n, 1), dtype=torch.int64, device=device)
    if buf.multi_rows is None or buf.multi_rows.numel() < n:
        buf.multi_rows = torch.empty(max(n, 1), dtype=torch.int64, device=device)
        buf.multi_cand = torch.empty((max(n, 1), 17), dtype=torch.int32, device=device)
    if bounds and (buf.mflag is None or buf.mflag.numel() < n):
        buf.mflag = torch.zeros(max(n, 1), dtype=torch.int32, device=device)


def centroid_delta_native(X, labels, prev, sums, counts, qsum, k, ws: ReduceWorkspace, perm2,
                          qexp, lists=None):
    """Incremental fixed-point cluster statistics (csrc/kmeans.hip
    delta_segment_kernel): sums / counts / qsum are UPDATED by the rows whose
    label differs from ``prev`` (prev = -1: the row enters), and ``prev``
    becomes ``labels`` in the same pass.  Bit-identical to recomputing them
    from scratch (exact integer arithmetic in fp64).  ``perm2``: int32
    workspace of 4 n (2 n (row, label) entries).

    ``lists``: up to three (int64 rows, int32 [1] device length) pairs (None
    = empty) that together hold, once each, every row whose label can differ
    from ``prev`` (a filtered E-step's row lists): only those rows are
    walked - the same statistics."""
    n, d = X.shape
    assert X.dtype == torch.float32 and X.is_contiguous() and d % 4 == 0 and d <= 1024
    assert labels.dtype == torch.int32 and prev.dtype == torch.int32 and perm2.numel() >= 4 * n
    assert sums.dtype == torch.float64 and sums.numel() >= k * d and qsum.numel() >= k
    if lists is not None:
        lp = []
        for ent in list(lists) + [None] * (3 - len(lists)):
            if ent is None:
                lp += [0, 0]
            else:
                rows, cnt = ent
                assert rows.dtype == torch.int64 and cnt.dtype == torch.int32
                lp += [rows.data_ptr(), cnt.data_ptr()]
        rc = nat.native().centroid_delta_lists(X.data_ptr(), labels.data_ptr(), prev.data_ptr(),
                                               sums.data_ptr(), counts.data_ptr(),
                                               qsum.data_ptr(), n, d, k, ws.xexp, int(qexp),
                                               ws.hist.data_ptr(), ws.cursor.data_ptr(),
                                               perm2.data_ptr(), *lp, nat.stream_handle(X.device))
        if rc:
            raise RuntimeError(f"centroid_delta_lists failed (hip error {rc})")
        return
    rc = nat.native().centroid_delta(X.data_ptr(), labels.data_ptr(), prev.data_ptr(),
                                     sums.data_ptr(), counts.data_ptr(), qsum.data_ptr(), n, d, k,
                                     ws.xexp, int(qexp), ws.hist.data_ptr(), ws.cursor.data_ptr(),
                                     perm2.data_ptr(), nat.stream_handle(X.device))
    if rc:
        raise RuntimeError(f"centroid_delta failed (hip error {rc})")


def cluster_inertia_native(sums, counts, qsum, C, k, d, ws: ReduceWorkspace, qexp, part):
    """part[c] = Q_c - 2 c.S_c + n_c |c|^2 at the centroids C (fp32 [k][d])."""
    assert C.dtype == torch.float32 and C.is_contiguous() and tuple(C.shape) == (k, d)
    rc = nat.native().cluster_inertia(sums.data_ptr(), counts.data_ptr(), qsum.data_ptr(),
                                      C.data_ptr(), k, d, ws.xexp, int(qexp), part.data_ptr(),
                                      nat.stream_handle(C.device))
    if rc:
        raise RuntimeError(f"cluster_inertia failed (hip error {rc})")


def mstep_stats_native(sums, counts, qsum, C, k, d, ws: ReduceWorkspace, qexp, corr, n, part,
                       inertia, packed):
    """The incremental M-step's statistics in two launches (csrc/kmeans.hip
    mstep_parts_kernel + pack_sum_kernel): per-cluster inertia parts at the
    E-step's centroids C (fp32 [k][d]) and the fixed-range partial sums of
    the corrections ``corr`` [n] into ``part`` (fp64 >= 512 + k), then the
    packed all-reduce bucket [sums, counts, inertia] with inertia[0] = the
    sum of all partials (the same association as cluster_inertia_native +
    sum_f32_native + pack_stats_native, unweighted)."""
    assert C.dtype == torch.float32 and C.is_contiguous() and tuple(C.shape) == (k, d)
    assert part.numel() >= 512 + k and part.dtype == torch.float64
    assert corr.dtype == torch.float32 and corr.data_ptr() % 16 == 0
    rc = nat.native().mstep_stats(sums.data_ptr(), counts.data_ptr(), qsum.data_ptr(),
                                  C.data_ptr(), k, d, ws.xexp, int(qexp), corr.data_ptr(), int(n),
                                  part.data_ptr(), inertia.data_ptr(), packed.data_ptr(),
                                  nat.stream_handle(C.device))
    if rc:
        raise RuntimeError(f"mstep_stats failed (hip error {rc})")


def pack_stats_native(sums, counts, inertia, packed, k, d, ws: ReduceWorkspace, weighted=False):
    nat.native().pack_stats(sums.data_ptr(), counts.data_ptr(),
                            0 if inertia is None else inertia.data_ptr(), packed.data_ptr(), k, d,
                            ws.xexp, ws.wexp if weighted else 0, nat.stream_handle(sums.device))


def centroid_finalize_native(packed, C_old, C_new, C_bf16, cn, shift, k, d, noise_b, key: RngKey,
                             empty_policy=0, shift_part=None, scalars=None, buf=None, C_f16=None,
                             alpha=1.0, k_pad=None, cmax2=None, kept=None):
    """shift[0] = sum_j ||c_j' - c_j||^2 (per-centroid parts summed in a fixed
    order: deterministic); ``shift_part`` is a k-double workspace.

    With ``scalars`` (3 doubles) the same launch also writes the iteration's
    [inertia, shift, overflow rows] (inertia from the packed bucket, overflow
    count from ``buf``, an :class:`EStepBuffers`, whose counter it resets);
    ``kept`` (device int32 [1], needs 4 scalars): scalars[3] = its value."""
    if kept is not None:
        assert scalars is not None and scalars.numel() >= 4
    if k_pad is None:
        k_pad = (C_bf16 if C_bf16 is not None else C_f16).shape[0] * 64
    if shift_part is None:
        shift_part = torch.empty(max(k, 1), dtype=torch.float64, device=packed.device)
    assert shift_part.numel() >= k and shift_part.dtype == torch.float64
    nat.native().centroid_finalize(packed.data_ptr(), C_old.data_ptr(), C_new.data_ptr(),
                                   nat.ptr(C_bf16), shift_part.data_ptr(), cn.data_ptr(),
                                   shift.data_ptr(), k, d, k_pad, float(noise_b), key.k0, key.k1,
                                   key.s0, key.s1, int(empty_policy),
                                   0 if scalars is None else scalars.data_ptr(),
                                   0 if buf is None else buf.ovf_count.data_ptr(),
                                   nat.ptr(C_f16), float(alpha), nat.ptr(cmax2), nat.ptr(kept),
                                   nat.stream_handle(packed.device))
    if scalars is not None and buf is not None:
        buf.ovf_clean = True


def operand_shape(k_pad, d_pad):
    """Shape of the chunk-major E-step centroid operand (csrc/kmeans.hip,
    ``estep_kernel``): [tile][16-B chunk][centroid in tile][8 bf16]."""
    return (k_pad // 64, d_pad // 8 + 2, 64, 8)


def _split3_bf16(v):
    hi = v.to(torch.bfloat16)
    r = v - hi.float()
    mid = r.to(torch.bfloat16)
    lo = (r - mid.float()).to(torch.bfloat16)
    return hi, mid, lo


def centers_to_bf16(C, k_pad, d_pad):
    """E-step operand of the centroids and fp32 ||bf16(c)||^2 (BIG on pads).

    The operand holds -2 bf16(c) chunk-major plus an augmented chunk with the
    3-way bf16 split of ||bf16(c)||^2 (see ``operand_shape``), exactly what
    ``centroid_finalize`` writes on the device.
    """
    k, d = C.shape
    cb = torch.zeros((k_pad, d_pad + 16), dtype=torch.bfloat16, device=C.device)
    h = C.to(torch.bfloat16)
    cb[:k, :d] = (-2.0 * h.float()).to(torch.bfloat16)
    cn = torch.full((k_pad,), BIG, dtype=torch.float32, device=C.device)
    cn[:k] = (h.float() ** 2).sum(1)
    hi, mid, lo = _split3_bf16(cn)
    cb[:, d_pad] = hi
    cb[:k, d_pad + 1] = mid[:k]
    cb[:k, d_pad + 2] = lo[:k]
    op = cb.view(k_pad // 64, 64, d_pad // 8 + 2, 8).permute(0, 2, 1, 3).contiguous()
    return op, cn


def centers_from_operand(op, k, d):
    """Inverse of ``centers_to_bf16``: the bf16-rounded centroids [k, d]."""
    nt, cpr = op.shape[0], op.shape[1]
    rows = op.permute(0, 2, 1, 3).reshape(nt * 64, cpr * 8)
    return (rows[:k, :d].float() * -0.5).to(torch.bfloat16)


def centroid_sums_torch(X, labels, k, weights=None, acc_dtype=torch.float64):
    """Label-segmented sums (torch index_add) -> (sums [k,d], counts [k])."""
    d = X.shape[1]
    sums = torch.zeros((k, d), dtype=acc_dtype, device=X.device)
    counts = torch.zeros(k, dtype=torch.float64, device=X.device)
    lab = labels.to(torch.int64)
    ok = lab >= 0
    if not bool(ok.all()):
        lab = lab[ok]
        X = X[ok]
        weights = weights[ok] if weights is not None else None
    if weights is None:
        sums.index_add_(0, lab, X.to(acc_dtype))
        counts.index_add_(0, lab, torch.ones_like(lab, dtype=torch.float64))
    else:
        sums.index_add_(0, lab, X.to(acc_dtype) * weights.to(acc_dtype)[:, None])
        counts.index_add_(0, lab, weights.to(torch.float64))
    return sums, counts


# ------------------------------------------------- fp32-faithful E-step
# (csrc/estep_f32.hip): fp16 hi/lo split operands, 3 MFMA products, fp32
# accumulation; overflow rows re-selected in fp64.

def operand_f16_shape(k_pad, d_pad):
    """[tile][hi chunks d_pad/8 + 2 | lo chunks d_pad/8][centroid in tile][8 fp16]."""
    return (k_pad // 64, 2 * (d_pad // 8) + 2, 64, 8)


ALPHA_TARGET_LOG2 = 13   # alpha^2 * (max row norm)^2 <= 2^13 keeps fp16 pieces in range


def choose_alpha(max_sq_norm, margin=0.0):
    """Power-of-two scale of the fp16 split: alpha^2 (R + margin)^2 <= 2^13
    with R^2 the largest squared row norm (all ranks) and ``margin`` the
    largest norm any centroid can add on top of a mean (tomography noise)."""
    r = math.sqrt(max(float(max_sq_norm), 0.0)) + float(margin)
    if not math.isfinite(r):
        raise ValueError("non-finite values in the data")
    if r <= 0.0:
        return 1.0
    e = math.floor(ALPHA_TARGET_LOG2 / 2.0 - math.log2(r))
    return float(2.0 ** max(min(e, 60), -60))


def _split3_f16(t):
    hi = t.to(torch.float16)
    r = t - hi.float()
    mid = r.to(torch.float16)
    lo = (r - mid.float()).to(torch.float16)
    return hi, mid, lo


def centers_to_f16(C, k_pad, d_pad, alpha):
    """fp16 hi/lo operand of fp32 centroids C [k, d] (torch twin of
    ``centers_f16_operand_kernel``): hi/lo of -2 alpha c chunk-major, the
    3-way split of alpha^2 ||c||^2 (fp64 sum) in the augmented chunk, 65504
    norms on padding centroids."""
    k, d = C.shape
    Cf = C.float()
    s = (-2.0 * alpha) * Cf
    hi = s.to(torch.float16)
    lo = (s - hi.float()).to(torch.float16)
    H = torch.zeros((k_pad, d_pad + 16), dtype=torch.float16, device=C.device)
    Lo = torch.zeros((k_pad, d_pad), dtype=torch.float16, device=C.device)
    H[:k, :d] = hi
    Lo[:k, :d] = lo
    nn = ((Cf.double() * alpha) ** 2).sum(1).float()
    a, b, c = _split3_f16(nn)
    H[:k, d_pad], H[:k, d_pad + 1], H[:k, d_pad + 2] = a, b, c
    H[k:, d_pad:d_pad + 3] = 65504.0
    nt = k_pad // 64
    Hc = H.view(nt, 64, d_pad // 8 + 2, 8).permute(0, 2, 1, 3)
    Lc = Lo.view(nt, 64, d_pad // 8, 8).permute(0, 2, 1, 3)
    return torch.cat([Hc, Lc], dim=1).contiguous()


def centers_to_f16_native(C, op, k, d, d_pad, k_pad, alpha):
    C = C.float().contiguous()
    assert tuple(op.shape) == operand_f16_shape(k_pad, d_pad) and op.dtype == torch.float16
    nat.native().centers_f16_operand(C.data_ptr(), op.data_ptr(), k, d, d_pad, k_pad, float(alpha),
                                     nat.stream_handle(C.device))
    return op


def estep_f32_native(Xf, C_op, xn, C_master, k, delta, alpha, key: RngKey, row_offset,
                     buf: EStepBuffers, stream=None):
    """fp32-faithful fused E-step (labels, min distances; inertia in
    ``buf.inertia``) + fp64 re-selection of overflow rows; no host sync."""
    n, d_pad = Xf.shape
    k_pad = C_op.shape[0] * 64
    d = C_master.shape[1]
    assert Xf.dtype == torch.float32 and Xf.is_contiguous() and d_pad in FAST_D
    assert C_op.dtype == torch.float16 and tuple(C_op.shape) == operand_f16_shape(k_pad, d_pad)
    assert C_op.is_contiguous() and C_master.dtype == torch.float32 and C_master.is_contiguous()
    assert C_master.shape[0] >= k and k <= k_pad and d <= d_pad
    assert xn.dtype == torch.float32 and xn.numel() >= n
    assert buf.labels.numel() >= n and buf.part_cap >= 4
    st = stream if stream is not None else nat.stream_handle(Xf.device)
    m = nat.native()
    if not buf.ovf_clean:
        buf.ovf_count.zero_()
    buf.ovf_clean = False
    rc = m.estep_f32(Xf.data_ptr(), C_op.data_ptr(), xn.data_ptr(), buf.labels.data_ptr(),
                     buf.mind.data_ptr(), buf.ovf_rows.data_ptr(), buf.ovf_count.data_ptr(),
                     buf.inertia_part.data_ptr(), int(buf.part_cap), buf.inertia.data_ptr(), n,
                     d_pad, k_pad, float(alpha), float(delta), key.k0, key.k1, key.s0, key.s1,
                     int(row_offset), buf.ovf_cap, st)
    rows_f64_native(Xf, C_master, buf.labels, buf.mind, delta, key, row_offset,
                    rows=(buf.ovf_rows, buf.ovf_count, buf.ovf_cap), stream=st)
    return buf.labels, buf.mind


def rows_f64_native(X, C, labels, mind, delta, key: RngKey, row_offset, rows=None, corr=None,
                    ub=None, d=None, grid=None, stream=None):
    """Exact fp64 E-step over a row list (csrc/rows_f64.hip: fp64-MFMA
    candidates with a rigorous bound, direct-form sum_f (x_f - c_f)^2 re-check,
    the delta-band rule of band.h).  ``rows`` = (list int64, count int32 [1]
    on the device, cap) or None for every row of X.  X fp32 [n][ldx], C fp32
    [k][ldc] (the first ``d`` columns of each are used).  Writes labels,
    mind (the min distance) and, when given, corr = mind - d(label) and
    ub = |x - c_label|.  No host sync."""
    n, ldx = X.shape
    k, ldc = C.shape
    d = int(min(ldx, ldc) if d is None else d)
    assert X.dtype == torch.float32 and X.stride(1) == 1 and X.stride(0) == ldx
    assert C.dtype == torch.float32 and C.is_contiguous() and d <= min(ldx, ldc)
    assert labels.dtype == torch.int32 and mind.dtype == torch.float32
    if rows is None:
        if n == 0:
            return labels, mind
        cnt_ptr, nd, cap, rptr = 0, n, n, 0
        groups = (n + 15) // 16
    else:
        rlist, count, cap = rows
        rptr, cnt_ptr, nd = rlist.data_ptr(), count.data_ptr(), 0
        groups = (int(cap) + 15) // 16
    if grid is None:
        grid = max(1, min(groups, 1024 if rows is None else 512))
    st = stream if stream is not None else nat.stream_handle(X.device)
    rc = nat.native().rows_f64(X.data_ptr(), int(ldx), C.data_ptr(), int(ldc), d, int(k), rptr,
                               cnt_ptr, int(nd), int(cap), labels.data_ptr(), mind.data_ptr(),
                               nat.ptr(corr), nat.ptr(ub), float(delta), key.k0, key.k1, key.s0,
                               key.s1, int(row_offset), int(grid), st)
    if rc:
        raise RuntimeError(f"rows_f64 failed (hip error {rc})")
    return labels, mind


def estep_x64_native(Xh, Xf, C_op, C_pad, xn, cmax2, k, delta, alpha, key: RngKey, row_offset,
                     buf: EStepBuffers, stream=None, bounds=None, rows=None, zero_counts=True,
                     screen=False, list_rs=0):
    """Certified E-step (``estep_x64_kernel``): one fp16 MFMA pass with a
    rigorous error bound, fp64 re-check of the candidate centroids, dense rows
    through the fp32-faithful 3-pass kernel.  Labels are the fp64 delta-band
    rule's; ``buf.mind`` holds -1 on single-candidate rows (filled by the
    M-step's row pass or ``fill_mind_native``).  No host sync.

    ``bounds`` = (ub, lb) fp32 [n]: the kernel writes each processed row's
    Hamerly bounds and multi flag (``buf.mflag``); ``rows`` =
    (rlist int64 [n], rcount int32 [1]): process only the listed rows (list
    mode, count on the device; the filter already started this iteration's
    multi list, so ``zero_counts`` is False).  ``screen``: multi rows go
    through the fp32 screen first (``recheck_fast_kernel``; their ``mind``
    is then fp32 - for steps whose inertia comes from the incremental
    statistics), the fp64 re-check takes the rest.  ``list_rs``: row sets
    per wave of the list-mode sweep (0 = default 1: a short list finishes
    in one half-length sweep; 2 = the full sweep's tiling, for a list the
    caller expects to hold nearly every row)."""
    n, d_pad = Xf.shape
    k_pad = C_op.shape[0] * 64
    assert Xf.dtype == torch.float32 and Xf.is_contiguous() and d_pad in X64_D
    assert Xh.dtype == torch.float16 and Xh.is_contiguous() and tuple(Xh.shape) == (n, d_pad)
    assert C_op.dtype == torch.float16 and tuple(C_op.shape) == operand_f16_shape(k_pad, d_pad)
    assert C_pad.dtype == torch.float32 and C_pad.is_contiguous()
    assert tuple(C_pad.shape) == (k, d_pad)
    assert cmax2.dtype == torch.float32 and xn.dtype == torch.float32 and xn.numel() >= n
    assert k <= k_pad <= X64_MAX_K and buf.labels.numel() >= n
    ensure_multi_buffers(buf, n, Xf.device, bounds is not None)
    if screen and (buf.exact_flag is None or buf.exact_flag.numel() < n):
        buf.exact_flag = torch.empty(max(n, 1), dtype=torch.uint8, device=Xf.device)
    st = stream if stream is not None else nat.stream_handle(Xf.device)
    if zero_counts:
        buf.counts.zero_()
    buf.ovf_clean = False
    # dense rows (d_pad <= 256): the 3-pass kernel's overflow rows get a
    # second pass with 3 band members per lane before the fp64 rows kernel
    import os
    if d_pad <= 256 and os.environ.get("SQ_OVF2", "1") != "0":
        if buf.ovf2_rows is None or buf.ovf2_rows.numel() < n:
            buf.ovf2_rows = torch.empty(max(n, 1), dtype=torch.int64, device=Xf.device)
        nat.native().set_overflow2(buf.ovf2_rows.data_ptr(), buf.counts[6:7].data_ptr())
    else:
        nat.native().set_overflow2(0, 0)
    nat.native().estep_x64(Xh.data_ptr(), Xf.data_ptr(), C_op.data_ptr(), C_pad.data_ptr(),
                           xn.data_ptr(), cmax2.data_ptr(), buf.labels.data_ptr(),
                           buf.mind.data_ptr(), buf.dense_rows.data_ptr(), buf.ovf_rows.data_ptr(),
                           buf.multi_rows.data_ptr(), buf.multi_cand.data_ptr(),
                           0 if buf.corr is None else buf.corr.data_ptr(),
                           0 if rows is None else rows[0].data_ptr(),
                           0 if rows is None else rows[1].data_ptr(),
                           0 if bounds is None else bounds[0].data_ptr(),
                           0 if bounds is None else bounds[1].data_ptr(),
                           0 if bounds is None else buf.mflag.data_ptr(),
                           buf.exact_flag.data_ptr() if screen else 0,
                           buf.counts.data_ptr(), buf.inertia_part.data_ptr(), int(buf.part_cap),
                           n, d_pad, d_pad, k, k_pad, float(alpha), float(delta), key.k0, key.k1,
                           key.s0, key.s1, int(row_offset), st, int(list_rs))
    return buf.labels, buf.mind


def fill_mind_native(Xf, C_master, labels, mind):
    """mind[i] = |x_i - c_label(i)|^2 (fp64, stored fp32) where mind[i] < 0."""
    n, ldx = Xf.shape
    nat.native().fill_mind(Xf.data_ptr(), ldx, C_master.data_ptr(), C_master.shape[1],
                           labels.data_ptr(), mind.data_ptr(), n, nat.stream_handle(Xf.device))


def sum_f32_native(v, n, part, out, extra=0):
    """out[0] = sum(v[:n]) + sum(part[512:512 + extra]) in a fixed order
    (deterministic); part >= 512 + extra doubles (the extra partials were
    written there by an earlier launch)."""
    assert part.numel() >= 512 + extra and part.dtype == torch.float64 and extra >= 0
    rc = nat.native().sum_f32(v.data_ptr(), int(n), part.data_ptr(), int(extra), out.data_ptr(),
                              nat.stream_handle(v.device))
    if rc:
        raise RuntimeError(f"sum_f32 failed (hip error {rc})")


# ------------------------------------------------- k-means++ (exact, pruned)
class KmppState:
    """Device state of the exact accelerated k-means++ (csrc/kmpp.hip) on
    one shard: per-row closest distance (fp32) and nearest chosen centre, the
    int8 row copy of the certified bound, the two (mask, D) buffers of the
    lazily applied winner, the survivor / exact row lists, the fixed-point
    block totals of the two-level sampler.  ``prune=False`` sends every row
    through the exact pass (same results: the screens only skip rows whose
    minimum provably stays the same)."""

    def __init__(self, Xf, k, t, w=None, prune=True, shared=None):
        """``shared``: another state over the same rows whose int8 row copy
        (and its scales / error norms) this one reads instead of its own."""
        n, d = Xf.shape
        dev = Xf.device
        assert Xf.dtype == torch.float32 and Xf.stride(1) == 1 and d % 4 == 0
        assert Xf.stride(0) % 4 == 0 and Xf.data_ptr() % 16 == 0 and 1 <= t <= 16
        self.X, self.n, self.d, self.t, self.k = Xf, n, d, t, int(k)
        self.ldx = Xf.stride(0)
        self.w = None if w is None else w.to(device=dev, dtype=torch.float64).contiguous()
        self.prune = bool(prune) and d <= 8192
        self.dq = -(-d // 64) * 64
        self.dev = dev
        m = nat.native()
        self.m = m
        self.st = nat.stream_handle(dev)
        G0 = m.kmpp_grid(max(n, 1))
        self.R = max(1, -(-n // G0))
        self.G = max(1, -(-n // self.R))
        self.owns_q = shared is None
        if self.prune and n and shared is not None:
            assert shared.prune and shared.X is Xf
            self.Xq, self.srow, self.erow, self.xq2 = shared.Xq, shared.srow, shared.erow, shared.xq2
        elif self.prune and n:
            self.Xq = torch.empty((n, self.dq), dtype=torch.int8, device=dev)
            self.srow = torch.empty(n, dtype=torch.float32, device=dev)
            self.erow = torch.empty(n, dtype=torch.float32, device=dev)
            self.xq2 = torch.empty(n, dtype=torch.int32, device=dev)   # |q|^2 (exact)
            # (filled by first_centre's pass over X)
        nn = max(n, 1)
        self.closest = torch.empty(nn, dtype=torch.float32, device=dev)
        self.nearest = torch.zeros(nn, dtype=torch.int32, device=dev)
        self.mask = [torch.zeros(nn, dtype=torch.int16, device=dev) for _ in range(2)]
        self.D = [torch.empty((t, nn), dtype=torch.float32, device=dev) for _ in range(2)]
        # per-block row-list segments (block b: rows [b R, b R + count[b]))
        self.surv = torch.empty(max(self.G * self.R, 1), dtype=torch.int32, device=dev)
        self.exact = torch.empty(max(self.G * self.R, 1), dtype=torch.int32, device=dev)
        self.scount = torch.zeros(self.G, dtype=torch.int32, device=dev)
        self.ecount = torch.zeros(self.G, dtype=torch.int32, device=dev)
        self.counters = torch.zeros(4, dtype=torch.int32, device=dev)
        # min over the trials of |cand_j - C_m|^2 per chosen centre m (triangle screen)
        self.cc = torch.zeros(self.k, dtype=torch.float32, device=dev)
        # two-term int8 candidates [hi / lo][16 trial slots][dq] and (s_c, ec, |c~|^2, 0)
        self.cinfo = torch.zeros((16, 4), dtype=torch.float64, device=dev)
        self.candq = torch.zeros((2, 16, self.dq), dtype=torch.int8, device=dev)
        self.delta = torch.zeros((self.G, t), dtype=torch.float64, device=dev)
        self.block_tot = torch.zeros(self.G, dtype=torch.float64, device=dev)
        self.pos = torch.zeros(t, dtype=torch.int64, device=dev)
        self.cur = 0            # index of the (mask, D) pair the next trial pass writes
        self.best = None        # device int32 [1]: the last step's winning trial
        self.c_last = -1        # centre index of that winner
        self.scale = 1.0

    def first_centre(self, c0):
        """closest / nearest for the first centre (and, pruned, the int8 row
        copy in the same pass over X); returns the local max of w * closest
        (device fp64 [1]) for the global fixed-point scale."""
        bmax = torch.zeros(self.m.kmpp_grid(-1), dtype=torch.float64, device=self.dev)
        if self.n:
            c0 = c0.to(torch.float32).contiguous()
            q = self.prune and self.owns_q
            _rc(self.m.kmpp_init(self.X.data_ptr(), self.ldx, self.d, self.n, c0.data_ptr(),
                                 0 if self.w is None else self.w.data_ptr(),
                                 self.closest.data_ptr(), self.nearest.data_ptr(), bmax.data_ptr(),
                                 self.Xq.data_ptr() if q else 0, self.dq,
                                 self.srow.data_ptr() if q else 0,
                                 self.erow.data_ptr() if q else 0,
                                 self.xq2.data_ptr() if q else 0, self.st), "kmpp_init")
        return bmax.max().reshape(1)

    def set_scale(self, max_pot, n_global):
        """Power-of-two fixed-point scale with n_global * max_pot * scale <=
        2^52 (every potential sum an exact fp64 integer); returns this
        shard's total (device fp64 [1])."""
        mx = float(max_pot)
        self.scale = 1.0 if not mx > 0.0 else 2.0 ** math.floor(
            math.log2(2.0 ** 52 / (max(n_global, 1) * mx)))
        if self.n:
            _rc(self.m.kmpp_block_totals(self.closest.data_ptr(),
                                         0 if self.w is None else self.w.data_ptr(), self.n,
                                         self.R, self.G, self.scale, self.block_tot.data_ptr(),
                                         self.st), "kmpp_block_totals")
        return self.block_tot.sum().reshape(1)

    def pick(self, vals, cands=None, cand_ids=None, row_offset=0, n_global=None):
        """Local rows of the potential values ``vals`` (device fp64 [t]):
        first row whose inclusive prefix reaches each value.  With ``cands``
        (fp32 [t, d]) / ``cand_ids`` (int64 [t]) the same launch also copies
        the rows and writes their global ids (clamped to the shard)."""
        t = vals.numel()
        if self.n == 0:
            return torch.zeros(t, dtype=torch.int64, device=self.dev)
        assert t <= self.pos.numel()
        vals = vals.to(torch.float64).contiguous()
        prev = 1 - self.cur
        if cands is not None:
            assert cands.dtype == torch.float32 and cands.is_contiguous()
            assert tuple(cands.shape) == (t, self.d) and cand_ids.dtype == torch.int64
        _rc(self.m.kmpp_pick(self.block_tot.data_ptr(), self.G, self.R, self.n, vals.data_ptr(), t,
                             self.closest.data_ptr(), self.mask[prev].data_ptr(),
                             self.D[prev].data_ptr(),
                             0 if self.best is None else self.best.data_ptr(),
                             0 if self.w is None else self.w.data_ptr(), self.scale,
                             self.pos.data_ptr(), self.X.data_ptr(), self.ldx, self.d,
                             0 if cands is None else cands.data_ptr(),
                             0 if cand_ids is None else cand_ids.data_ptr(), int(row_offset),
                             int(self.n if n_global is None else n_global), self.st), "kmpp_pick")
        return self.pos[:t].clone()

    def trials(self, cand, centers, c, reduce=True):
        """Trial pass for the candidates ``cand`` [t, d] against the ``c``
        centres chosen so far (``centers[:c]``): returns Delta (device fp64
        [t]), the fixed-point improvement of each trial over this shard."""
        t = cand.shape[0]
        assert t == self.t and 1 <= c <= self.k
        cand = cand.to(torch.float32).contiguous()
        Cc = (centers if centers.dtype == torch.float32 else centers.float()).contiguous()
        m, st = self.m, self.st
        prev, cur = 1 - self.cur, self.cur
        _rc(m.kmpp_cc(cand.data_ptr(), Cc.data_ptr(), int(c), self.d, t, self.cc.data_ptr(), self.k,
                      self.cinfo.data_ptr(), self.candq.data_ptr(), self.dq, self.delta.data_ptr(),
                      self.delta.numel(), self.counters.data_ptr(), st), "kmpp_cc")
        if self.n:
            _rc(m.kmpp_screen(self.closest.data_ptr(), self.nearest.data_ptr(),
                              self.mask[prev].data_ptr(), self.D[prev].data_ptr(),
                              0 if self.best is None else self.best.data_ptr(), self.c_last,
                              self.cc.data_ptr(), self.k, t, self.n, self.R, self.G,
                              self.mask[cur].data_ptr(), self.surv.data_ptr(),
                              self.exact.data_ptr(), self.scount.data_ptr(),
                              self.ecount.data_ptr(), int(self.prune), st), "kmpp_screen")
            if self.prune:
                _rc(m.kmpp_bound(self.Xq.data_ptr(), self.dq, self.srow.data_ptr(),
                                 self.erow.data_ptr(), self.xq2.data_ptr(),
                                 self.closest.data_ptr(), self.candq.data_ptr(),
                                 self.cinfo.data_ptr(), t, self.d, self.n, self.R, self.G,
                                 self.surv.data_ptr(), self.scount.data_ptr(),
                                 self.exact.data_ptr(), self.ecount.data_ptr(), st),
                    "kmpp_bound")
            _rc(m.kmpp_exact(self.X.data_ptr(), self.ldx, self.d, self.n, t, cand.data_ptr(),
                             self.closest.data_ptr(), 0 if self.w is None else self.w.data_ptr(),
                             self.scale, self.exact.data_ptr(), self.ecount.data_ptr(),
                             self.mask[cur].data_ptr(), self.D[cur].data_ptr(),
                             self.delta.data_ptr(), self.R, self.G, st), "kmpp_exact")
        return self.delta.sum(0) if reduce else None

    def apply(self, best, c):
        """The winning trial (device int64 scalar) of centre ``c``: block
        totals lose its improvements; its rows are updated lazily by the next
        screen / pick."""
        self.block_tot -= self.delta.index_select(1, best.reshape(1))[:, 0]
        self.best = best.reshape(1).to(torch.int32)
        self.c_last = int(c)
        self.cur ^= 1

    def finish(self, P, draws_next, vals, cands, cand_ids, centers, ids, c):
        """Single-rank winner of centre ``c`` in one launch: trial potentials
        P - Delta_j (exact integers), the first minimum wins; updates ``P``
        (fp64 [1]), the block totals, ``centers[c]``, ``ids[c]``, the lazily
        applied winner and ``vals`` = draws_next * P (the next centre's
        sampling values; ``draws_next`` None: last centre)."""
        if self.best is None:
            self.best = torch.zeros(1, dtype=torch.int32, device=self.dev)
        _rc(self.m.kmpp_finish(self.delta.data_ptr(), self.G, self.t, self.block_tot.data_ptr(),
                               P.data_ptr(), 0 if draws_next is None else draws_next.data_ptr(),
                               vals.data_ptr(), cands.data_ptr(), cand_ids.data_ptr(), self.d,
                               centers.data_ptr(), ids.data_ptr(), int(c), self.best.data_ptr(),
                               self.st), "kmpp_finish")
        self.c_last = int(c)
        self.cur ^= 1

    def list_counts(self):
        """[survivors of the triangle screen, rows of the exact pass] of the
        last trial pass (host read; diagnostics)."""
        if not self.prune:
            return [0, int(self.ecount.sum())]
        return [int(self.scount.sum()), int(self.ecount.sum())]



class KmppBatch:
    """NR restarts of the exact accelerated k-means++ (one rank), advanced
    through their centres in lockstep: per phase one launch for all of them
    (csrc/kmpp.hip ``sq_kmpp_batch``; the row passes interleave the
    restarts' workgroups of a row block, so rows two restarts need are read
    from HBM once).  Each restart is a ``KmppState`` (its own closest /
    nearest / masks / lists / fixed-point scale) over the shared int8 row
    copy; the results are those of NR sequential runs with the same draws."""

    NF = 32

    def __init__(self, Xf, k, t, nr, w=None, prune=True):
        self.states = [KmppState(Xf, k, t, w=w, prune=prune)]
        for _ in range(1, nr):
            self.states.append(KmppState(Xf, k, t, w=w, prune=prune, shared=self.states[0]))
        self.X, self.k, self.t, self.nr = Xf, int(k), int(t), int(nr)
        self.n, self.d = Xf.shape
        dev = Xf.device
        self.dev = dev
        self.cands = torch.empty((nr, t, self.d), dtype=torch.float32, device=dev)
        self.cand_ids = torch.empty((nr, t), dtype=torch.int64, device=dev)
        self.centers = torch.empty((nr, self.k, self.d), dtype=torch.float32, device=dev)
        self.ids = torch.empty((nr, self.k), dtype=torch.int64, device=dev)
        self.P = torch.zeros((nr, 1), dtype=torch.float64, device=dev)
        self.vals = torch.zeros((nr, t), dtype=torch.float64, device=dev)
        self.best = torch.zeros((nr, 1), dtype=torch.int32, device=dev)
        # fused screen / bound (ops 7 / 8): one read of a row per centre step
        # for all restarts (nr <= 16 restarts, nr tp <= 128 trial columns,
        # dq <= 256); SQ_KMPP_FUSED=0: the per-restart passes (same ids)
        st0 = self.states[0]
        self.tp = 1 << max(0, (self.t - 1).bit_length())
        self.fused = (prune and self.n > 0 and nr <= 16 and nr * self.tp <= 128
                      and st0.dq <= 256 and os.environ.get("SQ_KMPP_FUSED", "1") != "0")
        # exact pass with a lane per (row, trial) (op 9; d <= 256);
        # SQ_KMPP_EXACT2=0: a lane per row (op 4, same results)
        self.exact2 = (self.d <= 256 and self.t <= 16
                       and os.environ.get("SQ_KMPP_EXACT2", "1") != "0")
        # after the fused bound: only the undecided (row, trial) pairs (op 10)
        self.pairs = self.exact2 and os.environ.get("SQ_KMPP_PAIRS", "1") != "0"
        if self.fused:
            GR = max(st0.G * st0.R, 1)
            self.useg = torch.empty(GR, dtype=torch.int32, device=dev)
            self.umask = torch.empty(GR, dtype=torch.int16, device=dev)
            self.ucount = torch.zeros(st0.G, dtype=torch.int32, device=dev)

    def run(self, c0s, draws, ids0, n_global, row_offset=0):
        """``c0s`` fp32 [nr, d] (first centres), ``draws`` fp64 [nr, k - 1, t]
        (device), ``ids0`` int64 [nr] (the first centres' global ids):
        returns (centers [nr, k, d], ids [nr, k])."""
        st0 = self.states[0]
        m, stream = st0.m, st0.st
        nr, k, t = self.nr, self.k, self.t
        draws = draws.to(device=self.dev, dtype=torch.float64).contiguous()
        self.centers[:, 0].copy_(c0s)
        self.ids[:, 0].copy_(ids0)
        for r, s_ in enumerate(self.states):
            mx = s_.first_centre(c0s[r])
            self.P[r].copy_(s_.set_scale(mx.item(), n_global))
        if k > 1:
            self.vals.copy_(draws[:, 0] * self.P)
        F = self.NF
        tab = torch.zeros((nr, F), dtype=torch.int64)
        for r, s_ in enumerate(self.states):
            row = {0: s_.closest, 1: s_.nearest, 2: s_.mask[0], 3: s_.mask[1], 4: s_.D[0],
                   5: s_.D[1], 6: s_.surv, 7: s_.exact, 8: s_.scount, 9: s_.ecount, 10: s_.cc,
                   11: s_.cinfo, 12: s_.candq, 13: s_.delta, 14: s_.block_tot, 15: s_.pos,
                   16: self.cands[r], 17: self.cand_ids[r], 18: self.centers[r], 19: self.ids[r],
                   20: self.P[r], 21: self.vals[r], 22: draws[r], 23: self.best[r],
                   24: s_.counters}
            for f, ten in row.items():
                tab[r, f] = ten.data_ptr()
            tab[r, 25] = torch.tensor([s_.scale], dtype=torch.float64).view(torch.int64)[0]
        self._tab = tab.to(self.dev)
        ia = torch.zeros(32, dtype=torch.int64)
        ia[0], ia[1] = self._tab.data_ptr(), nr
        ia[2], ia[3], ia[4], ia[5] = self.X.data_ptr(), st0.ldx, self.d, self.n
        ia[6], ia[7], ia[8] = t, k, st0.dq
        if st0.prune and self.n:
            ia[9], ia[10], ia[11], ia[12] = (st0.Xq.data_ptr(), st0.srow.data_ptr(),
                                             st0.erow.data_ptr(), st0.xq2.data_ptr())
        ia[13] = 0 if st0.w is None else st0.w.data_ptr()
        ia[14], ia[15] = st0.R, st0.G
        ia[19] = int(st0.prune)
        ia[20], ia[21] = int(row_offset), int(n_global)
        ia[23] = st0.delta.numel()
        ia[27] = self.tp
        if self.fused:
            ia[24], ia[25], ia[26] = (self.useg.data_ptr(), self.umask.data_ptr(),
                                      self.ucount.data_ptr())
        iap = ia.data_ptr()

        def run_op(op):
            _rc(m.kmpp_batch(op, iap, stream), f"kmpp_batch op {op}")

        cur, c_prev = 0, -1
        for c in range(1, k):
            ia[16], ia[17], ia[18] = c, c_prev, cur
            ia[22] = c * t if c < k - 1 else -1
            run_op(5)                       # pick (+ candidate rows)
            run_op(1)                       # candidate quantisation, centre distances
            if self.n and self.fused:
                run_op(7)                   # triangle screen, all restarts: union list
                run_op(8)                   # certified int8 bound, one row read
                run_op(10 if self.pairs else (9 if self.exact2 else 4))   # exact pass
            elif self.n:
                run_op(2)                   # triangle screen (+ lazy winner)
                if st0.prune:
                    run_op(3)               # certified int8 bound
                run_op(9 if self.exact2 else 4)   # exact pass
            run_op(6)                       # winners, next sampling values
            c_prev, cur = c, cur ^ 1
        return self.centers, self.ids

def _rc(rc, name):
    if rc:
        raise RuntimeError(f"{name} failed (hip error {rc})")


# ------------------------------------------------ certified fp16 IPE screen
# (csrc/ipe16.hip): the IPE E-step without a per-pair fp32 inner product.

IPE16_D = X64_D           # d_pad of the fp16 sweep (> 256: values pass first, see Ipe16.gv)
IPE16_MAX_K = 16384       # centroid ids in 14 bits
IPE16_CAPR = 64           # listed pairs per row (csrc kCapR)
# rows per launch group at most (bounds the pair list: 8 B x 64 per row, 8.6 GB
# at 2^24 rows of 288 GB); the groups of a shard are balanced.  10M x 256,
# k = 1024: 3 / 2 / 1 groups -> 11.87 / 11.66 / 11.39 ms per IPE step (every
# launch's tail is paid once per group)
IPE16_CHUNK = int(os.environ.get("SQ_IPE16_CHUNK", 1 << 24))


class Ipe16:
    """Buffers and launch sequence of the certified fp16 IPE screen for one
    engine (rows ``[0, n)`` of a shard).  Per E-step and row chunk: (first
    step only) the fp16 argmin sweep for the hints, prep (hint pair in full,
    far band, row budget), the fp16 screen sweep, the near-pair kernel,
    finalize; rows the screen leaves dense go to the fp32 row-group kernel
    (``ipe_fused_native`` list mode) with the same hint and threshold."""

    def __init__(self, X, k, d_pad, k_pad, alpha, device):
        n, d = X.shape
        self.n, self.d, self.k, self.d_pad, self.k_pad = n, d, int(k), int(d_pad), int(k_pad)
        self.alpha = float(alpha)
        dev = device
        self.Xh = torch.zeros((n, d_pad), dtype=torch.float16, device=dev)
        step = 1 << 20
        for s in range(0, n, step):
            self.Xh[s:s + step, :d] = (X[s:s + step].float() * self.alpha).to(torch.float16)
        self.C_op = torch.zeros(operand_f16_shape(k_pad, d_pad), dtype=torch.float16, device=dev)
        self.thr = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
        self.hj = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        self.vlo = torch.empty((max(n, 1), 4), dtype=torch.float32, device=dev)   # [row][group]
        self.vhi = torch.empty((max(n, 1), 4), dtype=torch.float32, device=dev)
        self.H = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
        self.rfire = torch.empty((max(n, 1), 8), dtype=torch.int16, device=dev)
        self.rst = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        self.rflag = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        self.best = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        self.dense_rows = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        # wide rows (d_pad > 256; SQ_IPE16_GV=1 forces it): the sweep's
        # values [chunk rows][k_pad] fp32 come from a separate MFMA pass
        # (csrc/ipe16.hip ipe16_values_kernel, bit-identical values), the
        # chunk sized so that buffer stays <= 8 GiB
        self.gv = self.d_pad > 256 or os.environ.get("SQ_IPE16_GV", "0") == "1"
        cap = (min(IPE16_CHUNK, max(4096, (1 << 31) // self.k_pad)) if self.gv
               else IPE16_CHUNK)
        nch = max(1, -(-n // cap))
        self.chunk = min(cap, ((-(-n // nch) + 255) // 256) * 256) if n > 0 else cap
        cm = min(n, self.chunk)
        self.V = (torch.empty((max(cm, 1), self.k_pad), dtype=torch.float32, device=dev)
                  if self.gv else None)
        self.list = torch.empty(max(cm * IPE16_CAPR, 1), dtype=torch.int64, device=dev)
        self.nchunks = max(1, -(-n // self.chunk))
        # per chunk: [list count, dense count, sweep row count]
        self.counts = torch.zeros((self.nchunks, 3), dtype=torch.int32, device=dev)
        self.counts_host = torch.zeros((self.nchunks, 3), dtype=torch.int32, pin_memory=True)
        # row skip (csrc/ipe16.hip prep): per-row lower bound on the distance
        # to every non-label centroid, kept across E-steps (valid while the
        # hints are the previous E-step's labels), the bound's conversion
        # offset and the hint pair's distance bound, the sweep's row list
        self.lb = torch.zeros(max(n, 1), dtype=torch.float32, device=dev)
        self.lbo = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
        self.dhint = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
        self.ea2 = torch.empty(max(n, 1), dtype=torch.float32, device=dev)   # E / alpha^2
        self.rows = torch.empty(max(cm, 1), dtype=torch.int32, device=dev)
        self.smax = torch.zeros(1, dtype=torch.float32, device=dev)        # tau
        self.Rc = torch.zeros((max(int(k), 1), 4), dtype=torch.float32, device=dev)
        self.mw = torch.zeros(max(int(k), 1), dtype=torch.float32, device=dev)
        self.n_wild = 16
        self.native_bounds = os.environ.get("SQ_IPE16_NATIVE_BOUNDS", "1") != "0"
        self.C_prev = None
        self.lb_valid = False
        self.skip = __import__("os").environ.get("SQ_IPE16_SKIP", "1") != "0"
        self.ev = torch.cuda.Event()
        # per-pair hazard of the far band (the band edge's worst case): the
        # row fires somewhere with probability ~ k * ht; a larger ht narrows
        # the near set, a smaller one lists fewer fires
        # (a fired far pair costs one inner product and a thinning test in
        # prep; a near pair the sweep's listing and a full sampler).  10M x
        # 256, k = 1024: 2e-4 / 4e-4 / 9e-4 -> 13.4 / 13.1 / 13.7 ms per step
        self.ht = float(os.environ.get("SQ_IPE16_HT", "4e-4"))
        # bands narrower than this fraction of their lower edge: dense
        self.min_width = float(__import__("os").environ.get("SQ_IPE16_MINW", "0.5"))
        self.last_dense = 0

    def relaunch(self, op):
        """Re-run one phase of the last E-step's last chunk (kernel timing;
        prep re-lists the sweep rows from scratch, the screen sweep re-lists
        its pairs, so their counters restart)."""
        ia, da, st = self._last_args
        if op == 0:
            self.counts[-1, 2].zero_()
        if op == 2:
            self.counts[-1, :2].zero_()
        return nat.native().ipe16(op, ia.ctypes.data, da.ctypes.data, st)

    @staticmethod
    @__import__("functools").lru_cache(maxsize=64)
    def band_m(Q, ht):
        """The bin distance m at which the far band's hazard bound (row_cut's
        pu(m)) equals ``ht``: the band starts where m_lo >= this."""
        h = (Q + 1) // 2
        cq = 1.0
        for i in range(h):
            cq = cq * (Q - i) / (i + 1)
        cqh = float(torch.tensor(cq * 1.0002 * (1 + 1e-6), dtype=torch.float32))

        def pu(m):
            r = (1.0 / m) * (1 + 1e-5)
            pb = (r + r * r) * 0.500012 * (1 + 1e-5)
            return cqh * pb ** h * (1 + 2e-3)

        lo, hi = 3.0, 1e9
        if pu(lo) <= ht:
            return lo
        for _ in range(200):
            mid = math.sqrt(lo * hi)
            if pu(mid) <= ht:
                hi = mid
            else:
                lo = mid
        return hi

    def invalidate_bounds(self):
        """The hints no longer are the labels the bounds were kept for
        (new centres, restored hints): no row skip until a full sweep."""
        self.lb_valid = False

    def _skip_bounds(self, C32):
        """Device inputs of the row skip for centres C32 (fp32, the E-step's;
        after ``set_centers``), fp64 then rounded outward to fp32: the
        centroids' shifts since the last E-step's centres - the n_wild
        largest are "wild", tau (smax) bounds every other one, so a kept
        bound decays by tau only; mw[a] = min over the wild j != a of
        |c_a - c_j| (the wild centroids are bounded through the hint's
        centre instead); Rc[a][g] = max over norm group g of |c_a - c_j|
        (the upper side)."""
        k = C32.shape[0]
        dev = C32.device
        C64 = C32.double()
        if k <= 4096 and self.native_bounds:
            # csrc/ipe16.hip op 5: the same quantities in three launches after
            # the fp64 GEMM (each torch op below is a launch of its own)
            G = C64 @ C64.T
            if not hasattr(self, "_sb_work") or self._sb_work[0].shape[0] != k:
                self._sb_work = (torch.empty(k, dtype=torch.float64, device=dev),
                                 torch.empty(k, dtype=torch.float64, device=dev),
                                 torch.zeros(1, dtype=torch.float64, device=dev),
                                 torch.zeros(1, dtype=torch.int32, device=dev))
            sh, nn, tau, wn = self._sb_work
            prev = self.C_prev is not None and self.C_prev.shape == C32.shape
            C32c = C32.contiguous()
            # (host argument arrays in numpy: a torch CPU tensor costs a few us
            # per element assignment, on the step boundary's critical path)
            ia = np.zeros(20, dtype=np.int64)
            ia[0] = C32c.data_ptr()
            ia[1] = self.C_prev.data_ptr() if prev else 0
            ia[2], ia[4] = G.data_ptr(), self.perm.data_ptr()
            ia[5], ia[6], ia[7], ia[8] = k, C32.shape[1], self.G, self.n_wild
            for g in range(4):
                ia[9 + g] = self.gstart[g]
            ia[13], ia[14], ia[15], ia[16] = sh.data_ptr(), nn.data_ptr(), tau.data_ptr(), wn.data_ptr()
            ia[17], ia[18], ia[19] = self.smax.data_ptr(), self.mw.data_ptr(), self.Rc.data_ptr()
            da = np.array([1e-12], dtype=np.float64)
            nat.native().ipe16(5, ia.ctypes.data, da.ctypes.data, nat.stream_handle(dev))
            if prev:
                self.last_wild = wn
            self.C_prev = C32c.clone()
            return
        # (outward fp32 rounding by a 2^-20 relative margin - plain products,
        # not nextafter / pow / median: every distinct torch kernel costs
        # 30-130 ms of lazy loading at its first use in a process, which the
        # first IPE step paid)
        up, dn = 1.0 + 2.0 ** -20, 1.0 - 2.0 ** -20
        nrm = (C64 * C64).sum(1)
        D2 = nrm[:, None] + nrm[None, :] - 2.0 * (C64 @ C64.T)
        marg = 1e-12 * nrm.max()
        Dlo = (D2 - marg).clamp_min(0.0).sqrt() * (1.0 - 1e-9)
        Dhi = (D2 + marg).clamp_min(0.0).sqrt() * (1.0 + 1e-9)
        W = min(self.n_wild, k)
        if self.C_prev is not None and self.C_prev.shape == C32.shape:
            dd = C64 - self.C_prev.double()
            sh = (dd * dd).sum(1).sqrt() * (1.0 + 1e-9)
            # adaptive wild set: at least n_wild, and every centroid that moved
            # more than 1 % of the median nearest-centroid distance (up to
            # k / 2) - a few hundred centroids contesting unclaimed blobs jump
            # by ~10 units per IPE step at 10M x 256 while the rest barely
            # move, and a kept bound decays by tau every step
            # (device-side: no host read of the count)
            Dn = Dlo + torch.diag(torch.full((k,), float("inf"), dtype=torch.float64, device=dev))
            tgt = 0.01 * torch.sort(Dn.amin(1)).values[(k - 1) // 2]   # the median
            Wd = (sh > tgt).sum().clamp(min=W, max=max(k // 2, 1)).clamp(max=k - 1)
            srt = torch.sort(sh, descending=True).values
            tau = srt.gather(0, Wd.reshape(1))[0] if k > W else torch.zeros(
                (), dtype=torch.float64, device=dev)
            self.smax.copy_((tau * up).float().reshape(1))
            wild = sh > tau
            self.last_wild = Wd
        else:
            wild = torch.zeros(k, dtype=torch.bool, device=dev)
        Dw = torch.where(wild[None, :] & ~torch.eye(k, dtype=torch.bool, device=dev), Dlo,
                         torch.full_like(Dlo, float("inf")))
        self.mw[:k].copy_((Dw.amin(1) * dn).float())
        # centroid -> norm group (operand column order: perm, group starts)
        # (operand column order = the groups' contiguous tile ranges)
        Dp = Dhi.index_select(1, self.perm.long())
        Rc = torch.zeros((k, 4), dtype=torch.float64, device=dev)
        for g in range(self.G):
            c0 = min(64 * self.gstart[g], k)
            c1 = min(64 * self.gstart[g + 1], k) if g + 1 < self.G else k
            if c1 > c0:
                Rc[:, g] = Dp[:, c0:c1].amax(1)
        self.Rc[:k].copy_((Rc * up).float())
        self.C_prev = C32.clone()

    def set_centers(self, C32, cn=None):
        """The fp16 operand of the centroids SORTED by |c|^2 (``perm``: operand
        column -> centroid id): its tiles fall into G groups of contiguous
        norms, each with its own band per row (a narrower S range, a tighter
        band).  ``cn`` = the fp32 |c|^2 the E-step uses."""
        if cn is None:
            cn = (C32 * C32).sum(1)
        nt = self.k_pad // 64
        G = max(1, min(4, nt))
        order = torch.argsort(cn, stable=True)
        self.perm = order.to(torch.int32).contiguous()
        Cs = C32.index_select(0, order).contiguous()
        centers_to_f16_native(Cs, self.C_op, self.k, self.d, self.d_pad, self.k_pad, self.alpha)
        cs = cn.index_select(0, order)
        # the law's |c|^2 by operand column (the sweep's pair certificate)
        self.cns = torch.zeros(self.k_pad, dtype=torch.float32, device=cn.device)
        self.cns[:self.k].copy_(cs.float())
        lo_t = self.group_tiles(cs.double().cpu().numpy(), self.k, nt, G)
        hi_t = lo_t[1:] + [nt]
        # (views and a cat: no host -> device copy of the group indices)
        first = [min(64 * t, self.k - 1) for t in lo_t]
        last = [min(64 * t, self.k) - 1 for t in hi_t]
        self.gS = torch.stack([torch.cat([cs[f:f + 1] for f in first]),
                               torch.cat([cs[l:l + 1] for l in last])], 1)
        self.gS = self.gS.float().contiguous()
        self.G = G
        self.gstart = lo_t + [nt] * (4 - G)   # first tile of each group (unused: n_tiles)

    @staticmethod
    def group_tiles(cs, k, nt, G):
        """``group_tiles_np`` in the host library (``sqh_group_tiles``, the same
        fp64 expressions and ties): called once per IPE step while the GPU
        waits at the step boundary."""
        import ctypes
        from . import _host
        c = np.ascontiguousarray(cs, dtype=np.float64)
        out = (ctypes.c_int * max(int(G), 1))()
        rc = _host.lib().sqh_group_tiles(c.ctypes.data, int(k), int(nt), int(G), out)
        if rc:
            raise ValueError(f"sqh_group_tiles: bad arguments (k={k}, nt={nt}, G={G})")
        return [int(v) for v in out[:max(int(G), 1)]]

    @staticmethod
    def group_tiles_np(cs, k, nt, G):
        """First tile of each of the G norm groups: contiguous tile ranges of
        the sorted norms ``cs`` minimising sum_g (centroids in g) x (|c|^2
        range of g) - a row's band loses about its group's S range, so a few
        outlying norms get a small group of their own instead of widening a
        quarter of the centroids' range (dynamic programme over tile cuts)."""
        import numpy as np
        if G <= 1:
            return [0]
        lo = np.array([cs[min(64 * t, k - 1)] for t in range(nt)])
        hi = np.array([cs[min(64 * t + 63, k - 1)] for t in range(nt)])
        cnt = np.array([max(0, min(64, k - 64 * t)) for t in range(nt)], dtype=np.float64)
        ccnt = np.concatenate([[0.0], np.cumsum(cnt)])

        # cost[a, b] of tiles [a, b) (a < b), vectorised (a Python triple
        # loop cost ~0.2 ms of host time per IPE step)
        inf = float("inf")
        A = np.arange(nt + 1)
        valid = A[:, None] < A[None, :]
        hib = np.concatenate([[0.0], hi])          # hi[b - 1] at index b
        lo1 = np.concatenate([lo, [0.0]])
        cost = np.where(valid, (ccnt[None, :] - ccnt[:, None]) * (hib[None, :] - lo1[:, None]), inf)
        best = np.full((G + 1, nt + 1), inf)
        arg = np.zeros((G + 1, nt + 1), dtype=np.int64)
        best[0, 0] = 0.0
        for g in range(1, G + 1):
            tot = best[g - 1][:, None] + cost          # [a, b]
            tot[: g - 1, :] = inf                      # a >= g - 1
            arg[g] = np.argmin(tot, axis=0)            # first minimum: the loop's a order
            best[g] = tot[arg[g], A]
            best[g, :g] = inf
        cuts, b = [], nt
        for g in range(G, 0, -1):
            a = int(arg[g, b])
            cuts.append(a)
            b = a
        return sorted(cuts)

    def estep(self, X, C32, hint, xn, cn, labels, mind, eps, Q, key: RngKey, tie: RngKey,
              skey: RngKey, bkey: RngKey, row_offset, first, stats=None, fallback=None):
        """``hint`` (int32 [n]) is read (and, when ``first``, written by the
        argmin sweep first); ``fallback(rows, count, list_n, thr, hj, s, e)``
        runs the fp32 kernel over the dense rows of chunk [s, e)."""
        n = self.n
        if n == 0:
            return
        m = nat.native()
        st = nat.stream_handle(X.device)
        if first:
            self.lb_valid = False
        skip = self.skip
        if skip:
            self._skip_bounds(C32)
        # (numpy host arrays: see _skip_bounds)
        ia = np.zeros(72, dtype=np.int64)
        if self.gv:
            ia[65], ia[66] = self.V.data_ptr(), self.V.shape[0]
        ia[48] = self.perm.data_ptr()
        ia[60] = self.cns.data_ptr()
        ia[49] = self.gS.data_ptr()
        ia[50] = self.G
        ia[61], ia[62], ia[63] = self.gstart[1], self.gstart[2], self.gstart[3]
        da = np.array([float(eps), self.alpha, self.band_m(int(Q), min(self.ht, 9.0e-4)),
                       self.min_width], dtype=np.float64)
        ldx = X.stride(0)
        ia[1] = ldx
        ia[2] = C32.data_ptr()
        ia[4] = self.C_op.data_ptr()
        ia[8] = cn.data_ptr()
        ia[24] = 0 if stats is None else stats.data_ptr()
        ia[52] = 1 if (skip and self.lb_valid) else 0
        ia[53] = self.smax.data_ptr()
        ia[54] = self.Rc.data_ptr()
        ia[64] = self.mw.data_ptr()
        ia[26], ia[27], ia[28], ia[29], ia[30] = self.d, self.d_pad, self.k, self.k_pad, int(Q)
        for i, kk in ((32, key), (36, tie), (40, skey), (44, bkey)):
            ia[i], ia[i + 1], ia[i + 2], ia[i + 3] = kk.k0, kk.k1, kk.s0, kk.s1
        self.counts.zero_()
        iap, dap = ia.ctypes.data, da.ctypes.data
        last = self.nchunks - 1

        def run(op):
            rc = m.ipe16(op, iap, dap, st)
            if rc:
                raise RuntimeError(f"ipe16 op {op} failed (hip error {rc})")

        for c in range(self.nchunks):
            s, e = c * self.chunk, min(n, (c + 1) * self.chunk)
            ia[0] = X.data_ptr() + s * ldx * 4
            ia[3] = self.Xh.data_ptr() + s * self.d_pad * 2
            ia[5] = ia[6] = hint.data_ptr() + s * 4
            ia[7] = xn.data_ptr() + s * 4
            for i, t in ((9, self.thr), (10, self.hj), (11, self.vlo), (12, self.vhi),
                         (13, self.H), (14, self.rfire), (15, self.rst), (16, self.best),
                         (19, self.dense_rows), (21, self.rflag), (22, labels), (23, mind),
                         (51, self.lb), (55, self.lbo), (56, self.dhint), (59, self.ea2)):
                ia[i] = t.data_ptr() + s * t.stride(0) * t.element_size()
            if not skip:
                ia[51] = 0
            ia[17] = self.list.data_ptr()
            ia[18] = self.counts[c].data_ptr()
            ia[20] = self.counts[c].data_ptr() + 4
            ia[57] = self.rows.data_ptr()
            ia[58] = self.counts[c].data_ptr() + 8
            ia[25] = e - s
            ia[31] = int(row_offset) + s
            if first:
                run(1)
            run(0)
            run(2)
            if c == last:
                self.counts_host.copy_(self.counts, non_blocking=True)
                self.ev.record()
            run(3)
            run(4)
        # the bounds now hold for these labels (the next E-step's hints)
        self.lb_valid = skip
        self._last_args = (ia, da, st)   # the last chunk's launch arguments (benchmarks)
        self.ev.synchronize()
        dense = self.counts_host[:, 1].tolist()
        self.last_dense = int(sum(dense))
        parts = [(c, int(nd)) for c, nd in enumerate(dense) if nd > 0]
        if len(parts) == 1:
            c, nd = parts[0]
            s, e = c * self.chunk, min(n, (c + 1) * self.chunk)
            fallback(self.dense_rows[s:], self.counts[c, 1:2], nd, self.thr[s:e], self.hj[s:e],
                     s, e)
        elif parts:
            # the chunks' dense rows in ONE fallback launch over the shard (the
            # fp32 row-group kernel is latency-bound on a few rows: one launch
            # per chunk cost ~90 us each at steady state)
            tot = sum(nd for _, nd in parts)
            if getattr(self, "_dense_all", None) is None or self._dense_all.numel() < tot:
                self._dense_all = torch.empty(max(tot, 1024), dtype=self.dense_rows.dtype,
                                              device=self.dense_rows.device)
                self._dense_cnt = torch.zeros(1, dtype=torch.int32, device=self.dense_rows.device)
            off = 0
            for c, nd in parts:
                s = c * self.chunk
                torch.add(self.dense_rows[s:s + nd], s, out=self._dense_all[off:off + nd])
                off += nd
            self._dense_cnt.fill_(tot)
            fallback(self._dense_all, self._dense_cnt, tot, self.thr[:n], self.hj[:n], 0, n)
