"""Simulated estimation failure with optional resampling.

The reference's failure model is implicit (AE/PE tails, median boosting,
Ta-Shma's gamma).  ``failure_prob`` makes it explicit: each row's distance
estimation fails with probability ``p``; policy ``'ignore'`` keeps the
corrupted outcome (the label becomes a uniformly random centroid),
``'resample'`` repeats a failed estimation up to ``max_attempts`` times, so
a row is corrupted with probability ``p ** max_attempts`` and the expected
cost grows by ``(1 - p**R) / (1 - p)`` estimations per row.

One HIP kernel on the device (``csrc/failure.hip``); the torch twin below
produces bit-identical labels on CPU (same Philox words, same fp32 math).
"""

import torch

from ..runtime.rng import Philox, RngKey, uniform_from_u32
from . import _native as nat


def _keys(key: RngKey):
    # outlier labels come from a separate sub-stream of the same purpose
    return key, key.derive(sub=(key.stream & ((1 << 48) - 1)) | (1 << 47))


def failure_inject_(labels, k, p, attempts, key: RngKey, row_offset, counters, lb=None,
                    corr=None, X=None, C=None, mind=None):
    """In place on int32/int64 ``labels``; ``counters`` (int64[2] on the same
    device) += [estimations made, corrupted rows].  Device only: ``lb`` (fp32
    [n], the Hamerly lower bounds) is zeroed on corrupted rows, and ``corr``
    (fp32 [n], the incremental M-step's min-vs-label corrections) moves with
    the label: += |x - C[old]|^2 - |x - C[new]|^2 (``X`` fp32 rows, ``C`` fp32
    centres of the E-step); ``mind`` (fp32 [n]): a corrupted row whose min
    distance is still unfilled (< 0) gets |x - C[old]|^2."""
    n = labels.numel()
    if n == 0 or p <= 0:
        if n:
            counters[0] += n
        return labels
    k1, k2 = _keys(key)
    if nat.use_native(labels) and labels.dtype == torch.int32:
        need = corr is not None or mind is not None
        if need:
            assert X is not None and C is not None and X.dtype == torch.float32
            assert C.dtype == torch.float32 and X.stride(1) == 1 and C.stride(1) == 1
        d = min(X.shape[1], C.shape[1]) if need else 0
        nat.native().failure_inject(labels.data_ptr(), n, int(k), float(p), int(attempts),
                                    k1.k0, k1.k1, k1.s0, k1.s1, k2.k0, k2.k1, k2.s0, k2.s1,
                                    int(row_offset), counters.data_ptr(),
                                    0 if lb is None else lb.data_ptr(),
                                    0 if corr is None else corr.data_ptr(),
                                    0 if mind is None else mind.data_ptr(),
                                    X.data_ptr() if need else 0, X.stride(0) if need else 0,
                                    C.data_ptr() if need else 0, C.stride(0) if need else 0,
                                    int(d),
                                    nat.stream_handle(labels.device))
        return labels
    dev = labels.device
    R = int(attempts)
    g = torch.arange(row_offset, row_offset + n, dtype=torch.int64, device=dev)
    ph = Philox(k1)
    ok = torch.zeros(n, dtype=torch.bool, device=dev)
    made = torch.zeros(n, dtype=torch.int64, device=dev)
    pf = torch.tensor(p, dtype=torch.float32)
    for r in range(R):
        e = g * R + r
        w = ph.u32x4(e >> 2)
        word = torch.stack(w, 1).gather(1, (e & 3)[:, None])[:, 0]
        u = uniform_from_u32(word, torch.float32)
        made += (~ok).to(torch.int64)
        ok |= u >= pf.to(dev)
    bad = ~ok
    if bool(bad.any()):
        w = Philox(k2).u32x4(g >> 2)
        word = torch.stack(w, 1).gather(1, (g & 3)[:, None])[:, 0]
        u = uniform_from_u32(word, torch.float32)
        lab = torch.floor(u * torch.tensor(float(k), dtype=torch.float32)).to(torch.int64)
        lab = lab.clamp(max=k - 1)
        labels[bad] = lab[bad].to(labels.dtype)
    counters[0] += int(made.sum())
    counters[1] += int(bad.sum())
    return labels
