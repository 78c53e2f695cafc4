"""Isolated E-step / M-step kernel timing (for rocprofv3 PMC runs)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch

from sq_learn_amd.ops import kmeans as K
from sq_learn_amd.ops import linalg as L
from sq_learn_amd.runtime.rng import RngKey

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--d", type=int, default=256)
ap.add_argument("--k", type=int, default=1024)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--delta", type=float, default=0.5)
ap.add_argument("--what", default="estep", choices=["estep", "reduce", "both"])
ap.add_argument("--prec", default="fp32", choices=["fp32", "bf16", "x64"])
ap.add_argument("--bounds", action="store_true", help="x64: write the Hamerly bounds too")
ap.add_argument("--stamps", action="store_true",
                help="x64 diagnostic variant (-DSQ_X64_STAMP=1 via SQ_NATIVE_VARIANT): "
                     "print the per-wave phase split of the last launch")
a = ap.parse_args()
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
C = torch.randn(a.k, a.d, device=dev, generator=g) * 3
X = torch.empty(a.n, a.d, dtype=torch.bfloat16 if a.prec == "bf16" else torch.float32, device=dev)
step = 1 << 20
for s in range(0, a.n, step):
    e = min(a.n, s + step)
    lab = torch.randint(0, a.k, (e - s,), device=dev, generator=g)
    X[s:e] = (C[lab] + torch.randn(e - s, a.d, device=dev, generator=g)).to(X.dtype)
kp, dp = K.pad_clusters(a.k), K.pad_features(a.d)
xn = L.row_norms_sq(X)
if a.prec == "bf16":
    Cb, cn = K.centers_to_bf16(C, kp, dp)
else:
    alpha = K.choose_alpha(float(xn.max()), 1.0)
    Cop = torch.empty(K.operand_f16_shape(kp, dp), dtype=torch.float16, device=dev)
    K.centers_to_f16_native(C, Cop, a.k, a.d, dp, kp, alpha)
    cmax2 = ((C.double() * alpha) ** 2).sum(1).max().float().reshape(1)
    Xh = (X * alpha).to(torch.float16)


def run_estep():
    if a.prec == "bf16":
        K.estep_native(X, Cb, cn, xn, a.k, a.delta, key, 0, buf)
    elif a.prec == "x64":
        K.estep_x64_native(Xh, X, Cop, C, xn, cmax2, a.k, a.delta, alpha, key, 0, buf,
                           bounds=bnd)
    else:
        K.estep_f32_native(X, Cop, xn, C, a.k, a.delta, alpha, key, 0, buf)

buf = K.EStepBuffers(a.n, dev)
bnd = ((torch.zeros(a.n, device=dev), torch.zeros(2 * a.n, device=dev))
       if a.bounds and a.prec == "x64" else None)
ws = K.ReduceWorkspace(a.n, a.k, dev).set_scale(float(X.float().abs().max()), a.n)
sums = torch.zeros(a.k, a.d, dtype=torch.float64, device=dev)
cnt = torch.zeros(a.k, dtype=torch.float64, device=dev)
key = RngKey(1, "band_select", 0)
run_estep()
torch.cuda.synchronize()
for name in (["estep", "reduce"] if a.what == "both" else [a.what]):
    t0 = time.perf_counter()
    for _ in range(a.iters):
        if name == "estep":
            run_estep()
        else:
            sums.zero_(); cnt.zero_()
            K.centroid_reduce_native(X, buf.labels, None, sums, cnt, a.k, ws)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.iters * 1e3
    fl = 2.0 * a.n * a.k * dp
    print(f"{a.prec} {name}: {ms:.3f} ms  ({fl / ms / 1e9:.1f} TFLOP/s equiv)  "
          f"counts(ovf,dense)={buf.counts.tolist()}")
if a.stamps:
    import ctypes
    import numpy as np
    lib = ctypes.CDLL(os.environ["SQ_NATIVE_VARIANT"])
    torch.cuda.synchronize()
    run_estep()
    torch.cuda.synchronize()
    buf_h = np.zeros((8192, 12), dtype=np.uint64)
    assert lib.sq_x64_stamps(ctypes.c_void_p(buf_h.ctypes.data), 8192) == 0
    w = buf_h[buf_h[:, 0] > 0].astype(np.float64)
    tot = w[:, 0].mean()
    names = ["total", "sweep", "tile sync", "first-tile sync", "row-set epilogue", "blocks",
             "stage() issue", "epilogue: min + cand lists", "A-load issue",
             "  - row min + T", "  - cand loop", "  - ub/lb + lgkm wait"]
    print(f"stamps over {len(w)} waves (shader cycles, mean per wave):")
    for i, nm in enumerate(names):
        v = w[:, i].mean()
        extra = "" if i in (0, 5) else f"  {100 * v / tot:.1f}% of total"
        per = "" if i == 5 else f"  {v / max(w[:, 5].mean(), 1):.0f} per block"
        print(f"  {nm:18s} {v:14.0f}{extra}{per}")

