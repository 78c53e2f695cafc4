"""What the ipe16 screen's listed NEAR pairs are (bench shape, steady state):
for a sample of the last chunk's listed near pairs, the pair's distance
against its row's far band [Dl, Dh] (the band edges back in D units), the
pair's own bin distance m (ipe_hazard's formula, fp64) against the band's
m_t, and whether it is below / above the band."""
import json
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from sq_learn_amd.models._data import Data, gather_rows  # noqa: E402
from sq_learn_amd.models.cluster._lloyd import LloydEngine  # noqa: E402
from sq_learn_amd.ops import kmeans as K  # noqa: E402
from sq_learn_amd.parallel.comm import Comm  # noqa: E402
from sq_learn_amd.utils.datasets import make_blobs_device  # noqa: E402


def q(t, ps=(0.01, 0.1, 0.5, 0.9, 0.99)):
    t = t.double()
    t = t[torch.isfinite(t)]
    if t.numel() == 0:
        return []
    return [round(float(v), 3) for v in torch.quantile(t.float(), torch.tensor(ps, device=t.device))]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    d, k, seed = 256, 1024, 2024
    dev = torch.device("cuda")
    X, _ = make_blobs_device(n, d, centers=1024, cluster_std=1.0, seed=seed, device=dev,
                             dtype=torch.float32)
    C0 = gather_rows(Data(X, n, 0, Comm(None), "sharded"),
                     np.random.RandomState(seed).choice(n, k, replace=False))
    eng = LloydEngine(X, k, delta=0.5, true_distance_estimate=True, intermediate_error=True,
                      true_tomography=False, seed=seed, comm=Comm(None), gemm_precision="fp32")
    eng.set_centers(C0)
    for s in range(steps):
        C = eng.centers().clone().double()
        eng.step()[1].tolist()
    st = eng._ipe16
    c = st.nchunks - 1
    s0 = c * K.IPE16_CHUNK
    cnt = int(st.counts[c, 0])
    ent = st.list[:cnt]
    rows = (ent >> 16) + s0
    j = (ent & 0x3FFF).long()
    near = (ent & 0x4000) != 0
    fired = (ent & 0x8000) != 0
    sel = torch.nonzero(near).flatten()
    sel = sel[torch.randperm(sel.numel(), device=dev)[:200000]]
    r, jj = rows[sel], j[sel]
    x = X[r].double()
    cc = C[jj]
    ip = (x * cc).sum(1)
    nx2, ny2 = (x * x).sum(1), (cc * cc).sum(1)
    S = nx2 + ny2
    D = S - 2 * ip
    thr = st.thr[r].double()
    eps = eng.delta / 2
    kq = 1 / (math.sqrt(2) * eps)
    m = (D.clamp_min(0).sqrt() * (1 - 4.8828125e-4) - thr.clamp_min(0).sqrt()) * S.sqrt() * kq \
        / ip.abs().clamp_min(1)
    mt = K.Ipe16.band_m(13, min(st.ht, 9e-4))
    # the pair's group band, back in D units
    col = torch.empty(k, dtype=torch.long, device=dev)
    col[st.perm.long()] = torch.arange(k, device=dev)
    grp = ((col[jj] // 64) * st.G) // (st.k_pad // 64)
    a2 = st.alpha ** 2
    vlo = st.vlo[r].double().gather(1, grp[:, None])[:, 0]
    vhi = st.vhi[r].double().gather(1, grp[:, None])[:, 0]
    Dl = vlo / a2 + nx2
    Dh = vhi / a2 + nx2
    below = D < Dl
    above = D > Dh
    rec = {"listed": cnt, "near": int(near.sum()), "fired": int(fired.sum()),
           "both": int((near & fired).sum()), "mt": mt,
           "below_frac": float(below.double().mean()), "above_frac": float(above.double().mean()),
           "inside_frac": float((~below & ~above).double().mean()),
           "m_over_mt_q(below)": q((m / mt)[below]), "m_over_mt_q(above)": q((m / mt)[above]),
           "m_ge_mt_frac(below)": float((m[below] >= mt).double().mean()),
           "sqrtD_minus_sqrtDl_q(below)": q((D.clamp_min(0).sqrt() - Dl.clamp_min(0).sqrt())[below]),
           "sqrtDl_q": q(Dl.clamp_min(0).sqrt()), "sqrtthr_q": q(thr.clamp_min(0).sqrt()),
           "sqrtD_q(below)": q(D.clamp_min(0).sqrt()[below]),
           "Dh_minus_Dl_over_Dl_q": q(((Dh - Dl) / Dl)),
           "a_q(above)": q((D / (2 * S))[above]),
           "per_row_near_q": q(torch.bincount(rows[near] - s0).double())}
    print(json.dumps(rec), flush=True)




def model_band(nx2, sthr, Smin, Smax, eps, mt):
    """row_cut (csrc/ipe16.hip) in torch fp64, no rounding margins: (Dl, Dh)."""
    kq = 1 / (math.sqrt(2) * eps)
    c = 1 - 4.8828125e-4
    ylo = (Smax * 2 ** -12).sqrt()
    yhi = (Smin * 1.998046875).sqrt()
    for S in (Smin, Smax):
        rS = S.sqrt()
        B = 2 * kq * rS * c
        C0 = 2 * kq * rS * sthr
        a = mt
        y0 = (mt / (kq * rS) + sthr) / c
        yA = (-B + (B * B + 4 * a * (a * S + C0)).sqrt()) / (2 * a)
        dB = B * B - 4 * a * (C0 - a * S)
        yB = (B + dB.clamp_min(0).sqrt()) / (2 * a)
        yBm = (B - dB.clamp_min(0).sqrt()) / (2 * a)
        ylo = torch.maximum(ylo, torch.maximum(y0, torch.maximum(yA, yBm)))
        yhi = torch.minimum(yhi, yB)
    return ylo ** 2, yhi ** 2


def band_check(n=4_000_000, steps=5):
    d, k, seed = 256, 1024, 2024
    dev = torch.device("cuda")
    X, _ = make_blobs_device(n, d, centers=1024, cluster_std=1.0, seed=seed, device=dev,
                             dtype=torch.float32)
    C0 = gather_rows(Data(X, n, 0, Comm(None), "sharded"),
                     np.random.RandomState(seed).choice(n, k, replace=False))
    eng = LloydEngine(X, k, delta=0.5, true_distance_estimate=True, intermediate_error=True,
                      true_tomography=False, seed=seed, comm=Comm(None), gemm_precision="fp32")
    eng.set_centers(C0)
    for s in range(steps):
        eng.step()[1].tolist()
    st = eng._ipe16
    sub = torch.arange(0, n, n // 4000, device=dev)[:4000]
    ok = (st.rst[sub] == 0)
    sub = sub[ok]
    nx2 = eng._ipe_xn[sub].double()
    sthr = st.thr[sub].double().sqrt() * 1.000001
    a2 = st.alpha ** 2
    mt = K.Ipe16.band_m(13, min(st.ht, 9e-4))
    out = {"G": st.G, "gS": st.gS.tolist(), "mt": mt}
    for g in range(st.G):
        Smin = nx2 + float(st.gS[g, 0])
        Smax = nx2 + float(st.gS[g, 1])
        Dl, Dh = model_band(nx2, sthr, Smin, Smax, eng.delta / 2, mt)
        kDl = st.vlo[sub, g].double() / a2 + nx2
        kDh = st.vhi[sub, g].double() / a2 + nx2
        fin = torch.isfinite(kDl)
        out[f"g{g}"] = {"finite": float(fin.double().mean()),
                        "sqrt_kDl_q": q(kDl[fin].clamp_min(0).sqrt()),
                        "sqrt_mDl_q": q(Dl[fin].clamp_min(0).sqrt()),
                        "sqrt_kDh_q": q(kDh[fin].clamp_min(0).sqrt()),
                        "sqrt_mDh_q": q(Dh[fin].clamp_min(0).sqrt())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[3] == "band":
        band_check(int(sys.argv[1]), int(sys.argv[2]))
    else:
        main()
