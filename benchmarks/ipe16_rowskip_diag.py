"""Where the ipe16 screen's near pairs come from, and how many rows a
row-level skip could drop (bench config: 10M x 256, k = 1024, 1024 blobs).

After each IPE step, on a row subsample: the row's far band (prep's
vlo / vhi per centroid group, fp16-filter units v = alpha^2 (|c|^2 - 2 x.c)),
every pair's v from an fp64 inner product, the hint (that step's input
labels) excluded: counts of near-low (v < vlo) / near-high (v > vhi) pairs,
the fraction of rows with none (the rows a skip could drop), and the slack
sqrt(min_{j != hint} D_j) - sqrt(D at the band's low edge) of those rows."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from sq_learn_amd.models._data import Data, gather_rows  # noqa: E402
from sq_learn_amd.models.cluster._lloyd import LloydEngine  # noqa: E402
from sq_learn_amd.parallel.comm import Comm  # noqa: E402
from sq_learn_amd.utils.datasets import make_blobs_device  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    d, k, seed = 256, 1024, 2024
    dev = torch.device("cuda")
    X, _ = make_blobs_device(n, d, centers=1024, cluster_std=1.0, seed=seed, device=dev,
                             dtype=torch.float32)
    C0 = gather_rows(Data(X, n, 0, Comm(None), "sharded"),
                     np.random.RandomState(seed).choice(n, k, replace=False))
    eng = LloydEngine(X, k, delta=0.5, true_distance_estimate=True, intermediate_error=True,
                      true_tomography=False, seed=seed, comm=Comm(None), gemm_precision="fp32")
    eng.set_centers(C0)
    eng.ipe16_stats = torch.zeros(8, dtype=torch.int64, device=dev)
    sub = torch.arange(0, n, max(1, n // 20000), device=dev)[:20000]
    for s in range(steps):
        C = eng.centers().clone().double()
        eng.ipe16_stats.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lab, sc = eng.step()
        sc.tolist()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        st = eng._ipe16
        hint = eng._ipe_lab[eng._ipe_cur ^ 1][sub].long()
        Xs = X[sub].double()
        a2 = st.alpha ** 2
        cn = (C * C).sum(1)
        xn = (Xs * Xs).sum(1)
        v = a2 * (cn[None, :] - 2.0 * Xs @ C.T)                   # [m][k]
        D = xn[:, None] + cn[None, :] - 2.0 * Xs @ C.T
        perm = st.perm.long()
        nt = st.k_pad // 64
        col = torch.empty(k, dtype=torch.long, device=dev)
        col[perm] = torch.arange(k, device=dev)
        grp = ((col // 64) * st.G) // nt                          # centroid -> group
        vlo = st.vlo[sub].double()[:, :4].gather(1, grp[None, :].expand(len(sub), k))
        vhi = st.vhi[sub].double()[:, :4].gather(1, grp[None, :].expand(len(sub), k))
        nh = torch.ones_like(v, dtype=torch.bool)
        valid = hint >= 0
        nh[valid, hint[valid]] = False
        low = (v < vlo) & nh
        high = (v > vhi) & nh
        band = torch.isfinite(st.vlo[sub, 0]) & (st.rst[sub] == 0)
        n_low, n_high = low.sum(1).double(), high.sum(1).double()
        none = band & (n_low == 0) & (n_high == 0)
        Dm = torch.where(nh, D, torch.full_like(D, float("inf"))).min(1).values
        # D at the low edge of the band of the nearest non-hint centroid's group
        edge = (vlo.min(1).values / a2 + xn)
        slack = (Dm.clamp_min(0).sqrt() - edge.clamp_min(0).sqrt())[none]
        q = [float(x) for x in torch.quantile(slack.float(), torch.tensor(
            [0.01, 0.1, 0.5], device=dev))] if none.any() else []
        rec = {"step": s, "ms": round(ms, 2), "band_rows": float(band.double().mean()),
               "near_low_per_row": float(n_low.mean()), "near_high_per_row": float(n_high.mean()),
               "rows_no_near": float(none.double().mean()),
               "rows_low_only": float((band & (n_low > 0) & (n_high == 0)).double().mean()),
               "rows_high_only": float((band & (n_low == 0) & (n_high > 0)).double().mean()),
               "slack_q01_q10_q50": q,
               "label_is_argmin": float((lab[sub].long() == D.argmin(1)).double().mean()),
               "hint_is_argmin": float((hint == D.argmin(1)).double().mean()),
               "stats": eng.ipe16_stats.tolist()}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
