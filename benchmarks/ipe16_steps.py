"""ipe16 over Lloyd steps on the bench data (blobs, random-row init): per
step ms and screen statistics; at the last step, a few dense rows in detail
(threshold, band, nearest distances)."""
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    d, k = 256, 1024
    dev = torch.device("cuda")
    X, _ = make_blobs_device(n, d, centers=1024, cluster_std=1.0, seed=2024, device=dev,
                             dtype=torch.float32)
    C0 = gather_rows(Data(X, n, 0, Comm(None), "sharded"),
                     np.random.RandomState(2024).choice(n, k, replace=False))
    eng = LloydEngine(X, k, delta=0.5, true_distance_estimate=True, intermediate_error=True,
                      seed=2024, comm=Comm(None))
    eng.set_centers(C0)
    eng.ipe16_stats = torch.zeros(8, dtype=torch.int64, device=dev)
    names = ["near", "fired", "fired_exact", "dense", "flagged", "no_band", "full"]
    for s in range(steps):
        eng.ipe16_stats.zero_()
        C = eng.centers().clone()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lab, sc = eng.step()
        vals = sc.tolist()
        ms = (time.perf_counter() - t0) * 1e3
        print(json.dumps({"step": s, "ms": round(ms, 2), "inertia": vals[0],
                          **dict(zip(names, eng.ipe16_stats.tolist()))}), flush=True)
    st = eng._ipe16
    rf = st.rflag[:n].cpu().numpy()
    rs = st.rst[:n].cpu().numpy()
    ovf = np.where((rf != 0) & (rs == 0))[0]
    nob = np.where(rs != 0)[0]
    print(json.dumps({"overflow_rows": int(len(ovf)), "no_band_rows": int(len(nob))}))
    xn = (X.double() ** 2).sum(1)
    for r in list(ovf[:5]) + list(nob[:3]):
        D = ((X[r].double()[None] - C.double()) ** 2).sum(1)
        ds = torch.sort(D).values.cpu().numpy()
        a2 = st.alpha ** 2
        print(json.dumps({"row": int(r), "thr": float(st.thr[r]), "hint": int(st.hj[r]),
                          "D_hint": float(D[int(st.hj[r])]) if st.hj[r] >= 0 else None,
                          "Dl": float(st.vlo[r, 0]) / a2 + float(xn[r]),
                          "Dh": float(st.vhi[r, 0]) / a2 + float(xn[r]),
                          "D_sorted": [round(float(v), 1) for v in ds[:6]],
                          "D_q10": float(np.quantile(ds, 0.1)), "D_max": float(ds[-1])}))


if __name__ == "__main__":
    main()
