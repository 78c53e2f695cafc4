"""IPE E-step (``true_distance_estimate=True``, the reference default,
``_dmeans.py:753-772``) on the headline data: ms per Lloyd step and the
screen's pair statistics (csrc/ipe.hip ``stats``).

    python benchmarks/ipe_bench.py [--rows N --k K --steps S --center]

``--center`` subtracts the column means first (as QMeans.fit does before
its Lloyd loop)."""
import argparse
import os
import sys
import json
import time

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from sq_learn_amd.models._data import Data, gather_rows
from sq_learn_amd.models.cluster._lloyd import LloydEngine
from sq_learn_amd.parallel.comm import Comm
from sq_learn_amd.utils.datasets import make_blobs_device


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--delta", type=float, default=0.5)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--center", action="store_true")
    ap.add_argument("--seed", type=int, default=2024)
    a = ap.parse_args()
    dev = torch.device("cuda")
    X, _ = make_blobs_device(a.rows, a.d, centers=1024, cluster_std=1.0, seed=a.seed, device=dev,
                             dtype=torch.float32)
    if a.center:
        X -= X.mean(0, keepdim=True)
    comm = Comm(None)
    data = Data(X, a.rows, 0, comm, "sharded")
    C0 = gather_rows(data, np.random.RandomState(a.seed).choice(a.rows, a.k, replace=False))
    eng = LloydEngine(X, a.k, delta=a.delta, true_distance_estimate=True, intermediate_error=True,
                      true_tomography=False, seed=a.seed, comm=comm, gemm_precision="fp32")
    eng.set_centers(C0)
    eng.ipe_stats = torch.zeros(5, dtype=torch.int64, device=dev)
    eng.ipe16_stats = torch.zeros(8, dtype=torch.int64, device=dev)
    out = {"rows": a.rows, "k": a.k, "d": a.d, "center": a.center, "steps": []}
    names = ["screened", "full", "fires", "exact", "pass1_wgs"]
    names16 = ["near", "fired", "fired_exact", "dense_rows", "flagged_rows", "no_band_rows", "full",
               "skipped"]
    for s in range(a.steps + 1):
        eng.ipe_stats.zero_()
        eng.ipe16_stats.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.step()[1].tolist()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        st = dict(zip(names, eng.ipe_stats.tolist()))
        st16 = dict(zip(names16, eng.ipe16_stats.tolist()))
        i16 = getattr(eng, "_ipe16", None)
        tau = float(i16.smax.item()) if i16 is not None and i16.skip else None
        wild = getattr(i16, "last_wild", None) if i16 is not None else None
        wild = int(wild) if wild is not None else None
        out["steps"].append({"ms": round(ms, 2), "tau": tau, "wild": wild, **st,
                             **{"i16_" + k: v for k, v in st16.items()}})
        print(json.dumps(out["steps"][-1]), flush=True)
    # timed without stats (the production kernel)
    eng.ipe_stats = None
    eng.ipe16_stats = None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.step()[1].tolist()
    torch.cuda.synchronize()
    out["ms_per_step"] = (time.perf_counter() - t0) / a.steps * 1e3
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
