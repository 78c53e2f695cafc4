"""ipe16 vs the fp32 fused IPE kernel on the same Lloyd trajectory start:
per-step inertia, label agreement with the exact argmin, screen statistics."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from sq_learn_amd.models._data import Data, gather_rows  # noqa: E402
from sq_learn_amd.models.cluster._lloyd import LloydEngine  # noqa: E402
from sq_learn_amd.parallel.comm import Comm  # noqa: E402
from sq_learn_amd.utils.datasets import make_blobs_device  # noqa: E402


def run(X, C0, k, use16, steps):
    os.environ["SQ_IPE16"] = "1" if use16 else "0"
    eng = LloydEngine(X, k, delta=0.5, true_distance_estimate=True, intermediate_error=True,
                      seed=3, comm=Comm(None))
    eng.set_centers(C0)
    eng.ipe16_stats = torch.zeros(8, dtype=torch.int64, device=X.device)
    out = []
    for s in range(steps):
        eng.ipe16_stats.zero_()
        C = eng.centers().clone()
        lab, sc = eng.step()
        vals = sc.tolist()
        D = torch.cdist(X[:20000].double(), C.double())
        agree = float((D.argmin(1) == lab[:20000].long()).double().mean())
        out.append({"inertia": vals[0], "agree_argmin": round(agree, 4),
                    "stats": eng.ipe16_stats.tolist()})
    return out


def main():
    n, d, k = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000, 64, 256
    dev = torch.device("cuda")
    X, _ = make_blobs_device(n, d, centers=k, cluster_std=1.0, seed=1, device=dev,
                             dtype=torch.float32)
    C0 = gather_rows(Data(X, n, 0, Comm(None), "sharded"),
                     np.random.RandomState(1).choice(n, k, replace=False))
    for use16 in (False, True):
        for r in run(X, C0, k, use16, 4):
            print(json.dumps({"ipe16": use16, **r}), flush=True)


if __name__ == "__main__":
    main()
