"""Time the ipe16 screen sweep alone after a few Lloyd steps (1M x 256,
k = 1024 blobs), in variants: as is; no listed fires (rM = -1); no near
pairs either (every row all-far)."""
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


def t_op(st, op, reps=5):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        st.counts.zero_()
        st.relaunch(op)
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps, 3)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    d, k = 256, 1024
    dev = torch.device("cuda")
    X, _ = make_blobs_device(n, d, centers=1024, cluster_std=1.0, seed=2024, device=dev,
                             dtype=torch.float32)
    C0 = gather_rows(Data(X, n, 0, Comm(None), "sharded"),
                     np.random.RandomState(2024).choice(n, k, replace=False))
    eng = LloydEngine(X, k, delta=0.5, true_distance_estimate=True, intermediate_error=True,
                      seed=2024, comm=Comm(None))
    eng.set_centers(C0)
    for _ in range(5):
        eng.step()[1].tolist()
    st = eng._ipe16
    out = {"prep": t_op(st, 0), "sweep": t_op(st, 2), "near": t_op(st, 3), "argmin": t_op(st, 1)}
    st.rfire[:, 0].zero_()
    out["sweep_no_fires"] = t_op(st, 2)
    st.vlo.fill_(-float("inf"))
    st.vhi.fill_(float("inf"))
    out["sweep_no_fires_no_near"] = t_op(st, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
