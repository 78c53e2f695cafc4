"""qPCA full fit with the quantum extras on the headline matrix (10M x 256
fp32, 1 GPU): wall-clock of the second (warm) fit.
python benchmarks/qpca_bench.py [--n N --d D --bf16 --lowrank --solver full|randomized]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from sq_learn_amd.models.decomposition import QPCA
from sq_learn_amd.parallel.comm import Comm
from sq_learn_amd.parallel.sharding import ShardedArray
from sq_learn_amd.utils.datasets import make_blobs_device


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--solver", default="full")
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--bf16", action="store_true")
    ap.add_argument("--true-tomography", action="store_true")
    ap.add_argument("--lowrank", action="store_true",
                    help="BASELINE config 2 data: low rank (32) + tail, as bench.py")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16 if a.bf16 else torch.float32
    if a.lowrank:
        from sq_learn_amd.utils.datasets import make_low_rank_device
        X = make_low_rank_device(a.n, a.d, effective_rank=32, tail_strength=0.3, seed=2024,
                                 device=dev, dtype=dt)
    else:
        X, _ = make_blobs_device(a.n, a.d, centers=1024, cluster_std=1.0, seed=1, device=dev,
                                 dtype=dt)
    sa = ShardedArray(X, a.n, 0, Comm(None))
    q = QPCA(n_components=16, svd_solver=a.solver, random_state=0, device=dev).fit(sa)
    theta = 0.5 * float(q.singular_values_[15])
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        q = QPCA(n_components=16, svd_solver=a.solver, random_state=0, device=dev,
                 quantum_truncated=a.solver != "full")
        q.fit(sa, eps=1e-3, theta_major=theta, delta=0.1, estimate_all=True,
              true_tomography=a.true_tomography)
        torch.cuda.synchronize()
        print(rep, f"qPCA {a.solver} fit {time.perf_counter() - t0:.3f} s", flush=True)
        ph = getattr(q, "fit_phases_", None)
        if ph:
            print("  phases (s):", {k: round(v, 4) for k, v in ph.items()},
                  "sum", round(sum(ph.values()), 4), flush=True)


if __name__ == "__main__":
    main()
