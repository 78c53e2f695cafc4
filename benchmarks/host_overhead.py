"""Host-side cost of one Lloyd iteration: time to enqueue ``eng.step()``
versus the full step including the convergence read-back (1 GPU).

    python benchmarks/host_overhead.py [--n 1250000]
"""
import argparse
import time

import numpy as np
import torch

from sq_learn_amd.models.cluster._lloyd import LloydEngine
from sq_learn_amd.utils.datasets import make_blobs_device


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_250_000)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    X, _ = make_blobs_device(a.n, a.d, centers=1024, cluster_std=1.0, seed=1, device=dev,
                             dtype=torch.bfloat16 if a.dtype == "bf16" else torch.float32)
    C0 = X[torch.from_numpy(np.random.RandomState(0).choice(a.n, a.k, replace=False)).to(dev)]
    eng = LloydEngine(X, a.k, delta=0.5, intermediate_error=True, seed=1, gemm_precision=a.dtype)
    eng.set_centers(C0.float())
    for _ in range(8):
        eng.step()[1].tolist()
    torch.cuda.synchronize()
    enq, tot = [], []
    for _ in range(a.steps):
        t0 = time.perf_counter()
        _, sc = eng.step()
        t1 = time.perf_counter()
        sc.tolist()
        t2 = time.perf_counter()
        enq.append(t1 - t0)
        tot.append(t2 - t0)
    print(f"n={a.n}: enqueue {np.median(enq) * 1e6:.1f} us, step {np.median(tot) * 1e6:.1f} us")


if __name__ == "__main__":
    main()
