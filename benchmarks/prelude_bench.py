"""q-means fit prelude on the headline matrix (eta, mu(A) grid, sigma_min by
sharded fp64 CholeskyQR2): wall-clock per part, 1 GPU.
python benchmarks/prelude_bench.py [--n N --d D]"""
import argparse
import time

import torch

from sq_learn_amd.models._data import Data, best_mu_distributed, sigma_min
from sq_learn_amd.ops import linalg as L
from sq_learn_amd.parallel.comm import Comm
from sq_learn_amd.utils.datasets import make_blobs_device


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=256)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    X, _ = make_blobs_device(a.n, a.d, centers=1024, cluster_std=1.0, seed=1, device=dev,
                             dtype=torch.float32)
    data = Data(X, a.n, 0, Comm(None), "sharded")
    for rep in range(2):
        out = {}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rn = L.row_norms_sq(X).double()
        float(rn.max())
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        best_mu_distributed(data, 0.0, 0.1, 0.05, fro_sq=float(rn.sum()))
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        sigma_min(data)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        out = {"eta_ms": (t1 - t0) * 1e3, "mu_ms": (t2 - t1) * 1e3, "sigma_min_ms": (t3 - t2) * 1e3}
        print(rep, {k: round(v, 2) for k, v in out.items()}, flush=True)


if __name__ == "__main__":
    main()
