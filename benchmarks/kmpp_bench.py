"""Device greedy k-means++ on the headline matrix (10M x 256 fp32, 1 GPU):
wall-clock per centre.  python benchmarks/kmpp_bench.py [--n N --k K]"""
import argparse
import time

import numpy as np
import torch

from sq_learn_amd.models._data import Data
from sq_learn_amd.models.cluster._init import kmeans_plusplus
from sq_learn_amd.parallel.comm import Comm
from sq_learn_amd.utils.datasets import make_blobs_device


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--k", type=int, default=64)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    X, _ = make_blobs_device(a.n, a.d, centers=1024, cluster_std=1.0, seed=1, device=dev,
                             dtype=torch.float32)
    data = Data(X, a.n, 0, Comm(None), "sharded")
    kmeans_plusplus(data, 4, np.random.RandomState(0))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kmeans_plusplus(data, a.k, np.random.RandomState(0))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"k-means++ n={a.n} d={a.d} k={a.k}: {el:.3f} s, {el / (a.k - 1) * 1e3:.3f} ms/centre")


if __name__ == "__main__":
    main()
