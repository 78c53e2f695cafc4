"""Device greedy k-means++ on the headline matrix (10M x 256 fp32, 1 GPU):
wall-clock per centre, with the screens (triangle + certified int8 bound)
on and off, and the mean survivor / exact-row fractions.
python benchmarks/kmpp_bench.py [--n N --k K --center --no-unpruned]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from sq_learn_amd.models._data import Data
from sq_learn_amd.models.cluster._init import kmeans_plusplus
from sq_learn_amd.parallel.comm import Comm
from sq_learn_amd.utils.datasets import make_blobs_device


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--center", action="store_true")
    ap.add_argument("--no-unpruned", action="store_true")
    ap.add_argument("--full-stats", action="store_true",
                    help="survivor / exact fractions over all k centres (by quarter)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    X, _ = make_blobs_device(a.n, a.d, centers=1024, cluster_std=1.0, seed=1, device=dev,
                             dtype=torch.float32)
    if a.center:
        X -= X.mean(0, keepdim=True)
    data = Data(X, a.n, 0, Comm(None), "sharded")
    kmeans_plusplus(data, 4, np.random.RandomState(0))
    torch.cuda.synchronize()
    ids = {}
    for prune in ((True,) if a.no_unpruned else (True, False)):
        stats = []
        t0 = time.perf_counter()
        _, ids[prune] = kmeans_plusplus(data, a.k, np.random.RandomState(0), prune=prune)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        kmeans_plusplus(data, a.k if a.full_stats else min(a.k, 64), np.random.RandomState(0),
                        prune=prune, stats=stats)
        st = np.asarray(stats, dtype=np.float64) / a.n
        if a.full_stats and len(st) >= 4:
            q = np.array_split(st, 4)
            print("survivor / exact frac by quarter of the centres:",
                  [(round(float(x[:, 0].mean()), 4), round(float(x[:, 1].mean()), 4)) for x in q],
                  "all:", round(float(st[:, 0].mean()), 4), round(float(st[:, 1].mean()), 4),
                  flush=True)
            st = st[:64]
        print(f"k-means++ prune={prune} n={a.n} d={a.d} k={a.k}: {el:.3f} s, "
              f"{el / max(a.k - 1, 1) * 1e3:.3f} ms/centre; first 64 centres: survivor frac "
              f"{st[:, 0].mean():.3f}, exact frac {st[:, 1].mean():.3f}", flush=True)
    if len(ids) == 2:
        print("ids identical:", bool(np.array_equal(ids[True], ids[False])))


if __name__ == "__main__":
    main()
