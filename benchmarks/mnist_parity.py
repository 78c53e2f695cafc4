#!/usr/bin/env python
"""BASELINE config 4: classical PCA + KMeans parity on an MNIST-shaped
matrix (70k x 784), framework (MI355X) vs scikit-learn (host CPU).

    python benchmarks/mnist_parity.py [--n 70000] [--k 10] [--components 61]

Checks that explained variances match and that the k-means inertias agree
(same k-means++ seeds are not comparable across implementations, so the
best-of-n_init inertia is compared with a tolerance) and reports both
wall-clocks.  Synthetic data (no network): see examples/mnist_pipeline.py.
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "examples")))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=70_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--components", type=int, default=61)
    ap.add_argument("--n-init", type=int, default=4)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--skip-sklearn", action="store_true")
    a = ap.parse_args()
    from mnist_pipeline import mnist_like
    from sq_learn_amd.cluster import KMeans
    from sq_learn_amd.decomposition import PCA

    X, _ = mnist_like(a.n, device=a.device)
    out = {"metric": "PCA+KMeans parity (MNIST-shape)", "n": a.n, "d": X.shape[1],
           "device": a.device}
    torch.cuda.synchronize() if a.device != "cpu" else None
    t = time.perf_counter()
    p = PCA(n_components=a.components, svd_solver="full", device=a.device).fit(X)
    Z = p.transform(X)
    km = KMeans(a.k, n_init=a.n_init, random_state=0, device=a.device).fit(Z)
    torch.cuda.synchronize() if a.device != "cpu" else None
    out["ours_s"] = time.perf_counter() - t
    out["ours_inertia"] = km.inertia_
    out["ours_evr_sum"] = float(np.sum(p.explained_variance_ratio_))
    if not a.skip_sklearn:
        import sklearn.cluster as skc
        import sklearn.decomposition as skd
        Xh = X.cpu().numpy().astype(np.float64)
        t = time.perf_counter()
        sp = skd.PCA(n_components=a.components, svd_solver="full").fit(Xh)
        sZ = sp.transform(Xh)
        sk = skc.KMeans(a.k, n_init=a.n_init, random_state=0).fit(sZ)
        out["sklearn_s"] = time.perf_counter() - t
        out["sklearn_inertia"] = float(sk.inertia_)
        out["sklearn_evr_sum"] = float(np.sum(sp.explained_variance_ratio_))
        out["evr_max_abs_diff"] = float(np.max(np.abs(sp.explained_variance_ratio_ -
                                                      p.explained_variance_ratio_)))
        out["inertia_rel_diff"] = abs(out["ours_inertia"] - out["sklearn_inertia"]) / \
            out["sklearn_inertia"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
