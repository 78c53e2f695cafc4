#!/usr/bin/env python
"""End-to-end example mirroring the reference's driver ``sklearn/MnistTrial.py``
(SURVEY.md E7): qPCA(61) on an MNIST-shaped matrix -> quantum representation
of the projected data (tomography with error epsilon_delta) -> 7-NN scored by
10-fold stratified cross-validation.

There is no network here, so instead of ``fetch_openml('mnist_784')`` the
data is a synthetic MNIST-shaped stand-in (70k x 784, 10 classes, pixel-like
non-negative features with low-rank class structure), generated on the
device.  Everything runs on the MI355X when one is present: the qPCA Gram
kernel + eigh, the batched tomography, the KNN distance GEMM + top-k kernel.

    python examples/mnist_pipeline.py [--n 70000] [--error 0.8] [--device cuda]
"""

import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

from sq_learn_amd.decomposition import qPCA  # noqa: E402
from sq_learn_amd.model_selection import StratifiedKFold, cross_validate  # noqa: E402
from sq_learn_amd.neighbors import KNeighborsClassifier  # noqa: E402
from sq_learn_amd.runtime.rng import RngKey  # noqa: E402
from sq_learn_amd.ops.random import philox_normal  # noqa: E402


def mnist_like(n, d=784, classes=10, rank=40, seed=0, device="cpu"):
    """Non-negative 'images': per class a low-rank template mixture + noise."""
    dev = torch.device(device)
    bases = philox_normal((classes, rank, d), RngKey(seed, "data", 11), dtype=torch.float32,
                          device=dev)
    y = torch.arange(n, device=dev) % classes
    coef = philox_normal((n, rank), RngKey(seed, "data", 12), dtype=torch.float32, device=dev)
    X = torch.einsum("nr,nrd->nd", coef, bases[y]) / np.sqrt(rank)
    X = X + 0.5 * philox_normal((n, d), RngKey(seed, "data", 13), dtype=torch.float32, device=dev)
    X = torch.relu(X) * 64.0       # pixel-like range
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(seed)).to(dev)
    return X[perm], y[perm].cpu().numpy()


def run(n=70_000, error=0.8, components=61, folds=10, device="cpu", preserve_norm=False,
        classic=True):
    """The pipeline; returns accuracies and per-stage seconds (also the
    bench.py ``mnist_pipeline_*`` extra)."""
    def sync():
        if str(device).startswith("cuda"):
            torch.cuda.synchronize()

    X, y = mnist_like(n, device=device)
    sync()
    t0 = time.perf_counter()
    pca = qPCA(svd_solver="full", device=device, preserve_norm_tomography=preserve_norm)
    pca.n_components = components
    pca_model = pca.fit(X)
    sync()
    t_fit = time.perf_counter() - t0
    # Transform the features: quantum representation with tomography error
    t0 = time.perf_counter()
    X_train_pca = pca_model.transform(X, classic_transform=False, epsilon_delta=error,
                                      quantum_representation=True, norm="est_representation",
                                      tomography=True)
    sync()
    t_tr = time.perf_counter() - t0
    est, eps_used, f_norm = X_train_pca["quantum_representation_results"]
    knn = KNeighborsClassifier(n_neighbors=7, device=device)
    t0 = time.perf_counter()
    score = cross_validate(knn, est, y, cv=StratifiedKFold(n_splits=folds, shuffle=True,
                                                          random_state=1234))
    sync()
    t_cv = time.perf_counter() - t0
    out = dict(accuracy=float(np.average(score["test_score"])), f_norm=float(f_norm),
               qpca_fit_s=t_fit, transform_s=t_tr, cv_s=t_cv, total_s=t_fit + t_tr + t_cv)
    if classic:
        c = cross_validate(KNeighborsClassifier(n_neighbors=7, device=device),
                           pca_model.transform(X), y,
                           cv=StratifiedKFold(n_splits=folds, shuffle=True, random_state=1234))
        out["classic_accuracy"] = float(np.average(c["test_score"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=70_000)
    ap.add_argument("--error", type=float, default=0.8)
    ap.add_argument("--components", type=int, default=61)
    ap.add_argument("--folds", type=int, default=10)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--preserve-norm", action="store_true",
                    help="rescale tomography rows to the true row norms (the reference's real "
                         "tomography returns unit rows, Utility.py:171-176)")
    a = ap.parse_args()
    r = run(a.n, a.error, a.components, a.folds, a.device, a.preserve_norm)
    print(f"{a.folds}-fold Cross-validation - Estimated UE")
    print(f"(delta + epsilon): {a.error}")
    print(f"Error-F_norm-Accuracy: {[[a.error, r['f_norm'], r['accuracy']]]}")
    print(f"classical-representation accuracy: {r['classic_accuracy']:.4f}")
    print(f"timings: qPCA fit {r['qpca_fit_s']:.2f}s, quantum transform {r['transform_s']:.2f}s, "
          f"CV {r['cv_s']:.2f}s on {a.device}")


if __name__ == "__main__":
    main()
