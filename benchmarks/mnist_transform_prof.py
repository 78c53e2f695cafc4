"""Where the MNIST-pipeline quantum transform (qPCA(61) -> tomography of the
70k projected rows, error 0.8) spends its time: wall per call and a cProfile
of the second call (host side)."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "examples")))
from mnist_pipeline import mnist_like  # noqa: E402
from sq_learn_amd.decomposition import qPCA  # noqa: E402


def main():
    X, y = mnist_like(70_000, device="cuda")
    pca = qPCA(svd_solver="full", device="cuda")
    pca.n_components = 61
    m = pca.fit(X)
    torch.cuda.synchronize()

    def tr():
        r = m.transform(X, classic_transform=False, epsilon_delta=0.8,
                        quantum_representation=True, norm="est_representation", tomography=True)
        torch.cuda.synchronize()
        return r
    for i in range(3):
        t = time.perf_counter()
        tr()
        print(f"transform {i}: {time.perf_counter() - t:.4f} s", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    tr()
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(30)


if __name__ == "__main__":
    main()
