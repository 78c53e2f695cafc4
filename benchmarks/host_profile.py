"""Python-side cost of the steady-state Lloyd step (GPU fast path): cProfile
of N enqueued steps at a 1.25M-row shard (the N=8 per-GPU share), sorted by
own time.  python benchmarks/host_profile.py [--n 1250000 --steps 200]"""
import argparse
import cProfile
import pstats

import numpy as np
import torch

from sq_learn_amd.models.cluster._lloyd import LloydEngine
from sq_learn_amd.utils.datasets import make_blobs_device


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_250_000)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    X, _ = make_blobs_device(a.n, 256, centers=1024, cluster_std=1.0, seed=1, device=dev,
                             dtype=torch.float32)
    C0 = X[torch.from_numpy(np.random.RandomState(0).choice(a.n, 1024, replace=False)).to(dev)]
    eng = LloydEngine(X, 1024, delta=0.5, intermediate_error=True, seed=1, gemm_precision="fp32")
    eng.set_centers(C0.float())
    for _ in range(8):
        eng.step()[1].tolist()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        eng.step()[1].tolist()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
