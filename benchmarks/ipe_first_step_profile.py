"""Host-side profile (cProfile) of the first two IPE Lloyd steps at the bench
shape: where the first step's wall time goes beyond its kernels."""
import cProfile
import io
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from sq_learn_amd.models._data import Data, gather_rows  # noqa: E402
from sq_learn_amd.models.cluster._lloyd import LloydEngine  # noqa: E402
from sq_learn_amd.parallel.comm import Comm  # noqa: E402
from sq_learn_amd.utils.datasets import make_blobs_device  # noqa: E402

n, d, k, seed = 10_000_000, 256, 1024, 2024
dev = torch.device("cuda")
X, _ = make_blobs_device(n, d, centers=1024, cluster_std=1.0, seed=seed, device=dev,
                         dtype=torch.float32)
C0 = gather_rows(Data(X, n, 0, Comm(None), "sharded"),
                 np.random.RandomState(seed).choice(n, k, replace=False))
eng = LloydEngine(X, k, delta=0.5, true_distance_estimate=True, intermediate_error=True,
                  true_tomography=False, seed=seed, comm=Comm(None), gemm_precision="fp32")
eng.set_centers(C0)
torch.cuda.synchronize()
for s in range(2):
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    eng.step()[1].tolist()
    torch.cuda.synchronize()
    pr.disable()
    print(f"step {s}: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
    out = io.StringIO()
    pstats.Stats(pr, stream=out).sort_stats("cumulative").print_stats(25)
    print(out.getvalue(), flush=True)
