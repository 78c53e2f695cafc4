"""Host cost of the pipelined Lloyd step (k = 1024): enqueue time of
eng.step() vs the wait in the scalar read, then a cProfile of 100 steps.
argv[1]: the share of the 10M x 256 problem (8: the N = 8 per-GPU share of
1.25M rows, the default; 1: the headline's 10M rows)."""
import cProfile
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from sq_learn_amd.models.cluster._lloyd import LloydEngine  # noqa: E402
from sq_learn_amd.models._data import Data, gather_rows  # noqa: E402
from sq_learn_amd.parallel.comm import Comm  # noqa: E402
from sq_learn_amd.utils.datasets import make_blobs_device  # noqa: E402

n, d, k = 10_000_000, 256, 1024
dev = torch.device("cuda", 0)
X, _ = make_blobs_device(n, d, centers=1024, cluster_std=1.0, seed=2024, device=dev,
                         dtype=torch.float32, row_range=(0, n))
comm = Comm(None)
C0 = gather_rows(Data(X, n, 0, comm, "sharded"), np.random.RandomState(2024).choice(n, k, replace=False))
share = int(sys.argv[1]) if len(sys.argv) > 1 else 8
Xs = X[: n // share].contiguous() if share > 1 else X
del X
eng = LloydEngine(Xs, k, delta=0.5, true_distance_estimate=False, intermediate_error=True,
                  true_tomography=False, seed=2024, comm=comm, row_offset=0, gemm_precision="fp32")
eng.set_centers(C0)
eng.pipeline = True
for _ in range(20 if share == 1 else 10):
    eng.step()[1].tolist()
torch.cuda.synchronize()
te = tw = 0.0
N = 100
t0 = time.perf_counter()
for _ in range(N):
    a = time.perf_counter()
    sc = eng.step()[1]
    b = time.perf_counter()
    sc.tolist()
    c = time.perf_counter()
    te += b - a
    tw += c - b
torch.cuda.synchronize()
print(f"wall {1e3 * (time.perf_counter() - t0) / N:.4f} ms/step, enqueue {1e3 * te / N:.4f}, wait {1e3 * tw / N:.4f}")
pr = cProfile.Profile()
pr.enable()
for _ in range(N):
    eng.step()[1].tolist()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(28)
