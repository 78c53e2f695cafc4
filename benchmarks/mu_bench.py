"""mu(A) power sums (csrc/linalg.hip mu_sums_kernel) on 10M x 256 fp32:
ms per call of ``mu_power_sums_local`` with the p-grid of the qPCA / q-means
prelude (0, 0.2, ..., 2.2)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from sq_learn_amd.ops import linalg as L  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 256
X = torch.randn(n, d, device="cuda") * 3
exps = [round(0.2 * i, 10) for i in range(12)]
mean = X.double().mean(0)
for _ in range(2):
    L.mu_power_sums_local(X, exps, mean=mean)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    L.mu_power_sums_local(X, exps, mean=mean)
torch.cuda.synchronize()
print(f"mu_power_sums n={n} d={d}: {(time.perf_counter() - t0) / 5 * 1e3:.2f} ms", flush=True)
