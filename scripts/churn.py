"""Label churn per Lloyd iteration on the bench data (how many rows change
cluster; how many go through the fp64 re-check) - sizing the incremental
M-step."""
import sys, os
sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
import numpy as np
import torch
from sq_learn_amd.utils.datasets import make_blobs_device
from sq_learn_amd.models.cluster._lloyd import LloydEngine
from sq_learn_amd.models._data import Data, gather_rows
from sq_learn_amd.parallel.comm import Comm
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
dev = torch.device("cuda")
X, _ = make_blobs_device(n, 256, centers=1024, cluster_std=1.0, seed=2024, device=dev,
                         dtype=torch.float32, row_range=(0, n))
data = Data(X, n, 0, Comm(None), "sharded")
idx = np.random.RandomState(2024).choice(n, 1024, replace=False)
eng = LloydEngine(X, 1024, delta=0.5, true_distance_estimate=False, intermediate_error=True,
                  true_tomography=False, seed=2024, comm=Comm(None), row_offset=0,
                  gemm_precision="fp32")
eng.set_centers(gather_rows(data, idx))
prev = None
for it in range(15):
    lab, sc = eng.step()
    lab = lab.clone()
    cnt = eng.buf.counts.tolist()
    ch = int((lab != prev).sum()) if prev is not None else n
    act = int(eng.rcount.item()) if getattr(eng, "bounds", False) and it > 0 else n
    print(f"it {it}: changed {ch} ({ch / n:.3%}), active (not pruned) {act} ({act / n:.2%}), "
          f"multi {cnt[2]} ({cnt[2] / n:.2%}), dense {cnt[1]}, ovf {cnt[0]}, "
          f"inertia {sc.tolist()[0]:.6e}", flush=True)
    prev = lab
