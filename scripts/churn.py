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
    if getattr(eng, "bounds", False):
        q = torch.quantile(eng.shift_s.float(), torch.tensor([0.5, 0.9, 0.99], device=dev)).tolist()
        print(f"   shifts: median {q[0]:.3g} p90 {q[1]:.3g} p99 {q[2]:.3g} max {eng.smax.item():.3g}")
    prev = lab
# exact candidate gaps of the last iteration's multi rows (candidate lists
# are stored per row)
if getattr(eng, "bounds", False):
    b = eng.buf
    m = int(b.counts[2].item())
    rows = b.multi_rows[:m]
    sel = torch.arange(0, m, max(1, m // 20000), device=dev)
    rows = rows[sel]
    cand = b.multi_cand[rows]
    C = eng.C.double()
    x = X[rows].double()
    cr = cand[:, 0].long()
    D = torch.full((sel.numel(), 16), float("inf"), dtype=torch.float64, device=dev)
    for c in range(16):
        ok = cr > c
        j = cand[:, 1 + c].long().clamp(0, 1023)
        d = ((x - C[j]) ** 2).sum(1)
        D[:, c] = torch.where(ok, d, D[:, c])
    Ds = D.sort(1).values
    gap = Ds[:, 1] - Ds[:, 0]
    band1 = gap > 0.5
    qs = torch.tensor([0.1, 0.5, 0.9], device=dev, dtype=torch.float64)
    print(f"multi rows sampled {sel.numel()}: band>=2 {(~band1).float().mean().item():.3f}; "
          f"c_r mean {cr.float().mean().item():.2f}; gap quantiles {torch.quantile(gap, qs).tolist()}; "
          f"dmin median {Ds[:, 0].median().item():.4g}")
    print("E-range of filter: alpha", eng.alpha)
