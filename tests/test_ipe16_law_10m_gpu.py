"""The ipe16 IPE E-step at the bench scale: 10M x 256, k = 1024.  The
rows' law is pinned against the full sampler on a 200k-row subsample.

The E-step runs in the middle of a Lloyd trajectory, so the row skip is on
for most rows and realistic bands, fires and dense rows all occur.  The full
sampler is the fp32 fused kernel (csrc/ipe.hip) with pruning off, so every
pair is sampled in full.  Its rows are drawn with independent keys.

Each row draws once per sampler.  The two samples are compared through a
joint histogram with three coordinates:

* the rank of the chosen centroid by exact distance (0, 1, 2 or more);
* the chosen estimate relative to that pair's exact distance (quantile bins);
* how many centroids lie within 1.2x the row's nearest distance (1, 2 or 3+).

The comparison is a chi^2 two-sample test (``_dmeans.py:753-772``,
``Utility.py:697-737``).  The subsample is every 50th row."""
import numpy as np
import pytest
import torch
from scipy import stats

from sq_learn_amd.models._data import Data, gather_rows
from sq_learn_amd.models.cluster._lloyd import LloydEngine
from sq_learn_amd.parallel.comm import Comm
from sq_learn_amd.utils.datasets import make_blobs_device

from test_ipe16_gpu import _run_full

pytestmark = pytest.mark.gpu


def _features(X, C, lab, mind):
    """(rank of the label by exact distance, estimate / exact distance of
    the label, crowding) per row, fp64."""
    Xd, Cd = X.double(), C.double()
    out_rank, out_ratio, out_crowd = [], [], []
    for s in range(0, X.shape[0], 20000):
        x = Xd[s:s + 20000]
        D = (x * x).sum(1)[:, None] + (Cd * Cd).sum(1)[None, :] - 2.0 * x @ Cd.T
        D = D.clamp_min(0.0)
        lb = lab[s:s + 20000].long()
        dl = D.gather(1, lb[:, None])[:, 0]
        out_rank.append((D < dl[:, None]).sum(1).clamp(max=2))
        out_ratio.append(mind[s:s + 20000].double() / dl.clamp_min(1e-30))
        dmin = D.min(1).values
        out_crowd.append((D <= 1.2 * dmin[:, None]).sum(1).clamp(max=3))
    return torch.cat(out_rank), torch.cat(out_ratio), torch.cat(out_crowd)


def test_ipe16_10m_law_on_subsample(cuda):
    n, d, k, seed = 10_000_000, 256, 1024, 2024
    X, _ = make_blobs_device(n, d, centers=1024, cluster_std=1.0, seed=seed, device=cuda,
                             dtype=torch.float32)
    C0 = gather_rows(Data(X, n, 0, Comm(None), "sharded"),
                     np.random.RandomState(seed).choice(n, k, replace=False))
    eng = LloydEngine(X, k, delta=0.5, true_distance_estimate=True, intermediate_error=True,
                      true_tomography=False, seed=7, comm=Comm(None), gemm_precision="fp32")
    eng.set_centers(C0)
    for _ in range(5):
        eng.step()[1].tolist()
    eng.ipe16_stats = torch.zeros(8, dtype=torch.int64, device=cuda)
    lab, mind, _ = eng.estep()
    torch.cuda.synchronize()
    skipped = int(eng.ipe16_stats[7])
    assert skipped > 0.3 * n, eng.ipe16_stats.tolist()   # the row skip carries most rows
    C = eng.C.float().contiguous()
    sub = torch.arange(0, n, 50, device=cuda)
    Xs = X[sub].contiguous()
    la, ma = lab[sub], mind[sub]
    lb_np, mb_np = _run_full(Xs, C, eng.delta / 2.0, eng.ipe_Q, 99)
    lb = torch.from_numpy(lb_np).to(cuda)
    mb = torch.from_numpy(mb_np).to(cuda)
    ra, qa, ca = _features(Xs, C, la, ma)
    rb, qb, cb = _features(Xs, C, lb, mb)
    # the chosen label is the exact argmin for most rows, but not all (the
    # estimates are noisy): both samplers must agree on how often
    assert 0.5 < float((ra == 0).double().mean()) < 1.0
    edges = torch.quantile(torch.cat([qa, qb]).float()[::7],
                           torch.linspace(0, 1, 11, device=cuda)[1:-1])
    ba = torch.bucketize(qa.float(), edges)
    bb = torch.bucketize(qb.float(), edges)
    cell_a = (ra * 10 + ba) * 4 + ca
    cell_b = (rb * 10 + bb) * 4 + cb
    m = int(max(cell_a.max(), cell_b.max())) + 1
    ta = torch.bincount(cell_a, minlength=m).cpu().numpy()
    tb = torch.bincount(cell_b, minlength=m).cpu().numpy()
    keep = (ta + tb) >= 40
    table = np.stack([np.append(ta[keep], ta[~keep].sum()), np.append(tb[keep], tb[~keep].sum())])
    table = table[:, table.sum(0) > 0]
    assert table.shape[1] >= 10
    p = stats.chi2_contingency(table)[1]
    assert p > 1e-4, (p, table)
