"""HIP Elkan bounded assignment (csrc/elkan.hip) vs fp64 exact distances."""
import numpy as np
import pytest
import torch

from sq_learn_amd.ops import elkan as E
from sq_learn_amd.ops import _native as nat

pytestmark = pytest.mark.gpu


def _blobs(n, d, k, seed):
    g = torch.Generator().manual_seed(seed)
    C = torch.randn(k, d, generator=g, dtype=torch.float64) * 2
    lab = torch.randint(0, k, (n,), generator=g)
    return C[lab] + torch.randn(n, d, generator=g, dtype=torch.float64)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("d,k", [(16, 8), (100, 300), (256, 64), (33, 1000), (700, 20)])
def test_elkan_kernel_exact_and_bounds(cuda, dtype, d, k):
    n = 3001
    X = _blobs(n, d, k, 0)
    C = X[torch.randperm(n, generator=torch.Generator().manual_seed(1))[:k]].clone()
    assert E._native_ok(X.to(cuda, dtype), k)
    Xg = X.to(cuda, dtype).contiguous()
    lab = torch.zeros(n, dtype=torch.int32, device=cuda)
    up = torch.zeros(n, dtype=dtype, device=cuda)
    lo = torch.zeros(n, k, dtype=dtype, device=cuda)
    sh = torch.zeros(k, dtype=dtype, device=cuda)
    tol = 1e-4 if dtype == torch.float32 else 1e-10
    for it in range(5):
        Cg = C.to(cuda, dtype).contiguous()
        hcc, sn = E.centre_geometry(Cg)
        E.elkan_step(Xg, Cg, hcc, sn, sh, lab, up, lo, init=(it == 0))
        torch.cuda.synchronize()
        Xr, Cr = Xg.double().cpu(), Cg.double().cpu()
        D = torch.cdist(Xr, Cr, compute_mode="donot_use_mm_for_euclid_dist")
        got = lab.cpu().long()
        dmin = D.min(1).values
        dg = D.gather(1, got[:, None])[:, 0]
        # exact argmin up to dtype rounding of near-ties
        assert bool((dg <= dmin * (1 + tol) + tol).all())
        assert (got == D.argmin(1)).float().mean() > 0.999
        assert bool((up.cpu().double() >= dg * (1 - tol) - tol).all())
        assert bool((lo.cpu().double() <= D * (1 + tol) + tol).all())
        newC = torch.stack([X[got == j].mean(0) if (got == j).any() else C[j] for j in range(k)])
        sh = E.centre_shift(C, newC).to(cuda, dtype)
        C = newC


def test_kmeans_elkan_gpu_matches_cpu(cuda):
    from sq_learn_amd.models.cluster import KMeans
    from sq_learn_amd.utils.datasets import make_blobs
    X, y = make_blobs(8000, 24, centers=15, random_state=3)
    X = np.asarray(X, dtype=np.float64)
    init = X[:15].copy()
    g = KMeans(15, init=init, n_init=1, algorithm="elkan", device="cuda").fit(X)
    c = KMeans(15, init=init, n_init=1, algorithm="elkan", device="cpu").fit(X)
    from sklearn.metrics import adjusted_rand_score
    assert adjusted_rand_score(g.labels_, c.labels_) > 0.999
    np.testing.assert_allclose(g.cluster_centers_, c.cluster_centers_, rtol=1e-4, atol=1e-4)
    assert abs(g.inertia_ - c.inertia_) / c.inertia_ < 1e-5
    assert nat.native() is not None


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("n,m,d", [(1, 1, 1), (70, 130, 33), (257, 64, 300)])
def test_pairwise_reduce_kernel(cuda, dtype, n, m, d):
    """csrc/pairwise_fast.hip tiles vs the fp64 torch reference."""
    from sq_learn_amd.utils.pairwise import pairwise_reduce, _torch_reduce
    g = torch.Generator().manual_seed(n + m + d)
    X = torch.rand(n, d, generator=g, dtype=torch.float64)
    Y = torch.rand(m, d, generator=g, dtype=torch.float64)
    tol = 1e-4 if dtype == torch.float32 else 1e-11
    for op, p in (("l1", 2.0), ("chi2", 2.0), ("chebyshev", 2.0), ("minkowski", 3.0)):
        got = pairwise_reduce(X.to(cuda, dtype), Y.to(cuda, dtype), op, p).cpu().double()
        ref = _torch_reduce(X, Y, op, p)
        torch.testing.assert_close(got, ref, rtol=tol, atol=tol)
