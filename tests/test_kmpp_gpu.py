"""Fused k-means++ trial pass (csrc/kmpp.hip) against an fp64 torch
reference of the same op, and the device k-means++ built on it."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from sq_learn_amd.ops import kmeans as K  # noqa: E402


@pytest.mark.parametrize("n,d,t,weighted", [(5000, 256, 8, False), (3001, 20, 3, True),
                                            (777, 64, 16, False), (1, 4, 1, False)])
def test_kmpp_trials_matches_fp64(n, d, t, weighted):
    g = torch.Generator().manual_seed(n + d + t)
    X = torch.randn(n, d, generator=g) * 3.0
    cand = X[torch.randint(0, n, (t,), generator=g)] + 0.1
    closest = torch.rand(n, generator=g, dtype=torch.float64) * 4 * d
    w = torch.rand(n, generator=g, dtype=torch.float64) if weighted else None
    Xc, cc, clc = X.cuda(), cand.cuda(), closest.cuda()
    wc = w.cuda() if weighted else None
    D, pots = K.kmpp_trials_native(Xc, cc.contiguous(), clc, wc)
    torch.cuda.synchronize()
    Dref = ((X.double()[None, :, :] - cand.double()[:, None, :]) ** 2).sum(2)   # [t, n]
    np.testing.assert_allclose(D.cpu().double().numpy(), Dref.numpy(), rtol=2e-6, atol=1e-4)
    m = torch.minimum(closest[None, :], Dref)
    pref = (m * (w[None, :] if weighted else 1.0)).sum(1)
    np.testing.assert_allclose(pots.cpu().numpy(), pref.numpy(), rtol=1e-6)
    # deterministic: same bits on a second call
    D2, pots2 = K.kmpp_trials_native(Xc, cc.contiguous(), clc, wc)
    assert torch.equal(pots, pots2) and torch.equal(D, D2)


def test_device_kmeans_plusplus_native_path():
    """QMeans-style device k-means++: distinct valid rows, centres are data
    rows, and the potential matches a well-spread seeding (vs the CPU path
    on the same data and RandomState)."""
    from sq_learn_amd.models._data import Data
    from sq_learn_amd.models.cluster._init import kmeans_plusplus
    from sq_learn_amd.parallel.comm import Comm
    rs = np.random.RandomState(0)
    G = rs.uniform(-10, 10, (32, 16))
    X = (G[rs.randint(32, size=20000)] + rs.randn(20000, 16)).astype(np.float32)
    out = {}
    for dev in ("cuda", "cpu"):
        Xt = torch.from_numpy(X).to(dev)
        data = Data(Xt, X.shape[0], 0, Comm(None), "sharded")
        C, ids = kmeans_plusplus(data, 32, np.random.RandomState(3))
        out[dev] = (C.double().cpu().numpy(), np.asarray(ids))
    Cg, idg = out["cuda"]
    assert len(set(idg.tolist())) == 32
    np.testing.assert_allclose(Cg, X[idg].astype(np.float64))
    def inertia(C):
        D = ((X[:, None, :].astype(np.float64) - C[None]) ** 2).sum(2)
        return D.min(1).sum()
    ig, ic = inertia(Cg), inertia(out["cpu"][0])
    assert ig <= 1.5 * ic and ic <= 1.5 * ig
