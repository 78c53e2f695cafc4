"""Exact accelerated k-means++ (csrc/kmpp.hip, ops.kmeans.KmppState) and
the device k-means++ built on it (models/cluster/_init.py).

The screens (triangle inequality against each row's nearest chosen centre,
certified int8 bound) only skip rows whose minimum provably stays the same,
and every potential is an exact fixed-point integer: the chosen ids are
IDENTICAL with the screens on and off.  The trial pass itself is checked
against an fp64 torch reference of the same op."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from sq_learn_amd.ops import kmeans as K  # noqa: E402
from sq_learn_amd.models._data import Data  # noqa: E402
from sq_learn_amd.models.cluster._init import kmeans_plusplus  # noqa: E402
from sq_learn_amd.parallel.comm import Comm  # noqa: E402


def _blobs(n, d, centers, seed, std=1.0, box=10.0):
    rs = np.random.RandomState(seed)
    G = rs.uniform(-box, box, (centers, d))
    return (G[rs.randint(centers, size=n)] + std * rs.randn(n, d)).astype(np.float32)


@pytest.mark.parametrize("n,d,t,weighted", [(5000, 256, 8, False), (3001, 20, 3, True),
                                            (777, 64, 16, False), (1, 4, 1, False)])
def test_kmpp_trial_pass_matches_fp64(n, d, t, weighted):
    """One trial pass after a first centre: Delta_j (fixed point) equals the
    fp64 improvement sum of the same op, the improving rows' distances
    match, and the pruned and unpruned passes agree bit for bit."""
    g = torch.Generator().manual_seed(n + d + t)
    X = torch.randn(n, d, generator=g) * 3.0
    cand = X[torch.randint(0, n, (t,), generator=g)] + 0.1
    c0 = X[0]
    w = torch.rand(n, generator=g, dtype=torch.float64) if weighted else None
    outs = []
    for prune in (True, False):
        st = K.KmppState(X.cuda(), 4, t, w=None if w is None else w.cuda(), prune=prune)
        mx = st.first_centre(c0.cuda())
        P = st.set_scale(mx.item(), n)
        C = torch.zeros((4, d), dtype=torch.float32, device="cuda")
        C[0] = c0.cuda()
        delta = st.trials(cand.cuda(), C, 1)
        torch.cuda.synchronize()
        outs.append((delta.cpu(), P.cpu(), st.mask[0].cpu(), st.D[0][:, :n].cpu(), st.scale,
                     st.closest[:n].cpu()))
    (da, Pa, ma, Da, scale, cl), (db, Pb, mb, Db, _, _) = outs
    assert torch.equal(da, db) and torch.equal(Pa, Pb) and torch.equal(ma, mb)
    sel = ma.numpy() != 0
    Dref = ((X.double()[None, :, :] - cand.double()[:, None, :]) ** 2).sum(2)   # [t, n]
    cl0 = ((X.double() - c0.double()) ** 2).sum(1)
    np.testing.assert_allclose(cl.double().numpy(), cl0.numpy(), rtol=3e-6, atol=1e-4)
    for j in range(t):
        bit = (ma.numpy().astype(np.int64) >> j) & 1
        rows = np.nonzero(bit)[0]
        np.testing.assert_allclose(Da[j, rows].double().numpy(), Dref[j, rows].numpy(), rtol=3e-6,
                                   atol=1e-4)
        assert torch.equal(Da[j, rows], Db[j, rows])
    ww = w if weighted else torch.ones(n, dtype=torch.float64)
    imp = (cl.double()[None, :] - torch.minimum(cl.double()[None, :], Dref)) * ww[None, :]
    np.testing.assert_allclose(da.numpy() / scale, imp.sum(1).numpy(), rtol=1e-5,
                               atol=1e-5 * float(Pa) / scale)
    np.testing.assert_allclose(float(Pa) / scale, float((cl.double() * ww).sum()), rtol=1e-9,
                               atol=n * 1.0 / scale)
    assert sel.any() or n == 1


@pytest.mark.parametrize("n,d,k", [(60000, 64, 128), (20000, 256, 64), (9001, 20, 40)])
def test_kmpp_pruned_ids_identical_to_unpruned(n, d, k):
    """Same data, same RandomState: the pruned k-means++ chooses exactly the
    unpruned one's centres, while its screens skip most rows."""
    X = _blobs(n, d, k, seed=n + d)
    Xt = torch.from_numpy(X).cuda()
    res = {}
    for prune in (True, False):
        data = Data(Xt, n, 0, Comm(None), "sharded")
        stats = []
        C, ids = kmeans_plusplus(data, k, np.random.RandomState(5), prune=prune, stats=stats)
        res[prune] = (np.asarray(ids), C.cpu().numpy(), np.asarray(stats))
    ia, Ca, sa = res[True]
    ib, Cb, sb = res[False]
    assert np.array_equal(ia, ib)
    assert np.array_equal(Ca, Cb)
    np.testing.assert_array_equal(Ca, X[ia])
    assert len(set(ia.tolist())) == k
    # unpruned: every row through the exact pass; pruned: far fewer
    assert (sb[:, 1] == n).all()
    assert sa[:, 1].mean() < 0.5 * n, sa[:, 1].mean()
    assert sa[-k // 4:, 0].mean() < 0.5 * n, sa[-k // 4:, 0].mean()


def test_kmpp_weighted_and_duplicates():
    """Weighted potentials (the k-means|| reduction) and exact duplicate
    rows (zero potentials) stay identical with and without the screens."""
    rs = np.random.RandomState(7)
    base = _blobs(3000, 32, 12, seed=7)
    X = np.concatenate([base, base[:500]]).astype(np.float32)    # duplicates
    w = torch.from_numpy(rs.uniform(0.1, 5.0, X.shape[0]))
    Xt = torch.from_numpy(X).cuda()
    out = []
    for prune in (True, False):
        data = Data(Xt, X.shape[0], 0, Comm(None), "sharded")
        C, ids = kmeans_plusplus(data, 24, np.random.RandomState(2), sample_weight=w.cuda(),
                                 prune=prune)
        out.append(np.asarray(ids))
    assert np.array_equal(out[0], out[1])


def test_device_kmeans_plusplus_seeding_quality():
    """The device seeding is a k-means++ seeding: distinct valid rows, and a
    potential comparable with the CPU path's on the same data."""
    X = _blobs(20000, 16, 32, seed=0)
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


@pytest.mark.parametrize("n,dq", [(37, 64), (100, 256), (16, 832)])
def test_kmpp_int8_mfma_dots_exact(n, dq):
    """The certified bound's int8 MFMA dot products (v_mfma_i32_16x16x64_i8
    fragments built by kpp_i8_dots) equal numpy's integer dot products for
    both candidate terms and every trial slot."""
    from sq_learn_amd.ops import _native as nat
    rs = np.random.RandomState(dq)
    Xq = rs.randint(-127, 128, (n, dq)).astype(np.int8)
    cq = rs.randint(-127, 128, (2, 16, dq)).astype(np.int8)
    Xt = torch.from_numpy(Xq).cuda()
    ct = torch.from_numpy(cq).cuda()
    out = torch.zeros((2, n, 16), dtype=torch.int32, device="cuda")
    rc = nat.native().kmpp_dots(Xt.data_ptr(), dq, n, ct.data_ptr(), out.data_ptr(),
                                nat.stream_handle(Xt.device))
    assert not rc
    ref = np.einsum("nf,hjf->hnj", Xq.astype(np.int64), cq.astype(np.int64))
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
