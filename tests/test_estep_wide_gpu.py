"""The certified E-step beyond d = 256 / k = 4096 and the exact fp64 rows
kernel (csrc/estep_f32.hip sub-staged tiles, csrc/rows_f64.hip) against the
reference's fp64 band rule (``sklearn/cluster/_dmeans.py:736-751``: fp64
``cdist(X, C)**2``, uniform member of {j : D_j <= min + delta}).

Every label the certified path produces is an fp64 decision (filter with a
rigorous bound -> fp64 re-check; dense / overflow rows -> the exact rows
kernel), so the labels must equal the fp64 rule's on every row except where
some fp64 distance sits within rounding (1e-9 relative) of the band edge.
The torch reference is an independent computation (direct form on fp64
copies)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from sq_learn_amd.models.cluster._lloyd import LloydEngine  # noqa: E402
from sq_learn_amd.ops import kmeans as K  # noqa: E402


def _cdist2(Xd, Cd, step=256):
    """fp64 squared distances in direct form, sum_f (x_f - c_f)^2 (column
    chunks; torch.cdist's direct mode returns zeros for the trailing columns
    of very wide outputs on this ROCm build, k >~ 6000)."""
    out = torch.empty((Xd.shape[0], Cd.shape[0]), dtype=torch.float64, device=Xd.device)
    for s in range(0, Cd.shape[0], step):
        c = Cd[s:s + step]
        out[:, s:s + step] = ((Xd[:, None, :] - c[None, :, :]) ** 2).sum(-1)
    return out


def _fp64_rule(X, C, delta, key, k_pad):
    Xd = torch.from_numpy(X).double().cuda()
    Cd = torch.from_numpy(C).double().cuda()
    D = _cdist2(Xd, Cd)
    g = torch.arange(X.shape[0], dtype=torch.int64, device=D.device)
    lab, mn = K.band_select_torch(D, g, delta, key, k_pad)
    return D, lab, mn


def _near_edge(D, mn, delta, rel=1e-9):
    scale = D.max(1).values.clamp(min=1.0)
    edge = mn + delta
    near = ((D - edge[:, None]).abs() <= rel * scale[:, None]).any(1)
    if delta == 0:
        d2 = torch.topk(D, 2, dim=1, largest=False).values
        near = (d2[:, 1] - d2[:, 0]) <= rel * scale
    return near


def _data(n, d, k, seed=0, groups=24, s=0.08, spread=1.0):
    """Groups of near-duplicate centroids: wide bands, many multi-candidate
    and dense rows."""
    rs = np.random.RandomState(seed)
    G = rs.randn(groups, d) * spread
    C = G[np.arange(k) % groups] + s * rs.randn(k, d)
    X = G[rs.randint(groups, size=n)] + 0.4 * rs.randn(n, d)
    return X.astype(np.float32), C.astype(np.float32)


def _estep(X, C, delta, precision="fp32"):
    Xt = torch.from_numpy(X).cuda()
    eng = LloydEngine(Xt, C.shape[0], delta=delta, seed=11, gemm_precision=precision)
    eng.set_centers(torch.from_numpy(C).cuda())
    key = eng._key("band_select")
    lab, mind, inertia = eng.estep()
    torch.cuda.synchronize()
    return eng, key, lab.long()[: X.shape[0]], mind[: X.shape[0]], inertia


@pytest.mark.parametrize("d", [384, 512, 784, 1024])
@pytest.mark.parametrize("delta", [0.0, 0.5])
def test_certified_wide_d_is_fp64_band_rule(d, delta):
    n, k = 6000, 512
    X, C = _data(n, d, k, seed=d)
    eng, key, lab, mind, inertia = _estep(X, C, delta)
    assert eng.fast and eng.certified and eng.d_pad == K.pad_features(d) >= d
    D, lab64, mn64 = _fp64_rule(X, C, delta, key, eng.k_pad)
    if delta > 0:
        band = (D <= (mn64 + delta)[:, None]).sum(1).double().mean().item()
        assert band > 1.5, band   # multi-member bands: the kappa pick is exercised
    near = _near_edge(D, mn64, delta)
    assert near.double().mean().item() < 0.01
    bad = (lab != lab64) & ~near
    assert int(bad.sum()) == 0, (int(bad.sum()), int(eng.buf.counts[1].item()))
    # min distances: fp64 values stored in fp32
    rel = (mind.double() - mn64).abs() / mn64.clamp(min=1e-30)
    assert float(rel.max()) < 1e-6
    assert abs(float(inertia) - float(mn64.sum())) <= 1e-6 * float(mn64.sum())


@pytest.mark.parametrize("d", [256, 784])
def test_dense_rows_through_exact_rows_kernel(d):
    """delta = 40: nearly every row is dense (a lane with 3+ band members);
    at d_pad <= 256 they go through the 3-pass kernel and its overflow rows
    through the rows kernel, above 256 straight to the rows kernel - exact
    fp64 either way."""
    n, k = 3000, 512
    X, C = _data(n, d, k, seed=3)
    eng, key, lab, mind, _ = _estep(X, C, 40.0)
    dense = int(eng.buf.counts[1].item())
    assert dense > n // 2, dense
    D, lab64, mn64 = _fp64_rule(X, C, 40.0, key, eng.k_pad)
    near = _near_edge(D, mn64, 40.0)
    assert int(((lab != lab64) & ~near).sum()) == 0
    rel = (mind.double() - mn64).abs() / mn64.clamp(min=1e-30)
    assert float(rel.max()) < 1e-6


@pytest.mark.parametrize("n,d,k", [(4000, 1100, 96), (3001, 40, 20000), (2000, 7, 33)])
def test_generic_gpu_engine_is_exact(n, d, k):
    """Shapes outside the filter (d_pad > 1024, k_pad > 16384) and the
    generic engine run the exact fp64 rows kernel on every row - no
    uncertified library-GEMM fallback."""
    rs = np.random.RandomState(k)
    X = (rs.randn(n, d) * 1.5).astype(np.float32)
    C = (X[rs.choice(n, k, replace=True)] + 0.05 * rs.randn(k, d)).astype(np.float32)
    Xt = torch.from_numpy(X).cuda()
    eng = LloydEngine(Xt, k, delta=0.3, seed=5, gemm_precision="fp32",
                      generic=(d == 7))
    assert not eng.fast
    eng.set_centers(torch.from_numpy(C).cuda())
    key = eng._key("band_select")
    lab, mind, inertia = eng.estep()
    D, lab64, mn64 = _fp64_rule(X, C, 0.3, key, eng.k_pad)
    near = _near_edge(D, mn64, 0.3)
    assert int(((lab.long()[:n] != lab64) & ~near).sum()) == 0
    rel = (mind[:n].double() - mn64).abs() / mn64.clamp(min=1e-30)
    assert float(rel.max()) < 1e-6


def test_large_k_filter():
    """k = 6000 (k_pad 6016 > the former 4096 cap): the filter's packed tile
    index takes 8 bits; labels still the fp64 rule's."""
    n, d, k = 5000, 64, 6000
    X, C = _data(n, d, k, seed=9, groups=200)
    eng, key, lab, mind, _ = _estep(X, C, 0.5)
    assert eng.fast and eng.k_pad == 6016
    D, lab64, mn64 = _fp64_rule(X, C, 0.5, key, eng.k_pad)
    near = _near_edge(D, mn64, 0.5)
    assert int(((lab != lab64) & ~near).sum()) == 0


def test_rows_kernel_wide_band_scan():
    """More than 64 candidates (a band of > 64 near-identical centroids):
    the rows kernel's exact direct-form scan over all k."""
    rs = np.random.RandomState(2)
    n, d, k = 200, 32, 300
    X = rs.randn(n, d).astype(np.float32)
    C = (0.001 * rs.randn(k, d)).astype(np.float32)   # all centroids ~ the origin
    Xt = torch.from_numpy(X).cuda()
    lab = torch.empty(n, dtype=torch.int32, device="cuda")
    mind = torch.empty(n, dtype=torch.float32, device="cuda")
    key = LloydEngine(Xt, k, delta=0.5, seed=1)._key("band_select")
    K.rows_f64_native(Xt, torch.from_numpy(C).cuda(), lab, mind, 0.5, key, 0)
    D, lab64, mn64 = _fp64_rule(X, C, 0.5, key, ((k + 63) // 64) * 64)
    assert float((D <= (mn64 + 0.5)[:, None]).sum(1).double().min()) > 64
    near = _near_edge(D, mn64, 0.5)
    assert int(((lab.long() != lab64) & ~near).sum()) == 0


def test_qmeans_mnist_shape():
    """BASELINE config 4 shape: 70k x 784, k = 10 (the certified filter at
    d_pad 896), a full fit; labels of the final E-step equal the fp64 rule
    at the returned centroids."""
    from sq_learn_amd.models.cluster import QMeans
    rs = np.random.RandomState(0)
    n, d, k = 70000, 784, 10
    G = rs.rand(k, d).astype(np.float32)
    X = np.clip(G[rs.randint(k, size=n)] + 0.3 * rs.randn(n, d).astype(np.float32), 0, 1)
    est = QMeans(n_clusters=k, delta=0.5, true_distance_estimate=False, intermediate_error=True,
                 n_init=1, max_iter=10, random_state=0, device="cuda:0").fit(X)
    assert est.labels_.shape == (n,) and np.isfinite(est.inertia_)
    assert len(np.unique(est.labels_)) == k
    # the final E-step ran on the centred fp32 rows at the returned centres:
    # every label is a member of the fp64 delta-band there (rows within
    # rounding of the band edge aside) and the inertia is the sum of the fp64
    # minimum distances
    mean = torch.from_numpy(np.asarray(est._mean, dtype=np.float64))
    Xc = (torch.from_numpy(X) - mean.float()).double().cuda()
    C = (torch.from_numpy(est.cluster_centers_) - mean).cuda()
    D = _cdist2(Xc, C)
    mn = D.min(1).values
    near = _near_edge(D, mn, 0.5, rel=1e-7)
    lab = torch.from_numpy(est.labels_.astype(np.int64)).cuda()
    inband = D.gather(1, lab[:, None])[:, 0] <= mn + 0.5
    assert int((~inband & ~near).sum()) == 0
    assert int(near.sum()) < n // 1000
    assert est.inertia_ == pytest.approx(float(mn.sum()), rel=1e-6)
