"""HIP q-means kernels vs fp64 / torch references (run on an MI355X)."""
import numpy as np
import pytest
import torch

from sq_learn_amd.ops import kmeans as K
from sq_learn_amd.ops import linalg as L
from sq_learn_amd.runtime.rng import RngKey

pytestmark = pytest.mark.gpu


def _data(n, d, k, seed, dev):
    g = torch.Generator().manual_seed(seed)
    C = torch.randn(k, d, generator=g, dtype=torch.float64) * 3
    lab = torch.randint(0, k, (n,), generator=g)
    X = C[lab] + torch.randn(n, d, generator=g, dtype=torch.float64)
    return X, C


@pytest.mark.parametrize("d,k", [(16, 8), (64, 100), (256, 1024), (100, 300)])
def test_estep_exact_matches_fp64(cuda, d, k):
    n = 4099
    X, C = _data(n, d, k, 0, cuda)
    dp, kp = K.pad_features(d), K.pad_clusters(k)
    Xb = torch.zeros(n, dp, dtype=torch.bfloat16)
    Xb[:, :d] = X.to(torch.bfloat16)
    Cb, cn = K.centers_to_bf16(C.float(), kp, dp)
    Xg, Cbg, cng = Xb.to(cuda), Cb.to(cuda), cn.to(cuda)
    xn = L.row_norms_sq(Xg)
    buf = K.EStepBuffers(n, cuda)
    key = RngKey(1, "band_select", 0)
    lab, mind = K.estep_native(Xg, Cbg, cng, xn, k, 0.0, key, 0, buf)
    torch.cuda.synchronize()
    # fp64 reference on the bf16-rounded operands
    Xr = Xb[:, :d].double()
    Cr = K.centers_from_operand(Cb, k, d).double()
    D = K.distances_torch(Xr, Cr)
    ref = D.argmin(1)
    got = lab.cpu().long()
    agree = (got == ref).float().mean().item()
    assert agree > 0.999, agree
    # where they disagree the distances must be near-ties
    bad = torch.nonzero(got != ref).reshape(-1)
    if bad.numel():
        dg = D[bad, got[bad]]
        dr = D[bad, ref[bad]]
        assert torch.all((dg - dr).abs() <= 1e-3 * dr.abs() + 1e-2)
    mr = D.min(1).values
    assert torch.allclose(mind.cpu().double(), mr, rtol=2e-3, atol=1e-2)
    # inertia accumulator
    assert abs(buf.inertia.item() - mind.double().sum().item()) < 1e-3 * mind.double().sum().item()


@pytest.mark.parametrize("d,k", [(32, 192), (256, 1024)])
def test_estep_persistent_many_blocks(cuda, d, k):
    """n far above the resident grid: every workgroup walks many row blocks
    (continuous tile ring across blocks, early next-block X loads)."""
    n = 300_001
    g = torch.Generator(device=cuda).manual_seed(11)
    C = torch.randn(k, d, device=cuda, generator=g) * 3
    lab0 = torch.randint(0, k, (n,), device=cuda, generator=g)
    dp, kp = K.pad_features(d), K.pad_clusters(k)
    Xb = torch.zeros(n, dp, dtype=torch.bfloat16, device=cuda)
    Xb[:, :d] = (C[lab0] + torch.randn(n, d, device=cuda, generator=g)).to(torch.bfloat16)
    Cb, cn = K.centers_to_bf16(C, kp, dp)
    xn = L.row_norms_sq(Xb)
    buf = K.EStepBuffers(n, cuda)
    key = RngKey(2, "band_select", 0)
    lab, mind = K.estep_native(Xb, Cb, cn, xn, k, 0.0, key, 0, buf)
    torch.cuda.synchronize()
    Cr = K.centers_from_operand(Cb, k, d).double()
    ok = 0
    for s0 in range(0, n, 65536):
        xr = Xb[s0:s0 + 65536, :d].double()
        D = (xr * xr).sum(1, keepdim=True) + (Cr * Cr).sum(1)[None] - 2 * xr @ Cr.T
        got = lab[s0:s0 + 65536].long()
        ref = D.argmin(1)
        agree = got == ref
        ok += int(agree.sum())
        dg = D.gather(1, got.clamp(min=0)[:, None])[:, 0]
        dr = D.min(1).values
        assert (got >= 0).all()
        assert torch.all((dg - dr)[~agree] <= 1e-3 * dr[~agree].abs() + 1e-2)
        assert torch.allclose(mind[s0:s0 + 65536].double(), dr, rtol=2e-3, atol=1e-2)
    assert ok / n > 0.999
    assert abs(buf.inertia.item() - mind.double().sum().item()) < 1e-4 * mind.double().sum().item()


def test_estep_band_semantics(cuda):
    n, d, k = 20000, 32, 64
    g = torch.Generator().manual_seed(3)
    # clustered distances: several centroids near each point -> real bands
    C = torch.randn(k, d, generator=g, dtype=torch.float64) * 0.3
    X = torch.randn(n, d, generator=g, dtype=torch.float64) * 0.3
    delta = 0.5
    dp, kp = K.pad_features(d), K.pad_clusters(k)
    Xb = X.to(torch.bfloat16)
    Cb, cn = K.centers_to_bf16(C.float(), kp, dp)
    Xg = Xb.to(cuda)
    xn = L.row_norms_sq(Xg)
    buf = K.EStepBuffers(n, cuda)
    key = RngKey(7, "band_select", 0)
    lab, mind = K.estep_native(Xg, Cb.to(cuda), cn.to(cuda), xn, k, delta, key, 0, buf)
    torch.cuda.synchronize()
    D = K.distances_torch(Xb.double(), K.centers_from_operand(Cb, k, d).double())
    mn = D.min(1).values
    got = lab.cpu().long()
    assert (got >= 0).all() and (got < k).all()
    chosen = D[torch.arange(n), got]
    assert torch.all(chosen <= mn + delta + 1e-2 * (1 + mn.abs()))
    # uniformity: among rows with a band of size >= 2, the chosen member is not
    # always the argmin
    band = (D <= (mn + delta)[:, None]).sum(1)
    multi = band >= 2
    assert multi.float().mean() > 0.2
    frac_argmin = (got[multi] == D[multi].argmin(1)).float().mean().item()
    expect = (1.0 / band[multi].double()).mean().item()
    assert abs(frac_argmin - expect) < 0.05, (frac_argmin, expect)
    # torch CPU selection with the same keys agrees on the large majority
    lab_cpu, _ = K.band_select_torch(D.float(), torch.arange(n), delta, key, kp)
    # same rank rule and Philox words: identical except fp near-ties at the band edge
    assert (lab_cpu == got).float().mean() > 0.995


def test_centroid_accumulate(cuda):
    n, d, k = 50000, 256, 300
    X = torch.randn(n, d, dtype=torch.float32, device=cuda)
    lab = torch.randint(0, k, (n,), dtype=torch.int32, device=cuda)
    sums = torch.zeros(k, d, dtype=torch.float32, device=cuda)
    cnt = torch.zeros(k, dtype=torch.float64, device=cuda)
    K.centroid_accumulate_native(X, lab, None, sums, cnt, k)
    rs, rc = K.centroid_sums_torch(X.double(), lab, k)
    assert torch.allclose(sums.double(), rs, atol=1e-3)
    assert torch.equal(cnt, rc)
    Xb = X.to(torch.bfloat16)
    sums.zero_(); cnt.zero_()
    K.centroid_accumulate_native(Xb, lab, None, sums, cnt, k)
    rs, _ = K.centroid_sums_torch(Xb.double(), lab, k)
    assert torch.allclose(sums.double(), rs, atol=1e-3)


@pytest.mark.parametrize("dtype,d", [(torch.float32, 256), (torch.bfloat16, 256), (torch.float32, 20),
                                     (torch.bfloat16, 512)])
def test_centroid_reduce(cuda, dtype, d):
    n, k = 70001, 1000
    X = torch.randn(n, d, dtype=torch.float32, device=cuda).to(dtype)
    lab = torch.randint(0, k, (n,), dtype=torch.int32, device=cuda)
    lab[:5000] = 3  # a big cluster
    w = torch.rand(n, dtype=torch.float32, device=cuda)
    packed = torch.zeros(k * d + k + 1, dtype=torch.float64, device=cuda)
    for weights in (None, w):
        ws = K.ReduceWorkspace(n, k, cuda).set_scale(float(X.float().abs().max()), n,
                                                     None if weights is None else 1.0)
        outs = []
        for rep in range(2):
            sums = torch.zeros(k, d, dtype=torch.float64, device=cuda)
            cnt = torch.zeros(k, dtype=torch.float64, device=cuda)
            K.centroid_reduce_native(X, lab, weights, sums, cnt, k, ws)
            outs.append((sums.clone(), cnt.clone()))
        # exact integer-valued accumulation: bit-identical run to run
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
        K.pack_stats_native(outs[0][0], outs[0][1], None, packed, k, d, ws,
                            weighted=weights is not None)
        rs, rc = K.centroid_sums_torch(X.double(), lab, k, weights)
        got_s = packed[:k * d].reshape(k, d)
        got_c = packed[k * d:k * d + k]
        # error: fp32 product w*x per element, then a 2^-30-ish quantum
        assert torch.allclose(got_s, rs, atol=1e-4, rtol=1e-6)
        assert torch.allclose(got_c, rc, rtol=1e-6, atol=1e-6)
        if weights is None:
            assert torch.equal(got_c, rc)


def test_finalize_noise_and_shift(cuda):
    k, d = 70, 48
    ws = K.ReduceWorkspace(1, k, cuda, xexp=-20)
    sums_f = torch.randn(k, d, dtype=torch.float64, device=cuda)
    sums_i = torch.round(sums_f * 2.0 ** 20)
    sums = (sums_i.double() * 2.0 ** -20).float()
    cnt_i = torch.randint(1, 5, (k,), device=cuda).double()
    cnt_i[3] = 0
    cnt = cnt_i.double()
    inertia = torch.tensor([5.0], dtype=torch.float64, device=cuda)
    packed = torch.zeros(k * d + k + 1, dtype=torch.float64, device=cuda)
    K.pack_stats_native(sums_i, cnt_i, inertia, packed, k, d, ws)
    assert torch.equal(packed[:k * d].reshape(k, d), sums_i.double() * 2.0 ** -20)
    assert packed[-1].item() == 5.0
    Cold = torch.randn(k, d, dtype=torch.float32, device=cuda)
    Cnew = torch.empty_like(Cold)
    kp, dp = K.pad_clusters(k), K.pad_features(d)
    Cb = torch.full(K.operand_shape(kp, dp), 7.0, dtype=torch.bfloat16, device=cuda)
    cn = torch.empty(kp, dtype=torch.float32, device=cuda)
    shift = torch.zeros(1, dtype=torch.float64, device=cuda)
    b = 0.05
    K.centroid_finalize_native(packed, Cold, Cnew, Cb, cn, shift, k, d, b, RngKey(1, "trunc_normal", 2))
    ref = sums.double() / cnt.clamp(min=1)[:, None]
    ref[3] = Cold[3].double()
    diff = (Cnew.double() - ref)
    assert diff.abs().max().item() <= b + 1e-5
    assert diff.abs().max().item() > 0.5 * b
    assert abs(shift.item() - ((Cnew.double() - Cold.double()) ** 2).sum().item()) < 1e-3
    Ch = K.centers_from_operand(Cb, k, d)
    assert torch.equal(Ch, Cnew.to(torch.bfloat16))
    assert torch.allclose(cn[:k], (Ch.float() ** 2).sum(1), rtol=1e-5)
    assert (cn[k:] > 1e37).all()
    # the device-written E-step operand equals the host-built one bit for bit
    # (norm split may differ in the last bit of lo via the fp32 sum order)
    ref_op, _ = K.centers_to_bf16(Cnew, kp, dp)
    body = (slice(None), slice(0, dp // 8))
    assert torch.equal(Cb[body], ref_op[body])
    nb = Cb[:, dp // 8].permute(0, 1, 2).reshape(kp, 8).float()
    assert torch.allclose(nb[:k, :3].sum(1), cn[:k], rtol=1e-6)
    assert (nb[:, 3:] == 0).all() and (Cb[:, dp // 8 + 1] == 0).all()


def test_ipe_estep_kernel(cuda):
    n, d, k = 300, 16, 6
    X, C = _data(n, d, k, 5, cuda)
    G = (X @ C.T).float().to(cuda)
    xn = (X * X).sum(1).float().to(cuda)
    cn = (C * C).sum(1).float().to(cuda)
    lab = torch.empty(n, dtype=torch.int32, device=cuda)
    mind = torch.empty(n, dtype=torch.float32, device=cuda)
    K.ipe_estep_native(G, xn, cn, 0.05, 13, RngKey(2, "ipe", 0), 0, lab, mind)
    torch.cuda.synchronize()
    ref = K.distances_torch(X, C).argmin(1)
    assert (lab.cpu().long() == ref).float().mean() > 0.95


def test_qmeans_gpu_vs_cpu(cuda):
    from sq_learn_amd.models.cluster import QMeans
    from sq_learn_amd.utils.datasets import make_blobs
    X, y = make_blobs(6000, 64, centers=10, random_state=0)
    kw = dict(n_clusters=10, delta=0.5, true_distance_estimate=False, intermediate_error=True,
              true_tomography=False, random_state=1, n_init=1, init="k-means++")
    g = QMeans(device="cuda", **kw).fit(X)
    c = QMeans(device="cpu", **kw).fit(X)
    assert abs(g.inertia_ - c.inertia_) / c.inertia_ < 0.02
    from sklearn.metrics import adjusted_rand_score
    assert adjusted_rand_score(g.labels_, c.labels_) > 0.99
    assert adjusted_rand_score(g.labels_, y) > 0.99


def test_gram_power_mu_rownorm(cuda):
    n, d = 12345, 200
    X = torch.randn(n, d, dtype=torch.float32, device=cuda) * 2 + 1
    mean = X.double().mean(0)
    G = L.gram_local(X, mean)
    Xc = X.double() - mean
    Gr = Xc.T @ Xc
    assert torch.allclose(G.double(), Gr, rtol=1e-11, atol=1e-9 * Gr.abs().max().item())
    Q = torch.randn(d, 40, dtype=torch.float32, device=cuda)
    Z = L.power_iter_local(X, Q, mean)
    Zr = Xc.T @ (Xc @ Q.double())
    assert torch.allclose(Z.double(), Zr, rtol=1e-10, atol=1e-10 * Zr.abs().max().item())
    exps = [round(0.2 * i, 10) for i in range(11)]
    rm, cs = L.mu_power_sums_local(X, exps)
    rm2, cs2 = L.mu_power_sums_local(X.cpu(), exps)
    assert torch.allclose(rm.cpu(), rm2, rtol=1e-4)
    assert torch.allclose(cs.cpu(), cs2, rtol=1e-4)
    rn = L.row_norms_sq(X.to(torch.bfloat16))
    assert torch.allclose(rn.double().cpu(), (X.to(torch.bfloat16).double() ** 2).sum(1).cpu(), rtol=1e-5)


@pytest.mark.parametrize("d,dtype", [(32, torch.bfloat16), (30, torch.float32), (128, torch.bfloat16),
                                     (256, torch.float32), (5, torch.float32), (512, torch.bfloat16),
                                     (784, torch.float32), (1030, torch.float32)])
def test_mu_power_sums_shapes(cuda, d, dtype):
    """Every d: one launch per 512-column block beyond 512 (row power sums
    carried across the blocks)."""
    n = 50_003
    X = (torch.randn(n, d, device=cuda) * 3).to(dtype)
    X[::7, 0] = 0   # zeros: q = 0 counts nonzeros
    exps = [0.0, 0.1, 0.2, 1.0, 1.8, 1.9, 2.0]
    rm, cs = L.mu_power_sums_local(X, exps)
    rm2, cs2 = L.mu_power_sums_local(X.float().cpu(), exps)
    assert torch.allclose(rm.cpu(), rm2, rtol=2e-4)
    # strided rows (a column slice of a wider matrix)
    W = torch.zeros(n, d + 3, device=cuda, dtype=dtype)
    W[:, 1:d + 1] = X
    rs, css = L.mu_power_sums_local(W[:, 1:d + 1], exps)
    assert torch.allclose(rs.cpu(), rm2, rtol=2e-4) and torch.allclose(css.cpu(), cs2, rtol=2e-4)
    assert torch.allclose(cs.cpu(), cs2, rtol=2e-4)
    # deterministic (no float atomics in the column sums)
    rm3, cs3 = L.mu_power_sums_local(X, exps)
    assert torch.equal(cs, cs3) and torch.equal(rm, rm3)
