"""Certified fp16 IPE screen (csrc/ipe16.hip, ``ops.kmeans.Ipe16``): the
reference's default distance mode (``_dmeans.py:753-772`` ->
``Utility.py:697-737``) without a per-pair fp32 inner product.

* law: the (label, min D~) law of n copies of one row equals the full
  sampler's of the fp32 fused kernel (csrc/ipe.hip, prune off) - many
  centroids, a hazard target large enough that far pairs fire and reach the
  exact branch, and rows the screen leaves dense (fp32 row-group fallback);
* exact two-centroid law (pair 1 a few bins above the hint);
* invariance: labels and estimates are bit-identical however the rows are
  chunked and wherever the shard starts (global-row keyed streams)."""
import math

import numpy as np
import pytest
import torch
from scipy import stats

from sq_learn_amd.ops import kmeans as K
from sq_learn_amd.runtime.rng import RngKey

pytestmark = pytest.mark.gpu


def _keys(seed):
    return (RngKey(seed, "ipe", 0), RngKey(seed, "band_select", 0), RngKey(seed, "ipe16_skip", 0),
            RngKey(seed, "ipe16_row", 0), RngKey(seed, "ipe_skip", 0))


def _run16(X, C, eps, Q, seed, hint=None, row_offset=0, stats_t=None, ht=None, X_sub=None):
    """labels, mind (numpy) of the Ipe16 E-step over X's rows (tensors on the
    GPU); ``hint`` None: the fp16 argmin sweep first."""
    n, d = X.shape
    k = C.shape[0]
    d_pad, k_pad = K.pad_features(d), K.pad_clusters(k)
    xn = (X.double() ** 2).sum(1).float().contiguous()
    cn = (C * C).sum(1).contiguous()
    mx = float(xn.max())
    st = K.Ipe16(X, k, d_pad, k_pad, K.choose_alpha(mx, 0.0), X.device)
    if ht is not None:
        st.ht = ht
    st.set_centers(C)
    hint_t = (torch.full((n,), -1, dtype=torch.int32, device=X.device) if hint is None
              else hint.clone())
    lab = torch.empty(n, dtype=torch.int32, device=X.device)
    mind = torch.empty(n, dtype=torch.float32, device=X.device)
    key, tie, skey, bkey, okey = _keys(seed)

    def fallback(rl, rc, ln, thr, hj, s, e):
        dp = 32
        while dp < d:
            dp *= 2
        kp = -(-k // 16) * 16
        K.ipe_fused_native(X[s:e], K.ipe_center_fragments(C, kp, dp), xn[s:e], cn, k, kp, dp, eps,
                           Q, key, tie, row_offset + s, lab[s:e], mind[s:e], C=C, skip_key=okey,
                           rows=(rl, rc, ln), ext=(thr, hj))

    st.estep(X, C, hint_t, xn, cn, lab, mind, eps, Q, key, tie, skey, bkey, row_offset,
             hint is None, stats=stats_t, fallback=fallback)
    torch.cuda.synchronize()
    return lab.cpu().numpy(), mind.double().cpu().numpy(), st


def _run_full(X, C, eps, Q, seed):
    """The fp32 fused kernel with pruning off: every pair sampled in full."""
    n, d = X.shape
    k = C.shape[0]
    dp = 32
    while dp < d:
        dp *= 2
    kp = -(-k // 16) * 16
    xn = (X.double() ** 2).sum(1).float()
    cn = (C * C).sum(1)
    lab = torch.empty(n, dtype=torch.int32, device=X.device)
    mind = torch.empty(n, dtype=torch.float32, device=X.device)
    K.ipe_fused_native(X, K.ipe_center_fragments(C, kp, dp), xn, cn, k, kp, dp, eps, Q,
                       RngKey(seed, "ipe", 0), RngKey(seed, "band_select", 0), 0, lab, mind,
                       prune=False)
    torch.cuda.synchronize()
    return lab.cpu().numpy(), mind.double().cpu().numpy()


def _same_law(la, ma, lb, mb, min_cells=3):
    n = la.size
    ka = la.astype(np.int64) * 10**9 + np.round(ma * 1e3).astype(np.int64)
    kb = lb.astype(np.int64) * 10**9 + np.round(mb * 1e3).astype(np.int64)
    keys, inv = np.unique(np.concatenate([ka, kb]), return_inverse=True)
    ca = np.bincount(inv[:n], minlength=len(keys))
    cb = np.bincount(inv[n:], minlength=len(keys))
    keep = (ca + cb) >= 20
    table = np.stack([np.append(ca[keep], ca[~keep].sum()), np.append(cb[keep], cb[~keep].sum())])
    table = table[:, table.sum(0) > 0]
    assert table.shape[1] >= min_cells
    return stats.chi2_contingency(table)[1]


def _row_and_centroids(seed, d, k, spread, scale=1.5):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(d).astype(np.float32)
    C = (x[None] + rng.uniform(0.7, 1.3, (k, 1)) * rng.standard_normal((k, d)) / math.sqrt(d)
         * scale * spread)
    return x, C.astype(np.float32)


@pytest.mark.parametrize("Q", [13, 17])
def test_ipe16_matches_full_sampler_law_many_centroids(cuda, Q):
    """k = 40 centroids around the row (eps = 0.1, Q = 13 / 17: every pair
    near the hint, all listed and sampled in full): the (label, D~) law
    equals the full sampler's."""
    x, C = _row_and_centroids(12, 40, 40, 1.0)
    n = 400_000
    X = torch.tensor(np.tile(x, (n, 1)), device=cuda)
    Ct = torch.tensor(C, device=cuda)
    st = torch.zeros(8, dtype=torch.int64, device=cuda)
    la, ma, eng = _run16(X, Ct, 0.1, Q, 1, stats_t=st)
    lb, mb = _run_full(X, Ct, 0.1, Q, 2)
    assert eng.last_dense == 0, st.tolist()
    # (Q = 17 concentrates the median: fewer populated cells)
    assert _same_law(la, ma, lb, mb, min_cells=3 if Q == 13 else 2) > 1e-4


def _fire_case(d=96, K_=301, s=12.0):
    """Pair 0 near x (the hint), K_ - 1 competitors at distance s on
    orthonormal directions orthogonal to x: all in the far band, each with a
    hazard ~ 4e-4 against the row's band-edge bound (eps = 0.25)."""
    rng = np.random.default_rng(21)
    x = rng.standard_normal(d)
    B = rng.standard_normal((d, K_))
    B -= np.outer(x, x @ B) / (x @ x)
    B /= np.linalg.norm(B, axis=0, keepdims=True)   # unit directions orthogonal to x
    C = np.empty((K_, d))
    C[0] = x + 0.9 * B[:, 0]
    C[1:] = x[None] + s * B[:, 1:].T
    return x.astype(np.float32), C.astype(np.float32)


def test_ipe16_fire_path_matches_full_sampler_law(cuda):
    """A far band with hazard target 9e-4 over 300 competitors: ~1/4 of the
    rows list a fired far pair and some reach the exact branch; the (label,
    D~) law equals the full sampler's."""
    x, C = _fire_case()
    n = 400_000
    X = torch.tensor(np.tile(x, (n, 1)), device=cuda)
    Ct = torch.tensor(C, device=cuda)
    hint = torch.zeros(n, dtype=torch.int32, device=cuda)
    st = torch.zeros(8, dtype=torch.int64, device=cuda)
    la, ma, eng = _run16(X, Ct, 0.25, 13, 5, hint=hint, stats_t=st, ht=9e-4)
    s = st.tolist()
    # nothing near but the hint, except rows whose sampled threshold lands in
    # an unusually high class (their band excludes the competitors: dense)
    assert eng.last_dense < 1e-3 * n and s[0] == 0, s
    assert s[1] > 0.05 * n and s[2] > 100 and s[4] > 0.05 * n, s
    lb, mb = _run_full(X, Ct, 0.25, 13, 6)
    assert _same_law(la, ma, lb, mb, min_cells=2) > 1e-4


def test_ipe16_two_centroid_exact_law(cuda):
    """Pair 0 is the hint; pair 1 a few bins above it: the joint law of
    (label, min D~) is that of min(V0, V1) (the fused kernel's exact test)."""
    from test_ipe_fused_gpu import _exact_law
    rng = np.random.default_rng(11)
    d, eps, Q = 48, 0.02, 3
    x = rng.standard_normal(d).astype(np.float32)
    u = rng.standard_normal(d)
    u -= (u @ x) / (x @ x) * x
    u /= np.linalg.norm(u)
    c0 = (x + 0.9 * u).astype(np.float32)
    c1 = (x - 1.6 * u).astype(np.float32)
    n = 1_000_000
    X = torch.tensor(np.tile(x, (n, 1)), device=cuda)
    Ct = torch.tensor(np.stack([c0, c1]), device=cuda)
    hint = torch.zeros(n, dtype=torch.int32, device=cuda)
    lab, mind, _ = _run16(X, Ct, eps, Q, 0, hint=hint)
    xn = float((X[0].double() ** 2).sum().float())
    cn = (Ct.double() ** 2).sum(1).float().double().cpu().numpy()
    ip = (Ct.double() @ X[0].double()).cpu().numpy()
    M0, v0, p0 = _exact_law(ip[0], xn, cn[0], eps, Q)
    M1, v1, p1 = _exact_law(ip[1], xn, cn[1], eps, Q)
    F1 = np.array([p1[v1 < v].sum() for v in v0])
    G0 = np.array([p0[v0 > v].sum() for v in v1])
    cells_e = np.concatenate([p0 * (1 - F1), p1 * G0])
    vals = np.concatenate([v0, v1])
    labs = np.concatenate([np.zeros_like(v0), np.ones_like(v1)])
    P1 = (p1 * G0).sum()
    assert 1e-4 < P1 < 0.2, P1
    obs = np.zeros(len(vals))
    for L in (0, 1):
        sel = lab == L
        cand = np.where(labs == L)[0]
        idx = cand[np.argmin(np.abs(mind[sel][:, None] - vals[cand][None, :]), axis=1)]
        assert np.allclose(mind[sel], vals[idx], rtol=2e-6, atol=1e-5)
        obs += np.bincount(idx, minlength=len(vals))
    exp = cells_e * n
    big = exp >= 5
    o = np.append(obs[big], obs[~big].sum())
    e = np.append(exp[big], exp[~big].sum())
    chi2 = ((o - e) ** 2 / e).sum()
    assert stats.chi2.sf(chi2, len(e) - 1) > 1e-4


def test_ipe16_dense_rows_take_the_fp32_kernel(cuda):
    """200 centroids crowded around the row (every pair competitive): the
    rows are dense for the screen and the fp32 row-group kernel's list mode
    resolves them - same law as the full sampler."""
    x, C = _row_and_centroids(5, 32, 200, 0.15)
    n = 200_000
    X = torch.tensor(np.tile(x, (n, 1)), device=cuda)
    Ct = torch.tensor(C, device=cuda)
    st = torch.zeros(8, dtype=torch.int64, device=cuda)
    la, ma, eng = _run16(X, Ct, 0.25, 13, 3, stats_t=st)
    assert eng.last_dense == n, (eng.last_dense, st.tolist())
    lb, mb = _run_full(X, Ct, 0.25, 13, 4)
    assert _same_law(la, ma, lb, mb) > 1e-4


@pytest.mark.parametrize("with_hint", [False, True])
def test_ipe16_rows_invariant_to_chunks_and_offsets(cuda, monkeypatch, with_hint):
    """Blob data (some dense rows, some fires): labels and estimates are
    bit-identical with small launch chunks and for a shard starting at
    global row 7."""
    rng = np.random.default_rng(31)
    n, d, k, eps, Q = 20000, 64, 200, 0.25, 13
    ctr = rng.standard_normal((20, d)) * 3
    X = (ctr[rng.integers(0, 20, n)] + rng.standard_normal((n, d))).astype(np.float32)
    Cn = (ctr[rng.integers(0, 20, k)] + 0.5 * rng.standard_normal((k, d))).astype(np.float32)
    Xt = torch.tensor(X, device=cuda)
    Ct = torch.tensor(Cn, device=cuda)
    hint = (torch.tensor(rng.integers(0, k, n).astype(np.int32), device=cuda) if with_hint
            else None)
    st = torch.zeros(8, dtype=torch.int64, device=cuda)
    la, ma, e1 = _run16(Xt, Ct, eps, Q, 9, hint=hint, stats_t=st, ht=5e-4)
    monkeypatch.setattr(K, "IPE16_CHUNK", 4096)
    lb, mb, _ = _run16(Xt, Ct, eps, Q, 9, hint=hint, ht=5e-4)
    lc, mc, _ = _run16(Xt[7:], Ct, eps, Q, 9, hint=None if hint is None else hint[7:],
                       row_offset=7, ht=5e-4)
    assert np.array_equal(la, lb) and np.array_equal(ma, mb)
    if with_hint:
        assert np.array_equal(la[7:], lc) and np.array_equal(ma[7:], mc)
    else:
        # argmin hints depend only on the row: the same from row 7 on
        assert np.array_equal(la[7:], lc) and np.array_equal(ma[7:], mc)
    s = st.tolist()
    assert s[0] > 0, s


def test_ipe16_lloyd_trajectory_matches_fp32_kernel(cuda, monkeypatch):
    """Blob data (256 centroids in 4 norm groups, some groups without a band
    for some rows): the Lloyd trajectory's inertia with the screen follows
    the fp32 fused kernel's to within the law's (tiny) sampling noise."""
    from sq_learn_amd.models.cluster._lloyd import LloydEngine
    from sq_learn_amd.utils.datasets import make_blobs_device
    from sq_learn_amd.models._data import Data, gather_rows
    from sq_learn_amd.parallel.comm import Comm
    n, d, k = 200_000, 64, 256
    X, _ = make_blobs_device(n, d, centers=k, cluster_std=1.0, seed=1, device=cuda,
                             dtype=torch.float32)
    C0 = gather_rows(Data(X, n, 0, Comm(None), "sharded"),
                     np.random.RandomState(1).choice(n, k, replace=False))
    out = {}
    for use16 in ("0", "1"):
        monkeypatch.setenv("SQ_IPE16", use16)
        eng = LloydEngine(X, k, delta=0.5, true_distance_estimate=True, intermediate_error=True,
                          seed=3)
        eng.set_centers(C0)
        out[use16] = [eng.step()[1].tolist()[0] for _ in range(4)]
    a, b = np.array(out["0"]), np.array(out["1"])
    assert np.all(np.abs(a - b) <= 2e-3 * a), (a, b)
