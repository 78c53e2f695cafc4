"""Fused IPE E-step (csrc/ipe.hip) - the reference's default distance mode
(``_dmeans.py:753-772`` -> ``Utility.py:697-737``).

Law tests: with one centroid the kernel's per-row output IS the estimated
distance D~ = 2 S a~ of that pair, so n identical rows give n iid draws of
the median-of-Q amplitude-estimation law.  It is compared (chi^2) with the
EXACT law computed from the Fejer pmf (fejer_pmf, the reference's p_aj) and
with the CPU twin (ops/kmeans.py ipe_estep_torch), on pairs whose M falls
in the exact median-law walk (M <= 128) and in the draw path (large M, even Q).
"""
import math

import numpy as np
import pytest
import torch
from scipy import stats

from sq_learn_amd.ops import kmeans as K
from sq_learn_amd.quantum.fejer import fejer_pmf, ae_bins
from sq_learn_amd.runtime.rng import RngKey

pytestmark = pytest.mark.gpu


def _exact_law(ip, nx2, ny2, eps, Q):
    """{D~ value: probability} of the median of Q AE draws."""
    S = nx2 + ny2
    a = min(max((S - 2 * ip) / (2 * S), 0.0), 1.0)
    eps_a = eps * max(1.0, abs(ip)) / S
    M = int(ae_bins(a, eps_a))
    omega = M * math.asin(math.sqrt(a)) / math.pi
    p = fejer_pmf(omega, M)
    p = p / p.sum()
    t = np.minimum(np.arange(M), M - np.arange(M))
    mass = np.bincount(t, weights=p)              # value classes t = 0..M/2
    F = np.cumsum(mass)
    h = (Q + 1) // 2
    G = stats.binom.sf(h - 1, Q, np.clip(F, 0, 1)) if Q % 2 else None
    vals = 2 * S * np.sin(np.pi * np.arange(len(mass)) / M) ** 2
    if Q % 2:
        pm = np.diff(np.concatenate([[0.0], G]))
        return M, vals, pm
    return M, vals, None


def _run_kernel(x, c, n, eps, Q, cuda, seed=0):
    d = x.size
    X = torch.tensor(np.tile(x, (n, 1)), dtype=torch.float32, device=cuda)
    C = torch.tensor(c[None], dtype=torch.float32, device=cuda)
    dp = 32
    while dp < d:
        dp *= 2
    assert dp <= 2048
    xn = (X.double() ** 2).sum(1).float()
    cn = (C.double() ** 2).sum(1).float()
    lab = torch.empty(n, dtype=torch.int32, device=cuda)
    mind = torch.empty(n, dtype=torch.float32, device=cuda)
    K.ipe_fused_native(X, K.ipe_center_fragments(C, 16, dp), xn, cn, 1, 16, dp, eps, Q,
                       RngKey(seed, "ipe", 0), RngKey(seed, "band_select", 0), 0, lab, mind)
    torch.cuda.synchronize()
    assert int(lab.max()) == 0
    return mind.double().cpu().numpy(), float(xn[0]), float(cn[0]), float((X[0].double() @ C[0].double()))


def _gof(samples, vals, pm):
    idx = np.argmin(np.abs(samples[:, None] - vals[None, :]), axis=1)
    assert np.allclose(samples, vals[idx], rtol=2e-6, atol=1e-5)
    obs = np.bincount(idx, minlength=len(vals)).astype(float)
    exp = pm * len(samples)
    big = exp >= 5
    o = np.append(obs[big], obs[~big].sum())
    e = np.append(exp[big], exp[~big].sum())
    if e[-1] == 0:
        o, e = o[:-1], e[:-1]
    chi2 = ((o - e) ** 2 / e).sum()
    return stats.chi2.sf(chi2, max(len(e) - 1, 1))


@pytest.mark.parametrize("case", ["walk", "walk_q1", "draws"])
def test_ipe_fused_law_exact(cuda, case):
    rng = np.random.default_rng(1)
    d = 200
    x = rng.standard_normal(d)
    if case.startswith("walk"):
        c = x + 0.8 * rng.standard_normal(d)      # |ip| ~ S/2 -> M ~ 30
        eps = 0.25
    else:
        c = rng.standard_normal(d)                  # nearly orthogonal -> small eps_a, large M
        eps = 0.25
    Q = 1 if case == "walk_q1" else 13
    n = 60000
    s, nx2, ny2, ip = _run_kernel(x, c, n, eps, Q, cuda)
    M, vals, pm = _exact_law(ip, nx2, ny2, eps, Q)
    if case.startswith("walk"):
        assert M <= 128
    else:
        assert M > 128
    if Q == 1:
        # single draw: value class law = class masses
        S = nx2 + ny2
        a = min(max((S - 2 * ip) / (2 * S), 0.0), 1.0)
        omega = M * math.asin(math.sqrt(a)) / math.pi
        p = fejer_pmf(omega, M)
        t = np.minimum(np.arange(M), M - np.arange(M))
        pm = np.bincount(t, weights=p / p.sum())
    assert _gof(s, vals, pm) > 1e-4


def test_ipe_fused_even_q_matches_cpu_twin(cuda):
    rng = np.random.default_rng(2)
    d = 64
    x = rng.standard_normal(d)
    c = x + 0.5 * rng.standard_normal(d)
    n = 20000
    g, *_ = _run_kernel(x, c, n, 0.3, 4, cuda)
    X = torch.tensor(np.tile(x, (3000, 1)), dtype=torch.float32)
    C = torch.tensor(c[None], dtype=torch.float32)
    _, mind = K.ipe_estep_torch(X, C, 0.3, RngKey(5, "ipe", 0), 0, 16, Q=4)
    a = np.round(g, 3)
    b = np.round(mind.numpy(), 3)
    vals, inv = np.unique(np.concatenate([a, b]), return_inverse=True)
    ca = np.bincount(inv[: len(a)], minlength=len(vals))
    cb = np.bincount(inv[len(a):], minlength=len(vals))
    keep = (ca + cb) >= 10
    table = np.stack([np.append(ca[keep], ca[~keep].sum()), np.append(cb[keep], cb[~keep].sum())])
    table = table[:, table.sum(0) > 0]
    assert stats.chi2_contingency(table)[1] > 1e-4


def test_ipe_fused_argmin_and_inertia(cuda):
    """Many centroids: the label is the argmin of the per-pair estimates;
    with a small eps the estimates are close to the true distances."""
    rng = np.random.default_rng(3)
    n, d, k = 4096, 48, 70
    centers = rng.standard_normal((k, d)) * 4
    X = centers[rng.integers(0, k, n)] + 0.3 * rng.standard_normal((n, d))
    Xt = torch.tensor(X, dtype=torch.float32, device=cuda)
    Ct = torch.tensor(centers, dtype=torch.float32, device=cuda)
    xn = (Xt.double() ** 2).sum(1).float()
    cn = (Ct.double() ** 2).sum(1).float()
    lab = torch.empty(n, dtype=torch.int32, device=cuda)
    mind = torch.empty(n, dtype=torch.float32, device=cuda)
    K.ipe_fused_native(Xt, K.ipe_center_fragments(Ct, 80, 64), xn, cn, k, 80, 64, 0.05, 13,
                       RngKey(7, "ipe", 0), RngKey(7, "band_select", 0), 0, lab, mind)
    D = ((X[:, None, :] - centers[None]) ** 2).sum(-1)
    true = D.argmin(1)
    assert np.mean(lab.cpu().numpy() == true) > 0.99
    m = mind.cpu().numpy()
    assert np.median(np.abs(m - D.min(1)) / D.min(1).clip(1)) < 0.5


def test_qmeans_ipe_end_to_end_gpu(cuda):
    from sq_learn_amd.models.cluster import QMeans
    from sq_learn_amd.utils.datasets import make_blobs
    from sklearn.metrics import adjusted_rand_score
    X, y = make_blobs(6000, 32, centers=6, cluster_std=1.0, random_state=0)
    kw = dict(n_clusters=6, delta=0.5, true_distance_estimate=True, random_state=0, n_init=1,
              max_iter=10, init="k-means++")
    g = QMeans(device=cuda, **kw).fit(X)
    c = QMeans(device="cpu", **kw).fit(X)
    assert adjusted_rand_score(y, g.labels_) > 0.95
    assert adjusted_rand_score(y, c.labels_) > 0.95
    assert abs(g.inertia_ - c.inertia_) < 0.1 * c.inertia_


@pytest.mark.parametrize("d", [384, 784])
def test_ipe_fused_law_exact_wide(cuda, d):
    """d_pad 512 / 1024: the workgroup-shared A tile; same exact median law."""
    rng = np.random.default_rng(d)
    x = rng.standard_normal(d)
    c = x + 0.8 * rng.standard_normal(d)
    s, nx2, ny2, ip = _run_kernel(x, c, 40000, 0.25, 13, cuda, seed=3)
    M, vals, pm = _exact_law(ip, nx2, ny2, 0.25, 13)
    assert M <= 128
    assert _gof(s, vals, pm) > 1e-4


def test_ipe_fused_argmin_wide(cuda):
    rng = np.random.default_rng(4)
    n, d, k = 2048, 600, 40
    centers = rng.standard_normal((k, d)) * 4
    X = centers[rng.integers(0, k, n)] + 0.3 * rng.standard_normal((n, d))
    Xt = torch.tensor(X, dtype=torch.float32, device=cuda)
    Ct = torch.tensor(centers, dtype=torch.float32, device=cuda)
    xn = (Xt.double() ** 2).sum(1).float()
    cn = (Ct.double() ** 2).sum(1).float()
    lab = torch.empty(n, dtype=torch.int32, device=cuda)
    mind = torch.empty(n, dtype=torch.float32, device=cuda)
    K.ipe_fused_native(Xt, K.ipe_center_fragments(Ct, 48, 1024), xn, cn, k, 48, 1024, 0.05, 13,
                       RngKey(7, "ipe", 0), RngKey(7, "band_select", 0), 0, lab, mind)
    D = ((X[:, None, :] - centers[None]) ** 2).sum(-1)
    assert np.mean(lab.cpu().numpy() == D.argmin(1)) > 0.99


# ------------------------------------------------------------------ pruning
def _run_rows(x, C, n, eps, Q, cuda, seed, prune, hint=None, stats=None):
    d = x.size
    dp = 32
    while dp < d:
        dp *= 2
    k = C.shape[0]
    kp = -(-k // 16) * 16
    X = torch.tensor(np.tile(x, (n, 1)), dtype=torch.float32, device=cuda)
    Ct = torch.tensor(C, dtype=torch.float32, device=cuda)
    xn = (X.double() ** 2).sum(1).float()
    cn = (Ct.double() ** 2).sum(1).float()
    lab = torch.empty(n, dtype=torch.int32, device=cuda)
    mind = torch.empty(n, dtype=torch.float32, device=cuda)
    hl = None
    if hint is not None:
        hl = torch.as_tensor(np.broadcast_to(np.asarray(hint, dtype=np.int32), (n,)).copy(),
                             device=cuda)
    K.ipe_fused_native(X, K.ipe_center_fragments(Ct, kp, dp), xn, cn, k, kp, dp, eps, Q,
                       RngKey(seed, "ipe", 0), RngKey(seed, "band_select", 0), 0, lab, mind,
                       prune=prune, C=Ct if hl is not None else None, hint_labels=hl,
                       stats=stats)
    torch.cuda.synchronize()
    ip = (Ct.double() @ X[0].double()).cpu().numpy()
    return lab.cpu().numpy(), mind.double().cpu().numpy(), float(xn[0]), cn.double().cpu().numpy(), ip


@pytest.mark.parametrize("Q,s1", [(3, 1.6), (1, 2.0)])
def test_ipe_pruned_two_centroid_exact_law(cuda, Q, s1):
    """Pair 0 is the exact-distance argmin (the hint, sampled in full); pair 1
    sits a few bins above it, so the pruned sampler's bound rejects most of
    its draws and its rare exact branch decides the rest.  The joint law of
    (label, min D~) is the exact law of min(V0, V1) of two independent
    median-of-Q AE estimates."""
    rng = np.random.default_rng(11)
    d, eps = 48, 0.02
    x = rng.standard_normal(d).astype(np.float32)
    u = rng.standard_normal(d)
    u -= (u @ x) / (x @ x) * x
    u /= np.linalg.norm(u)
    c0 = (x + 0.9 * u).astype(np.float32)
    c1 = (x - s1 * u).astype(np.float32)      # pair 1 ~ 5-9 bins above pair 0
    n = 1_000_000
    lab, mind, nx2, cn, ip = _run_rows(x, np.stack([c0, c1]), n, eps, Q, cuda, 0, True)
    M0, v0, p0 = _exact_law(ip[0], nx2, cn[0], eps, Q)
    M1, v1, p1 = _exact_law(ip[1], nx2, cn[1], eps, Q)
    # P(V1 < V0) and the joint cells (label, value)
    F1 = np.array([p1[v1 < v].sum() for v in v0])          # P(V1 < v)
    G0 = np.array([p0[v0 > v].sum() for v in v1])          # P(V0 > v)
    cells_e = np.concatenate([p0 * (1 - F1), p1 * G0])
    vals = np.concatenate([v0, v1])
    labs = np.concatenate([np.zeros_like(v0), np.ones_like(v1)])
    P1 = (p1 * G0).sum()
    assert 1e-4 < P1 < 0.2, P1        # the pruned pair does win sometimes
    obs = np.zeros(len(vals))
    for L in (0, 1):
        sel = lab == L
        cand = np.where(labs == L)[0]
        idx = cand[np.argmin(np.abs(mind[sel][:, None] - vals[cand][None, :]), axis=1)]
        assert np.allclose(mind[sel], vals[idx], rtol=2e-6, atol=1e-5)
        obs += np.bincount(idx, minlength=len(vals))
    n1 = int((lab == 1).sum())
    assert abs(n1 - n * P1) <= 5 * math.sqrt(n * P1 * (1 - P1)) + 1, (n1, n * P1)
    exp = cells_e * n
    big = exp >= 5
    o = np.append(obs[big], obs[~big].sum())
    e = np.append(exp[big], exp[~big].sum())
    chi2 = ((o - e) ** 2 / e).sum()
    assert stats.chi2.sf(chi2, len(e) - 1) > 1e-4


def test_ipe_pruned_matches_unpruned_law_many_centroids(cuda):
    """k = 40 centroids over 3 tiles (waves split them, the hint merge runs
    across lanes and waves): the (label, D~) law with pruning equals the
    full sampler's (two-sample chi^2, independent seeds)."""
    rng = np.random.default_rng(12)
    d, k, eps, Q = 40, 40, 0.1, 13
    x = rng.standard_normal(d).astype(np.float32)
    C = (x[None] + rng.uniform(0.7, 1.3, (k, 1)) * rng.standard_normal((k, d)) / math.sqrt(d) * 1.5)
    C = C.astype(np.float32)
    n = 400_000
    la, ma, *_ = _run_rows(x, C, n, eps, Q, cuda, 1, True)
    lb, mb, *_ = _run_rows(x, C, n, eps, Q, cuda, 2, False)
    ka = la.astype(np.int64) * 10**9 + np.round(ma * 1e3).astype(np.int64)
    kb = lb.astype(np.int64) * 10**9 + np.round(mb * 1e3).astype(np.int64)
    keys, inv = np.unique(np.concatenate([ka, kb]), return_inverse=True)
    ca = np.bincount(inv[:n], minlength=len(keys))
    cb = np.bincount(inv[n:], minlength=len(keys))
    keep = (ca + cb) >= 20
    table = np.stack([np.append(ca[keep], ca[~keep].sum()), np.append(cb[keep], cb[~keep].sum())])
    table = table[:, table.sum(0) > 0]
    assert table.shape[1] >= 3
    assert stats.chi2_contingency(table)[1] > 1e-4


# ------------------------------------------------- hazard-budget screening
def _fire_case(d=96, K_=64):
    """Q = 1, eps = 0.001: pair 0 near, 63 identical competitors (same |c|,
    same x.c) ~ 600+ bins above it: each competitor's hazard ~ 8e-4, so
    ~5 % of the rows fire at least once; ~0.1 % are won by a competitor."""
    rng = np.random.default_rng(21)
    x = rng.standard_normal(d)
    B = rng.standard_normal((d, K_))
    B -= np.outer(x, x @ B) / (x @ x)
    Qm, _ = np.linalg.qr(B)                      # K_ orthonormal directions, all orthogonal to x
    C = np.empty((K_, d))
    C[0] = x + 0.9 * Qm[:, 0]
    C[1:] = x[None] - 6.0 * Qm[:, 1:].T
    return x.astype(np.float32), C.astype(np.float32)


def _competitor_law(x, C, eps):
    """Exact joint law of (label == 0, min D~) for Q = 1: pair 0 against
    K - 1 iid competitors (pair 1's law)."""
    xd = x.astype(np.float64)
    Cd = C.astype(np.float64)
    nx2 = float(xd @ xd)
    Kc = C.shape[0] - 1

    def classes(ip, ny2):
        S = nx2 + ny2
        a = min(max((S - 2 * ip) / (2 * S), 0.0), 1.0)
        M = int(ae_bins(a, eps * max(1.0, abs(ip)) / S))
        om = M * math.asin(math.sqrt(a)) / math.pi
        p = fejer_pmf(om, M)
        p = p / p.sum()
        t = np.minimum(np.arange(M), M - np.arange(M))
        return 2 * S * np.sin(np.pi * np.arange(M // 2 + 1) / M) ** 2, np.bincount(t, weights=p)

    v0, p0 = classes(float(Cd[0] @ xd), float(Cd[0] @ Cd[0]))
    v1, p1 = classes(float(Cd[1] @ xd), float(Cd[1] @ Cd[1]))
    gt1 = lambda v: p1[v1 > v].sum()
    ge1 = lambda v: p1[v1 >= v].sum()
    gt0 = lambda v: p0[v0 > v].sum()
    cells0 = np.array([p0[i] * gt1(v) ** Kc for i, v in enumerate(v0)])
    cells1 = np.array([(ge1(w) ** Kc - gt1(w) ** Kc) * gt0(w) for w in v1])
    return v0, cells0, v1, cells1


@pytest.mark.parametrize("hint", [None, 0, 5])
def test_ipe_hazard_fire_path_exact_law(cuda, hint):
    """The hazard budgets fire on ~5 % of the rows (Q = 1: the Fejer bound
    is within a small factor of the true tail, so fired pairs really win
    sometimes): the joint (label is 0, min D~) law of 1M rows is the exact
    law, with the pass-1 hint, the right label hint and a wrong label hint
    (competitor 5 sampled first)."""
    eps = 0.001
    x, C = _fire_case()
    n = 1_000_000
    st = torch.zeros(5, dtype=torch.int64, device=cuda)
    lab, mind, *_ = _run_rows(x, C, n, eps, 1, cuda, 3, True, hint=hint, stats=st)
    scr, full, fires, exact, p1 = st.tolist()
    if hint == 5:
        # a far hint's estimate is a poor threshold: every pair is competitive
        # with it and takes the full sampler (same law, no pruning)
        assert full > 0.9 * n * C.shape[0], st.tolist()
    else:
        assert fires > 0.01 * n and exact > 0.001 * n, st.tolist()
    assert (p1 > 0) == (hint is None)
    v0, c0, v1, c1 = _competitor_law(x, C, eps)
    vals = np.concatenate([v0, v1])
    cells = np.concatenate([c0, c1])
    assert abs(cells.sum() - 1.0) < 1e-9
    obs = np.zeros(len(vals))
    for L, cand in ((True, np.arange(len(v0))), (False, len(v0) + np.arange(len(v1)))):
        sel = (lab == 0) if L else (lab != 0)
        idx = cand[np.argmin(np.abs(mind[sel][:, None] - vals[cand][None, :]), axis=1)]
        assert np.allclose(mind[sel], vals[idx], rtol=2e-6, atol=1e-5)
        obs += np.bincount(idx, minlength=len(vals))
    P_other = c1.sum()
    n1 = int((lab != 0).sum())
    assert abs(n1 - n * P_other) <= 5 * math.sqrt(n * P_other * (1 - P_other)) + 1, (n1, n * P_other)
    exp = cells * n
    big = exp >= 5
    o = np.append(obs[big], obs[~big].sum())
    e = np.append(exp[big], exp[~big].sum())
    chi2 = ((o - e) ** 2 / e).sum()
    assert stats.chi2.sf(chi2, len(e) - 1) > 1e-4


def test_ipe_hint_labels_match_unpruned_law(cuda):
    """Label hints (right, wrong, out of range -> first sweep) leave the
    (label, D~) law of the k = 40 case unchanged (two-sample chi^2 against the
    full sampler)."""
    rng = np.random.default_rng(12)
    d, k, eps, Q = 40, 40, 0.1, 13
    x = rng.standard_normal(d).astype(np.float32)
    C = (x[None] + rng.uniform(0.7, 1.3, (k, 1)) * rng.standard_normal((k, d)) / math.sqrt(d) * 1.5)
    C = C.astype(np.float32)
    n = 400_000
    lb, mb, *_ = _run_rows(x, C, n, eps, Q, cuda, 2, False)
    kb = lb.astype(np.int64) * 10**9 + np.round(mb * 1e3).astype(np.int64)
    for seed, hint in ((4, int(((C - x) ** 2).sum(1).argmin())), (5, 17), (6, 999)):
        la, ma, *_ = _run_rows(x, C, n, eps, Q, cuda, seed, True, hint=hint)
        ka = la.astype(np.int64) * 10**9 + np.round(ma * 1e3).astype(np.int64)
        keys, inv = np.unique(np.concatenate([ka, kb]), return_inverse=True)
        ca = np.bincount(inv[:n], minlength=len(keys))
        cb = np.bincount(inv[n:], minlength=len(keys))
        keep = (ca + cb) >= 20
        table = np.stack([np.append(ca[keep], ca[~keep].sum()), np.append(cb[keep], cb[~keep].sum())])
        table = table[:, table.sum(0) > 0]
        assert table.shape[1] >= 3
        assert stats.chi2_contingency(table)[1] > 1e-4, hint


@pytest.mark.parametrize("with_hint", [False, True])
def test_ipe_pruned_rows_invariant_to_grouping(cuda, with_hint):
    """Every pair's outcome depends on its row's threshold and its own
    stream only: the rows of a shard that starts at global row 7 (another
    workgroup grouping, another lane per row) get bit-identical labels and
    estimates - the property behind sharded fits equal to one rank's."""
    rng = np.random.default_rng(31)
    n, d, k, eps, Q = 6000, 64, 200, 0.25, 13
    ctr = rng.standard_normal((20, d)) * 3
    X = (ctr[rng.integers(0, 20, n)] + rng.standard_normal((n, d))).astype(np.float32)
    Cn = (ctr[rng.integers(0, 20, k)] + 0.5 * rng.standard_normal((k, d))).astype(np.float32)
    Xt = torch.tensor(X, device=cuda)
    Ct = torch.tensor(Cn, device=cuda)
    xn = (Xt * Xt).sum(1)
    cn = (Ct * Ct).sum(1)
    kp, dp = 208, 64
    frag = K.ipe_center_fragments(Ct, kp, dp)
    hint = torch.tensor(rng.integers(0, k, n).astype(np.int32), device=cuda) if with_hint else None
    outs = []
    for off in (0, 7):
        m = n - off
        lab = torch.empty(m, dtype=torch.int32, device=cuda)
        mind = torch.empty(m, dtype=torch.float32, device=cuda)
        K.ipe_fused_native(Xt[off:], frag, xn[off:].contiguous(), cn, k, kp, dp, eps, Q,
                           RngKey(9, "ipe", 1), RngKey(9, "band_select", 1), off, lab, mind,
                           C=Ct if with_hint else None,
                           hint_labels=hint[off:].contiguous() if with_hint else None)
        outs.append((lab.cpu().numpy(), mind.cpu().numpy()))
    torch.cuda.synchronize()
    assert np.array_equal(outs[0][0][7:], outs[1][0])
    assert np.array_equal(outs[0][1][7:], outs[1][1])


@pytest.mark.parametrize("dp,with_hint,prune", [(64, False, True), (64, True, True),
                                                (256, True, True), (512, False, True),
                                                (64, False, False)])
def test_ipe_layouts_bit_identical(cuda, dp, with_hint, prune):
    """The row-group kernel (1 or 2 groups of 16 rows per workgroup, wave-wide
    drain lists) and the per-lane-queue kernel share every stream, threshold
    and sampler: labels, estimates and the screen's counters are identical."""
    rng = np.random.default_rng(41 + dp)
    n, d, k, eps, Q = 5003, dp - 5, 200, 0.25, 13
    ctr = rng.standard_normal((20, d)) * 3
    X = (ctr[rng.integers(0, 20, n)] + rng.standard_normal((n, d))).astype(np.float32)
    Cn = (ctr[rng.integers(0, 20, k)] + 0.5 * rng.standard_normal((k, d))).astype(np.float32)
    Xt = torch.tensor(X, device=cuda)
    Ct = torch.tensor(Cn, device=cuda)
    xn = (Xt * Xt).sum(1)
    cn = (Ct * Ct).sum(1)
    kp = 208
    frag = K.ipe_center_fragments(Ct, kp, dp)
    hint = None
    if with_hint:   # mostly good hints, some invalid (-> the exact first sweep)
        hint = torch.tensor(np.where(rng.random(n) < 0.01, -1, rng.integers(0, k, n)).astype(np.int32),
                            device=cuda)
    outs = []
    for layout in (3, 1, 2):
        lab = torch.empty(n, dtype=torch.int32, device=cuda)
        mind = torch.empty(n, dtype=torch.float32, device=cuda)
        st = torch.zeros(5, dtype=torch.int64, device=cuda)
        K.ipe_fused_native(Xt, frag, xn, cn, k, kp, dp, eps, Q, RngKey(5, "ipe", 2),
                           RngKey(5, "band_select", 2), 11, lab, mind, prune=prune,
                           C=Ct if with_hint else None, hint_labels=hint, stats=st, layout=layout)
        outs.append((lab.cpu().numpy(), mind.cpu().numpy(), st.cpu().numpy()))
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert np.array_equal(outs[0][0], o[0])
        assert np.array_equal(outs[0][1], o[1])
        assert np.array_equal(outs[0][2][:4], o[2][:4])
    if prune:
        assert outs[0][2][0] > 0


# ------------------------------------------------ every shape the reference takes
@pytest.mark.parametrize("case", ["walk", "draws"])
def test_ipe_fused_law_exact_q17(cuda, case):
    """Q = 17 (median_evaluation at gamma = 0.05, Utility.py:564-568): the
    exact median-of-Q law on the order-statistic walk (M <= 128) and on the
    draw path (large M: the 16 smallest of the 17 draws kept)."""
    from sq_learn_amd.quantum.fejer import median_repetitions
    Q = median_repetitions(0.05)
    assert Q == 17
    rng = np.random.default_rng(17)
    d = 200
    x = rng.standard_normal(d)
    c = x + 0.8 * rng.standard_normal(d) if case == "walk" else rng.standard_normal(d)
    s, nx2, ny2, ip = _run_kernel(x, c, 60000, 0.25, Q, cuda, seed=4)
    M, vals, pm = _exact_law(ip, nx2, ny2, 0.25, Q)
    assert (M <= 128) == (case == "walk")
    assert _gof(s, vals, pm) > 1e-4


@pytest.mark.parametrize("Q", [13, 25])
def test_ipe_fused_law_exact_d1100(cuda, Q):
    """d = 1100 (d_pad 2048: 128 KiB of A fragments per workgroup): the same
    exact median law through the fused kernel."""
    rng = np.random.default_rng(1100)
    d = 1100
    x = rng.standard_normal(d)
    c = x + 0.8 * rng.standard_normal(d)
    s, nx2, ny2, ip = _run_kernel(x, c, 40000, 0.25, Q, cuda, seed=5)
    M, vals, pm = _exact_law(ip, nx2, ny2, 0.25, Q)
    assert M <= 128
    assert _gof(s, vals, pm) > 1e-4


def test_ipe_wide_q17_fit_runs_fused(cuda, monkeypatch):
    """A QMeans IPE fit at d = 1100, Q = 17 runs the fused kernel - the
    library-GEMM + sampler fallback is never called - and recovers the blobs."""
    from sq_learn_amd.models.cluster import QMeans
    from sq_learn_amd.utils.datasets import make_blobs
    from sklearn.metrics import adjusted_rand_score

    def boom(*a, **k):
        raise AssertionError("GEMM + sampler fallback used")
    monkeypatch.setattr(K, "ipe_estep_native", boom)
    X, y = make_blobs(3000, 1100, centers=5, cluster_std=1.0, random_state=1)
    g = QMeans(n_clusters=5, delta=0.5, true_distance_estimate=True, random_state=0, n_init=1,
               max_iter=8, init="k-means++", ipe_Q=17, device=cuda).fit(X)
    assert adjusted_rand_score(y, g.labels_) > 0.95
