"""Row skip of the certified fp16 IPE screen (csrc/ipe16.hip prep): a row
whose Hamerly-style bounds put every non-hint centroid inside its far band
is finished by prep (its fired pairs only) instead of the fp16 sweep.

* bit-identity: labels and estimates equal the no-skip path's (a skipped
  row's only listed pairs would be its fires; the same streams and the same
  arithmetic finish them), over a Lloyd trajectory and for a second E-step
  at fixed centres;
* law: a case whose rows straddle the skip condition (the bound at the band
  edge: the row's threshold, re-sampled every step, decides) keeps the
  full sampler's (label, D~) law (reference: ``_dmeans.py:753-772`` ->
  ``Utility.py:697-737``)."""
import numpy as np
import pytest
import torch

from sq_learn_amd.ops import kmeans as K
from sq_learn_amd.runtime.rng import RngKey

from test_ipe16_gpu import _fire_case, _keys, _run_full, _same_law

pytestmark = pytest.mark.gpu


def _two_steps(X, C, eps, Q, seed, skip, hint0=None, ht=None, stats=None):
    """Two E-steps at fixed centres through one Ipe16 (the second with the
    first's labels as hints and, with ``skip``, the first's bounds)."""
    n, d = X.shape
    k = C.shape[0]
    xn = (X.double() ** 2).sum(1).float().contiguous()
    cn = (C * C).sum(1).contiguous()
    st = K.Ipe16(X, k, K.pad_features(d), K.pad_clusters(k), K.choose_alpha(float(xn.max()), 0.0),
                 X.device)
    st.skip = skip
    if ht is not None:
        st.ht = ht
    st.set_centers(C)
    okey = _keys(seed)[4]
    out = []
    hint = (torch.full((n,), -1, dtype=torch.int32, device=X.device) if hint0 is None
            else hint0.clone())
    for s in range(2):
        lab = torch.empty(n, dtype=torch.int32, device=X.device)
        mind = torch.empty(n, dtype=torch.float32, device=X.device)
        # the step index moves the keys, as the engine's per-iteration keys do
        ks = [RngKey(seed + 7 * s, nm, 0) for nm in ("ipe", "band_select", "ipe16_skip",
                                                      "ipe16_row")]

        def fallback(rl, rc, ln, thr, hj, s0, e0):
            dp = 32
            while dp < d:
                dp *= 2
            kp = -(-k // 16) * 16
            K.ipe_fused_native(X[s0:e0], K.ipe_center_fragments(C, kp, dp), xn[s0:e0], cn, k, kp,
                               dp, eps, Q, ks[0], ks[1], s0, lab[s0:e0], mind[s0:e0], C=C,
                               skip_key=okey, rows=(rl, rc, ln), ext=(thr, hj))

        if stats is not None:
            stats[s].zero_()
        st.estep(X, C, hint, xn, cn, lab, mind, eps, Q, ks[0], ks[1], ks[2], ks[3], 0,
                 s == 0 and hint0 is None, stats=None if stats is None else stats[s],
                 fallback=fallback)
        torch.cuda.synchronize()
        out.append((lab.cpu().numpy(), mind.double().cpu().numpy()))
        hint = lab.clone()
    return out, st


def _blobs(seed, n=60000, d=64, k=200, nb=40):
    rng = np.random.default_rng(seed)
    ctr = rng.standard_normal((nb, d)) * 4
    X = (ctr[rng.integers(0, nb, n)] + rng.standard_normal((n, d))).astype(np.float32)
    C = (ctr[np.arange(k) % nb] + 0.3 * rng.standard_normal((k, d))).astype(np.float32)
    return X, C


def test_ipe16_skip_second_step_bit_identical(cuda):
    """Blob data, two E-steps at fixed centres: with the row skip the second
    step skips most rows, and its labels / estimates equal the no-skip
    path's bit for bit."""
    X, C = _blobs(3, k=40)
    Xt, Ct = torch.tensor(X, device=cuda), torch.tensor(C, device=cuda)
    st1 = torch.zeros((2, 8), dtype=torch.int64, device=cuda)
    on, eng = _two_steps(Xt, Ct, 0.25, 13, 5, True, stats=st1)
    off, _ = _two_steps(Xt, Ct, 0.25, 13, 5, False)
    s = st1.tolist()
    assert s[0][7] == 0 and s[1][7] > 0.3 * X.shape[0], s
    for (la, ma), (lb, mb) in zip(on, off):
        assert np.array_equal(la, lb) and np.array_equal(ma, mb)


def test_ipe16_skip_lloyd_trajectory_bit_identical(cuda, monkeypatch):
    """A q-means Lloyd trajectory (centres move, labels re-drawn every step,
    some rows' labels leave their hint): identical inertia, labels and
    centres with the row skip on and off; the skip engages."""
    from sq_learn_amd.models.cluster._lloyd import LloydEngine
    from sq_learn_amd.models._data import Data, gather_rows
    from sq_learn_amd.parallel.comm import Comm
    from sq_learn_amd.utils.datasets import make_blobs_device
    n, d, k = 200_000, 64, 128
    X, _ = make_blobs_device(n, d, centers=k, cluster_std=1.0, seed=4, device=cuda,
                             dtype=torch.float32)
    C0 = gather_rows(Data(X, n, 0, Comm(None), "sharded"),
                     np.random.RandomState(4).choice(n, k, replace=False))
    res = {}
    for skip in ("1", "0"):
        monkeypatch.setenv("SQ_IPE16_SKIP", skip)
        eng = LloydEngine(X, k, delta=0.5, true_distance_estimate=True, intermediate_error=True,
                          seed=3)
        eng.set_centers(C0)
        eng.ipe16_stats = torch.zeros(8, dtype=torch.int64, device=cuda)
        tr = []
        for _ in range(6):
            eng.ipe16_stats.zero_()
            lab, sc = eng.step()
            tr.append((sc.tolist()[0], lab.cpu().numpy().copy(), eng.centers().cpu().numpy().copy(),
                       int(eng.ipe16_stats[7])))
        res[skip] = tr
    for a, b in zip(res["1"], res["0"]):
        assert a[0] == b[0]
        assert np.array_equal(a[1], b[1])
        assert np.array_equal(a[2], b[2])
    skipped = [t[3] for t in res["1"]]
    assert skipped[0] == 0 and max(skipped[2:]) > 0.05 * n, skipped


def test_ipe16_skip_law_at_band_edge(cuda):
    """300 competitors on orthogonal directions at a distance where the skip
    condition holds for some rows and not for others (each row's threshold,
    re-sampled every step, moves its band): the second step's (label, D~)
    law equals the full sampler's, and both paths are exercised."""
    x, C = _fire_case(s=9.0)
    n = 400_000
    X = torch.tensor(np.tile(x, (n, 1)), device=cuda)
    Ct = torch.tensor(C, device=cuda)
    hint = torch.zeros(n, dtype=torch.int32, device=cuda)
    st = torch.zeros((2, 8), dtype=torch.int64, device=cuda)
    out, _ = _two_steps(X, Ct, 0.25, 13, 8, True, hint0=hint, ht=9e-4, stats=st)
    s = st.tolist()
    assert 0.05 * n < s[1][7] < 0.95 * n, s   # skipped and swept rows
    la, ma = out[1]
    lb, mb = _run_full(X, Ct, 0.25, 13, 9)
    assert _same_law(la, ma, lb, mb, min_cells=2) > 1e-4


@pytest.mark.parametrize("k", [40, 200, 1000, 3000])
def test_ipe16_native_skip_bounds_match_torch(cuda, k):
    """csrc/ipe16.hip op 5 (the skip bounds in three launches) against the
    torch formulation of ``Ipe16._skip_bounds``: the same wild count, tau,
    wild minimum and per-group upper distances (fp32, up to the fp64
    rounding order)."""
    d = 64
    g = torch.Generator().manual_seed(k)
    C0 = (torch.randn(k, d, generator=g) * 3).to(cuda)
    C1 = C0 + 1e-3 * torch.randn(k, d, generator=g).to(cuda)
    jump = torch.randperm(k, generator=g)[:max(k // 20, 1)].to(cuda)
    C1[jump] += 2.0 * torch.randn(len(jump), d, generator=g).to(cuda)
    X = torch.randn(256, d, device=cuda)
    outs = []
    for native in (True, False):
        st = K.Ipe16(X, k, K.pad_features(d), K.pad_clusters(k), 1.0, cuda)
        st.native_bounds = native
        for C in (C0, C1):
            st.set_centers(C)
            st._skip_bounds(C)
            if C is C0:
                first = (st.mw[:k].clone(), st.Rc[:k].clone())
        torch.cuda.synchronize()
        outs.append((first, int(st.last_wild), st.smax.clone(), st.mw[:k].clone(),
                     st.Rc[:k].clone()))
    (fa, wa, sa, ma, ra), (fb, wb, sb, mb, rb) = outs
    assert torch.isinf(fa[0]).all() and torch.isinf(fb[0]).all()
    torch.testing.assert_close(fa[1], fb[1], rtol=1e-6, atol=0)
    assert wa == wb and wa >= min(16, k // 2)
    torch.testing.assert_close(sa, sb, rtol=1e-6, atol=0)
    torch.testing.assert_close(ma, mb, rtol=1e-6, atol=0)
    torch.testing.assert_close(ra, rb, rtol=1e-6, atol=0)
