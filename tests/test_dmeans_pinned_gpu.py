"""The GPU q-means engines pinned to the REFERENCE's own ``_dmeans.py``
functions (AST-extracted, tests/_dmeans_ref.py; CPU twin of this file:
tests/test_dmeans_pinned_cpu.py):

* the certified delta-means E-step (csrc/estep_f32.hip) picks labels in the
  reference's fp64 band with the law of ``select_labels`` and returns the
  reference's inertia (sum of minimum distances);
* the GPU M-step (segmented reduce + finalize) gives the reference's
  ``_centers_update`` means;
* the fused IPE E-step (csrc/ipe.hip) has the reference's per-row label law
  and estimated-inertia law."""
import random

import numpy as np
import pytest
import torch
from scipy import stats

import _dmeans_ref
from sq_learn_amd.models.cluster._lloyd import LloydEngine

pytestmark = pytest.mark.gpu
P_MIN = 1e-4


@pytest.fixture(scope="module")
def R():
    if not _dmeans_ref.available():
        pytest.skip("reference _dmeans.py / Utility.py not present")
    try:
        import matplotlib  # noqa: F401
        import sklearn  # noqa: F401
    except ImportError:
        pytest.skip("matplotlib / scikit-learn missing")
    ns, _ = _dmeans_ref.load()
    return ns


def _seed(s):
    random.seed(s)
    np.random.seed(s)


def _contingency(ca, cb):
    tot = ca + cb
    keep = tot >= 10
    table = np.stack([np.append(ca[keep], ca[~keep].sum()), np.append(cb[keep], cb[~keep].sum())])
    table = table[:, table.sum(0) > 0]
    if table.shape[1] < 2:
        return 1.0
    return stats.chi2_contingency(table)[1]


def _estep(X, C, delta, ipe, seed):
    eng = LloydEngine(torch.from_numpy(X).cuda(), C.shape[0], delta=delta,
                      true_distance_estimate=ipe, seed=seed)
    lab, mind, inertia = eng.estep(torch.from_numpy(C).cuda())
    return lab.long().cpu().numpy(), float(inertia.sum()), eng


def test_certified_delta_estep_matches_reference(R):
    rng = np.random.default_rng(1)
    k, d, n = 6, 32, 200
    C = (rng.standard_normal(d)[None] + 0.3 * rng.standard_normal((k, d))).astype(np.float32)
    X = (C[rng.integers(0, k, n)] + 0.9 * rng.standard_normal((n, d))).astype(np.float32)
    Xd, Cd = X.astype(np.float64), C.astype(np.float64)
    D = ((Xd[:, None, :] - Cd[None]) ** 2).sum(-1)
    delta = 8.0
    band = D <= D.min(1, keepdims=True) + delta
    multi = band.sum(1) >= 2
    assert multi.sum() >= 40
    reps = 300
    cr = np.zeros(D.shape)
    co = np.zeros(D.shape)
    for s in range(reps):
        _seed(s)
        lab, _, inert = R["labels_estimation"](Xd, Cd, delta, None, False)
        lab = np.asarray(lab, dtype=np.int64)
        cr[np.arange(n), lab] += 1
        lo, io, eng = _estep(X, C, delta, False, 100 + s)
        if s == 0:
            assert eng.fast and eng.certified      # the certified filter ran
        assert band[np.arange(n), lo].all()
        co[np.arange(n), lo] += 1
        assert io == pytest.approx(float(inert), rel=1e-9)
    assert _contingency(cr[multi].ravel(), co[multi].ravel()) > P_MIN


def test_gpu_mstep_means_match_reference(R):
    rng = np.random.default_rng(2)
    k, d, n = 5, 64, 4000
    X = rng.standard_normal((n, d)).astype(np.float32)
    C = rng.standard_normal((k, d)).astype(np.float32)
    labels = rng.integers(0, k, n)
    labels[:k] = np.arange(k)
    ref = R["_centers_update"](X.astype(np.float64), labels, 0.0, False, False, True)
    eng = LloydEngine(torch.from_numpy(X).cuda(), k, delta=0.0, seed=0)
    eng.set_centers(torch.from_numpy(C).cuda())
    lab = torch.from_numpy(labels.astype(np.int32)).cuda()
    eng.mstep(lab, torch.zeros(1, dtype=torch.float64, device="cuda"))
    # fp32 centroids of exact (fixed-point) sums: within fp32 rounding of the fp64 means
    np.testing.assert_allclose(eng.centers().double().cpu().numpy(), ref, rtol=1e-6, atol=1e-6)


def test_fused_ipe_estep_law_matches_reference(R):
    C = np.array([[2.0, 0.0, 0.0, 0.5], [-2.0, 0.0, 0.0, 0.5], [0.0, 2.5, 0.0, -0.5]],
                 dtype=np.float32)
    X = np.array([[0.0, 0.2, 0.1, 0.4], [0.0, -0.3, 0.7, 0.1], [0.04, 0.4, -0.3, 0.2],
                  [-0.15, 0.1, 0.2, -0.1]], dtype=np.float32)
    delta = 0.5
    reps = 300
    cr = np.zeros((4, 3))
    ir = []
    for s in range(reps):
        _seed(s)
        lab, _, inert = R["labels_estimation"](X.astype(np.float64), C.astype(np.float64), delta,
                                               None, True)
        cr[np.arange(4), np.asarray(lab, dtype=np.int64)] += 1
        ir.append(float(inert))
    # the GPU kernel: 300 independent repetitions as 300 copies of the rows
    # in one launch (every row owns its own Philox streams)
    Xr = np.tile(X, (reps, 1))
    lo, _, eng = _estep(Xr, C, delta, True, 7)
    co = np.zeros((4, 3))
    for r in range(4):
        co[r] = np.bincount(lo[r::4], minlength=3)
    eng2 = LloydEngine(torch.from_numpy(Xr).cuda(), 3, delta=delta, true_distance_estimate=True,
                       seed=8)
    _, mind, _ = eng2.estep(torch.from_numpy(C).cuda())
    io = mind.double().cpu().numpy().reshape(reps, 4).sum(1)
    assert (cr > 0).sum() >= 6
    assert _contingency(cr.ravel(), co.ravel()) > P_MIN
    assert stats.ks_2samp(ir, io).pvalue > P_MIN
