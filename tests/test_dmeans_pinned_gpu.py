"""The GPU q-means engines pinned to the REFERENCE's own ``_dmeans.py``
functions.  The reference is not on the GPU box, so its outputs come from
tests/fixtures/dmeans_ref.npz, generated on the CPU by running the
AST-extracted reference functions (tests/fixtures/make_dmeans_ref.py,
``labels_estimation`` / ``select_labels`` / ``_centers_update``,
``_dmeans.py:732-830, 2252-2257``; ``ipe``, ``Utility.py:697-737``);
tests/test_dmeans_pinned_cpu.py re-derives the fixture from the reference
when it is present.

* the certified delta-means E-step (csrc/estep_f32.hip) picks labels in the
  reference's fp64 band with the law of ``select_labels`` and returns the
  reference's inertia (sum of minimum distances);
* the GPU M-step (segmented reduce + finalize) gives the reference's
  ``_centers_update`` means;
* the fused IPE E-step (csrc/ipe.hip) has the reference's per-row label law
  and estimated-inertia law."""
import os
import sys

import numpy as np
import pytest
import torch
from scipy import stats

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures"))
import make_dmeans_ref  # noqa: E402
from sq_learn_amd.models.cluster._lloyd import LloydEngine  # noqa: E402

pytestmark = pytest.mark.gpu
P_MIN = 1e-4
REPS = make_dmeans_ref.REPS


@pytest.fixture(scope="module")
def F():
    return make_dmeans_ref.load()


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


def test_certified_delta_estep_matches_reference(F):
    f, z = F
    X, C, delta = f["X1"], f["C1"], f["delta1"]
    n = X.shape[0]
    Xd, Cd = X.astype(np.float64), C.astype(np.float64)
    D = ((Xd[:, None, :] - Cd[None]) ** 2).sum(-1)
    band = D <= D.min(1, keepdims=True) + delta
    multi = band.sum(1) >= 2
    assert multi.sum() >= 40
    cr = z["cnt1"]
    assert (cr[~band] == 0).all()          # the reference's labels are band members
    co = np.zeros(D.shape)
    for s in range(REPS):
        lo, io, eng = _estep(X, C, delta, False, 100 + s)
        if s == 0:
            assert eng.fast and eng.certified      # the certified filter ran
        assert band[np.arange(n), lo].all()
        co[np.arange(n), lo] += 1
        # the inertia is the sum of minimum distances (fp32 per row on the
        # GPU, fp64 in the reference): the same every repetition
        assert io == pytest.approx(float(z["inert1"][s]), rel=2e-7)
    assert _contingency(cr[multi].ravel(), co[multi].ravel()) > P_MIN


def test_gpu_mstep_means_match_reference(F):
    f, z = F
    X, C, labels = f["X2"], f["C2"], f["L2"]
    k = C.shape[0]
    eng = LloydEngine(torch.from_numpy(X).cuda(), k, delta=0.0, seed=0)
    eng.set_centers(torch.from_numpy(C).cuda())
    lab = torch.from_numpy(labels.astype(np.int32)).cuda()
    eng.mstep(lab, torch.zeros(1, dtype=torch.float64, device="cuda"))
    # fp32 centroids of exact (fixed-point) sums: within fp32 rounding of the fp64 means
    np.testing.assert_allclose(eng.centers().double().cpu().numpy(), z["means2"], rtol=1e-6,
                               atol=1e-6)


def test_fused_ipe_estep_law_matches_reference(F):
    f, z = F
    X, C, delta = f["X3"], f["C3"], f["delta3"]
    cr, ir = z["cnt3"], z["inert3"]
    # the GPU kernel: REPS independent repetitions as REPS copies of the rows
    # in one launch (every row owns its own Philox streams)
    Xr = np.tile(X, (REPS, 1))
    lo, _, eng = _estep(Xr, C, delta, True, 7)
    co = np.zeros((4, 3))
    for r in range(4):
        co[r] = np.bincount(lo[r::4], minlength=3)
    eng2 = LloydEngine(torch.from_numpy(Xr).cuda(), 3, delta=delta, true_distance_estimate=True,
                       seed=8)
    _, mind, _ = eng2.estep(torch.from_numpy(C).cuda())
    io = mind.double().cpu().numpy().reshape(REPS, 4).sum(1)
    assert (cr > 0).sum() >= 6
    assert _contingency(cr.ravel(), co.ravel()) > P_MIN
    # the estimated inertia takes discrete values (sums of 2 S sin^2 classes),
    # evaluated in fp32 on the GPU and fp64 in the reference: compare the
    # laws of the values rounded to 6 significant digits
    rnd = lambda v: np.round(np.asarray(v, dtype=np.float64), 4)
    vals, inv = np.unique(np.concatenate([rnd(ir), rnd(io)]), return_inverse=True)
    ca = np.bincount(inv[:len(ir)], minlength=len(vals))
    cb = np.bincount(inv[len(ir):], minlength=len(vals))
    assert _contingency(ca.astype(float), cb.astype(float)) > P_MIN
