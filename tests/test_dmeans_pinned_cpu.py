"""q-means estimator semantics pinned to the REFERENCE's own ``_dmeans.py``.

``labels_estimation`` (E-step: delta-band uniform pick via ``select_labels``,
or IPE-estimated distances with a random argmin), ``_centers_update``
(M-step means + tomography error) are AST-extracted from
``/root/reference/sklearn/cluster/_dmeans.py`` (tests/_dmeans_ref.py) and
run side by side with the framework's Lloyd engine (CPU here;
tests/test_dmeans_pinned_gpu.py runs the GPU engines):

* delta-means: every label the engine picks lies in the reference's band
  {j : D_ij <= min_i + delta}, the per-row label law equals the reference's
  uniform ``random.choice`` (two-sample chi^2), and the inertia is the same
  sum of minimum distances;
* M-step: identical cluster means; the Gaussian tomography perturbation has
  the reference's law (two-sample Kolmogorov-Smirnov);
* IPE (``true_distance_estimate=True``): the per-row label law and the law
  of the estimated inertia equal the reference's (median-of-13 amplitude
  estimation per pair through ``Utility.ipe``).

The reference draws from python's ``random`` / ``np.random`` (seeded per
repetition); the engine from its Philox keys (seeded per repetition).
Thresholds p > 1e-4."""
import random

import numpy as np
import pytest
import torch
from scipy import stats

import _dmeans_ref
from sq_learn_amd.models.cluster._lloyd import LloydEngine

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
    ns, U = _dmeans_ref.load()
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


def _problem(seed, n, d, k, spread):
    rng = np.random.default_rng(seed)
    C = rng.standard_normal((k, d))
    X = C[rng.integers(0, k, n)] + spread * rng.standard_normal((n, d))
    return X, C


def _engine_estep(X, C, delta, ipe, seed):
    eng = LloydEngine(torch.from_numpy(X), C.shape[0], delta=delta, true_distance_estimate=ipe,
                      seed=seed)
    lab, mind, inertia = eng.estep(torch.from_numpy(C))
    return lab.numpy().astype(np.int64), mind.numpy(), float(inertia.sum())


def test_delta_band_labels_follow_select_labels(R):
    X, C = _problem(1, 60, 4, 5, 0.9)
    delta = 1.5
    D = ((X[:, None, :] - C[None]) ** 2).sum(-1)
    band = D <= D.min(1, keepdims=True) + delta
    assert (band.sum(1) >= 2).sum() >= 20          # plenty of multi-member bands
    reps = 400
    cr = np.zeros(D.shape)
    co = np.zeros(D.shape)
    for s in range(reps):
        _seed(s)
        lab, _, inert = R["labels_estimation"](X, C, delta, None, False)
        lab = np.asarray(lab, dtype=np.int64)
        assert band[np.arange(len(lab)), lab].all()
        cr[np.arange(len(lab)), lab] += 1
        lo, _, io = _engine_estep(X, C, delta, False, seed=1000 + s)
        assert band[np.arange(len(lo)), lo].all()
        co[np.arange(len(lo)), lo] += 1
        # the reference's inertia: sum of the minimum distances
        assert io == pytest.approx(float(inert), rel=1e-12)
    multi = band.sum(1) >= 2
    assert _contingency(cr[multi].ravel(), co[multi].ravel()) > P_MIN
    # both uniform over the band
    for cnt in (cr, co):
        for i in np.nonzero(multi)[0]:
            obs = cnt[i, band[i]]
            assert stats.chisquare(obs).pvalue > P_MIN / len(band)


def test_centers_update_means_and_tomography_law(R):
    X, C = _problem(2, 300, 6, 4, 0.7)
    rng = np.random.default_rng(3)
    labels = rng.integers(0, 4, 300)
    labels[:4] = np.arange(4)                     # every cluster non-empty
    ref = R["_centers_update"](X, labels, 0.0, False, False, True)
    eng = LloydEngine(torch.from_numpy(X), 4, delta=0.0, seed=0)
    eng.set_centers(torch.from_numpy(C))
    eng.mstep(torch.from_numpy(labels), torch.zeros(1, dtype=torch.float64))
    np.testing.assert_allclose(eng.centers().numpy(), ref, rtol=1e-12, atol=1e-13)
    # intermediate_error=True, Gaussian tomography with error delta/2
    delta = 0.8
    nr, ne = [], []
    for s in range(150):
        _seed(s)
        noisy = R["_centers_update"](X, labels, delta / 2, True, False, True)
        nr.append((noisy - ref).ravel())
        eng = LloydEngine(torch.from_numpy(X), 4, delta=delta, intermediate_error=True,
                          true_tomography=False, seed=500 + s)
        eng.set_centers(torch.from_numpy(C))
        eng.mstep(torch.from_numpy(labels), torch.zeros(1, dtype=torch.float64))
        ne.append((eng.centers().numpy() - ref).ravel())
    nr, ne = np.concatenate(nr), np.concatenate(ne)
    bound = delta / 2 / np.sqrt(4 * 6)
    assert np.abs(nr).max() <= bound + 1e-12 and np.abs(ne).max() <= bound + 1e-12
    assert stats.ks_2samp(nr, ne).pvalue > P_MIN


def test_ipe_labels_and_inertia_law_match_reference(R):
    """``true_distance_estimate=True``: distances |x|^2 + |c|^2 - 2 ipe(x, c,
    delta / 2) with the median of 13 AE draws per pair; label = random
    argmin.  Rows sit on (or near) the mirror plane of two centres, so the
    two estimated distances tie or nearly tie and both labels occur."""
    C = np.array([[2.0, 0.0, 0.0, 0.5], [-2.0, 0.0, 0.0, 0.5], [0.0, 2.5, 0.0, -0.5]])
    X = np.array([[0.0, 0.2, 0.1, 0.4], [0.0, -0.3, 0.7, 0.1], [0.04, 0.4, -0.3, 0.2],
                  [-0.15, 0.1, 0.2, -0.1]])
    delta = 0.5
    reps = 300
    cr = np.zeros((4, 3))
    co = np.zeros((4, 3))
    ir, io = [], []
    for s in range(reps):
        _seed(s)
        lab, _, inert = R["labels_estimation"](X, C, delta, None, True)
        lab = np.asarray(lab, dtype=np.int64)
        cr[np.arange(4), lab] += 1
        ir.append(float(inert))
        lo, _, i_o = _engine_estep(X, C, delta, True, seed=2000 + s)
        co[np.arange(4), lo] += 1
        io.append(i_o)
    assert (cr > 0).sum() >= 6                     # the labels really vary
    assert _contingency(cr.ravel(), co.ravel()) > P_MIN
    assert stats.ks_2samp(ir, io).pvalue > P_MIN


def test_gpu_fixture_is_the_references_output(R):
    """tests/fixtures/dmeans_ref.npz (what the GPU-box pinned tests compare
    against) is exactly what the reference functions produce."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures"))
    import make_dmeans_ref
    f, z = make_dmeans_ref.load()
    got = make_dmeans_ref.generate(R)
    for key in ("cnt1", "inert1", "means2", "cnt3", "inert3"):
        np.testing.assert_array_equal(got[key], z[key], err_msg=key)
