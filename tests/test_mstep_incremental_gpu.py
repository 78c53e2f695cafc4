"""Incremental M-step (csrc/kmeans.hip delta_segment_kernel): only moved rows
are re-read, the fixed-point statistics are updated exactly - centroids must
be BIT-identical to the full segmented reduce, the inertia (per-cluster
formula + E-step corrections) equal to the sum of exact min distances."""
import os

import numpy as np
import pytest
import torch

from sq_learn_amd.models.cluster._lloyd import LloydEngine
from sq_learn_amd.utils.datasets import make_blobs

pytestmark = pytest.mark.gpu


def _engine(X, k, delta, incremental):
    old = os.environ.get("SQ_MSTEP_INCREMENTAL")
    os.environ["SQ_MSTEP_INCREMENTAL"] = "1" if incremental else "0"
    try:
        return LloydEngine(X, k, delta=delta, intermediate_error=delta > 0, seed=3,
                           gemm_precision="fp32")
    finally:
        if old is None:
            del os.environ["SQ_MSTEP_INCREMENTAL"]
        else:
            os.environ["SQ_MSTEP_INCREMENTAL"] = old


@pytest.mark.parametrize("delta,d", [(0.0, 64), (0.5, 256), (3.0, 100), (0.5, 512), (0.5, 784)])
def test_incremental_mstep_bit_identical(cuda, delta, d):
    X, _ = make_blobs(60000 if d <= 256 else 20000, d, centers=40, cluster_std=1.5, random_state=0)
    Xt = torch.tensor(X, dtype=torch.float32, device=cuda)
    k = 48
    C0 = Xt[torch.as_tensor(np.random.RandomState(1).choice(Xt.shape[0], k, replace=False), device=cuda)]
    inc = _engine(Xt, k, delta, True)
    ful = _engine(Xt, k, delta, False)
    assert inc.incremental and not ful.incremental
    inc.set_centers(C0)
    ful.set_centers(C0)
    for it in range(8):
        la, sa = inc.step()
        lb, sb = ful.step()
        assert torch.equal(la, lb)
        assert torch.equal(inc.C, ful.C), f"centroids differ at iteration {it}"
        a, b = sa.tolist(), sb.tolist()
        assert abs(a[0] - b[0]) <= 1e-9 * abs(b[0]) + 1e-6, (it, a[0], b[0])
        assert a[1] == pytest.approx(b[1], rel=1e-12, abs=1e-12)
    # a restart (set_centers) resets the statistics
    inc.set_centers(C0)
    ful.set_centers(C0)
    la, sa = inc.step()
    lb, sb = ful.step()
    assert torch.equal(inc.C, ful.C)


def _engine_b(X, k, delta, bounds, tomo=False):
    old = os.environ.get("SQ_ESTEP_BOUNDS")
    os.environ["SQ_ESTEP_BOUNDS"] = "1" if bounds else "0"
    try:
        return LloydEngine(X, k, delta=delta, intermediate_error=delta > 0, true_tomography=tomo,
                           seed=5, gemm_precision="fp32")
    finally:
        if old is None:
            del os.environ["SQ_ESTEP_BOUNDS"]
        else:
            os.environ["SQ_ESTEP_BOUNDS"] = old


@pytest.mark.parametrize("delta,tomo", [(0.0, False), (0.5, False), (2.0, True)])
def test_hamerly_pruning_is_exact(cuda, delta, tomo):
    """Pruned rows provably keep a one-member band: labels, centroids and
    inertia BIT-identical to the unpruned certified E-step, and most rows
    are pruned once the centroids settle."""
    X, _ = make_blobs(80000, 64, centers=30, cluster_std=1.0, random_state=2)
    Xt = torch.tensor(X, dtype=torch.float32, device=cuda)
    k = 32
    C0 = Xt[torch.as_tensor(np.random.RandomState(3).choice(80000, k, replace=False), device=cuda)]
    a = _engine_b(Xt, k, delta, True, tomo)
    b = _engine_b(Xt, k, delta, False, tomo)
    assert a.bounds and not b.bounds
    a.set_centers(C0)
    b.set_centers(C0)
    active = []
    for it in range(10):
        la, sa = a.step()
        lb, sb = b.step()
        assert torch.equal(la, lb), f"labels differ at iteration {it}"
        assert torch.equal(a.C, b.C)
        assert sa.tolist()[0] == sb.tolist()[0]
        if it > 0:
            active.append(int(a.rcount.item()))
    if not tomo:   # (shot tomography moves every centroid far each step)
        assert min(active) < 0.5 * 80000, active


def test_adaptive_filter_modes_are_exact(cuda):
    """The adaptive Hamerly policy's every mode - filter, dormant bounds
    ('none'), bound-maintaining sweeps ('bounds') and measure-only probes -
    gives labels and centroids BIT-identical to the bounds-off engine
    (keep_max = 0 treats every measured kept fraction as too high, so the
    skip / probe cycle runs from the third step on)."""
    X, _ = make_blobs(60000, 64, centers=30, cluster_std=1.0, random_state=4)
    Xt = torch.tensor(X, dtype=torch.float32, device=cuda)
    k = 32
    C0 = Xt[torch.as_tensor(np.random.RandomState(5).choice(60000, k, replace=False), device=cuda)]
    a = _engine_b(Xt, k, 0.5, True)
    b = _engine_b(Xt, k, 0.5, False)
    a.keep_max = 0.0
    a.set_centers(C0)
    b.set_centers(C0)
    modes = []
    orig = a._filter_mode

    def spy():
        m = orig()
        modes.append("probe" if (m == "filter" and a._probing) else m)
        return m

    a._filter_mode = spy
    for it in range(14):
        la, sa = a.step()
        lb, sb = b.step()
        assert torch.equal(la, lb), f"labels differ at iteration {it} ({modes[-1:]})"
        assert torch.equal(a.C, b.C), f"centroids differ at iteration {it}"
        assert sa.tolist()[0] == sb.tolist()[0]
    assert {"none", "bounds", "probe"} <= set(modes), modes


@pytest.mark.parametrize("d", [64, 100])
def test_ipe_incremental_mstep_bit_identical(cuda, monkeypatch, d):
    """The IPE E-step's Lloyd loop (generic M-step): the incremental
    statistics (moved rows only) give bit-identical centroids and scalars to
    the full fixed-point reduce."""
    X, _ = make_blobs(40000, d, centers=30, cluster_std=1.5, random_state=2)
    Xt = torch.tensor(X, dtype=torch.float32, device=cuda)
    k = 32
    C0 = Xt[torch.as_tensor(np.random.RandomState(3).choice(Xt.shape[0], k, replace=False),
                            device=cuda)]
    out = {}
    for inc in ("1", "0"):
        monkeypatch.setenv("SQ_MSTEP_INCREMENTAL", inc)
        eng = LloydEngine(Xt, k, delta=0.5, true_distance_estimate=True, intermediate_error=True,
                          seed=5)
        eng.set_centers(C0)
        tr = []
        for _ in range(5):
            lab, sc = eng.step()
            tr.append((sc.tolist(), eng.centers().cpu().numpy().copy()))
        assert eng._g_inc == (inc == "1")
        out[inc] = tr
    for (sa, ca), (sb, cb) in zip(out["1"], out["0"]):
        assert sa == sb
        assert np.array_equal(ca, cb)
