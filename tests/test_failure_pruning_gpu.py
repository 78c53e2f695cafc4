"""Failure injection on the pruned, incremental Lloyd step.

Corrupted rows get lb = 0 (re-evaluated by the next E-step) and their
min-vs-label correction moves with the label, so a failure-injected run is
bit-identical with the Hamerly bounds on and off, and the incremental
M-step gives the full M-step's centres and (to fp32 rounding of the
corrections) its inertia."""
import numpy as np
import pytest
import torch

from sq_learn_amd.models.cluster._lloyd import LloydEngine

pytestmark = pytest.mark.gpu


def _data(n=40000, d=64, k=48, seed=0):
    rs = np.random.RandomState(seed)
    G = rs.uniform(-4, 4, (k, d))
    X = (G[rs.randint(k, size=n)] + rs.randn(n, d)).astype(np.float32)
    C0 = X[rs.choice(n, k, replace=False)]
    return X, C0


def _run(monkeypatch, X, C0, bounds, incremental, p=0.05, attempts=1, iters=8):
    monkeypatch.setenv("SQ_ESTEP_BOUNDS", "1" if bounds else "0")
    monkeypatch.setenv("SQ_MSTEP_INCREMENTAL", "1" if incremental else "0")
    Xt = torch.from_numpy(X).cuda()
    eng = LloydEngine(Xt, C0.shape[0], delta=0.5, intermediate_error=True, true_tomography=False,
                      failure_prob=p, failure_attempts=attempts, seed=3)
    assert eng.fast and eng.certified
    assert eng.bounds == bounds and eng.incremental == incremental
    eng.set_centers(torch.from_numpy(C0).cuda())
    out = []
    for _ in range(iters):
        labels, sc = eng.step()
        out.append((labels.clone().cpu(), eng.centers().clone().cpu(), sc.tolist()))
    return out, eng.failure_counters.tolist()


@pytest.mark.parametrize("attempts", [1, 2])
def test_failure_injection_bounds_on_off_bit_identical(monkeypatch, attempts):
    X, C0 = _data()
    a, ca = _run(monkeypatch, X, C0, True, True, attempts=attempts)
    b, cb = _run(monkeypatch, X, C0, False, True, attempts=attempts)
    assert ca == cb and ca[1] > 0
    for (la, Ca, sa), (lb, Cb, sb) in zip(a, b):
        assert torch.equal(la, lb)
        assert torch.equal(Ca, Cb)
        assert sa[0] == sb[0] and sa[1] == sb[1]


def test_failure_injection_incremental_matches_full_mstep(monkeypatch):
    X, C0 = _data(seed=1)
    a, _ = _run(monkeypatch, X, C0, True, True)
    b, _ = _run(monkeypatch, X, C0, True, False)
    for (la, Ca, sa), (lb, Cb, sb) in zip(a, b):
        assert torch.equal(la, lb)
        assert torch.equal(Ca, Cb)
        assert sa[0] == pytest.approx(sb[0], rel=2e-6)


def test_adaptive_filter_skips_and_stays_exact(monkeypatch):
    """Adaptive pruning: with keep_max = 0 every measured filter pass
    'kept too much', so the engine sweeps all rows directly (bounds still
    maintained) and re-probes every 4th E-step; labels and centres equal
    the always-filtered run's bit for bit, and the kept count travels in
    the iteration's scalars."""
    X, C0 = _data(seed=2)

    def run(keep_max):
        monkeypatch.setenv("SQ_ESTEP_BOUNDS", "1")
        monkeypatch.setenv("SQ_ESTEP_KEEP_MAX", str(keep_max))
        eng = LloydEngine(torch.from_numpy(X).cuda(), C0.shape[0], delta=0.5,
                          intermediate_error=True, seed=4)
        eng.set_centers(torch.from_numpy(C0).cuda())
        eng.pipeline = True
        out, ran = [], []
        for _ in range(10):
            labels, sc = eng.step()
            vals = sc.tolist()
            out.append((labels.clone().cpu(), eng.centers().clone().cpu(), vals[:2]))
            ran.append(vals[3] >= 0)
        eng.pipeline = False
        eng.drop_pending()
        return out, ran

    a, ran_a = run(1.0)
    b, ran_b = run(0.0)
    assert sum(ran_a) >= 8                 # every E-step after the first filtered
    assert 0 < sum(ran_b) < sum(ran_a)      # skipped, with periodic probes
    for (la, Ca, sa), (lb, Cb, sb) in zip(a, b):
        assert torch.equal(la, lb) and torch.equal(Ca, Cb) and sa == sb
