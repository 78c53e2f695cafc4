"""Gap records of the multi-candidate rows (csrc/estep_f32.hip
recheck_fast_kernel writes them, bounds_filter_kernel lists rows with a
current record, gap_screen_kernel moves the gaps by the fp16 shift operand
and resolves rows whose band stays certainly {argmin} from the fp16 row).
The records only change which kernel certifies a row: labels, centres and the
iteration scalars are bit-identical with them on and off, across a centre
reset (records before it are void), with failure injection and pipelined
E-steps."""
import numpy as np
import pytest
import torch

from sq_learn_amd.models.cluster._lloyd import LloydEngine

pytestmark = pytest.mark.gpu


def _data(n=60000, d=128, k=64, seed=0, spread=3.0):
    rs = np.random.RandomState(seed)
    G = rs.uniform(-spread, spread, (k, d))
    X = (G[rs.randint(k, size=n)] + rs.randn(n, d)).astype(np.float32)
    C0 = X[rs.choice(n, k, replace=False)]
    return X, C0


def _run(monkeypatch, X, C0, on, iters=14, reset_at=None, p=0.0, delta=2.0, pipeline=False):
    monkeypatch.setenv("SQ_MULTI_RECORDS", "1" if on else "0")
    monkeypatch.setenv("SQ_ESTEP_BOUNDS", "1")
    monkeypatch.setenv("SQ_MSTEP_INCREMENTAL", "1")
    monkeypatch.setenv("SQ_ESTEP_KEEP_MAX", "1.0")   # always filter
    Xt = torch.from_numpy(X).cuda()
    eng = LloydEngine(Xt, C0.shape[0], delta=delta, intermediate_error=True,
                      true_tomography=False, failure_prob=p, seed=5)
    assert eng.fast and eng.certified and eng.bounds and eng.incremental
    assert (eng.mrec is not None) == on
    eng.set_centers(torch.from_numpy(C0).cuda())
    eng.pipeline = pipeline
    out, cert = [], 0
    for it in range(iters):
        if reset_at is not None and it == reset_at:
            # a restart-like reset to perturbed centres: old records are void
            eng.set_centers(eng.centers().clone() * 1.01)
        labels, sc = eng.step()
        vals = sc.tolist()[:2]
        torch.cuda.synchronize()
        if on and not pipeline:
            cert += int(eng.buf.counts[4].item())
        out.append((labels.clone().cpu(), eng.centers().clone().cpu(), vals))
    eng.pipeline = False
    eng.drop_pending()
    return out, cert


@pytest.mark.parametrize("case", ["plain", "reset", "failures", "pipeline"])
def test_records_on_off_bit_identical(monkeypatch, case):
    X, C0 = _data(seed={"plain": 0, "reset": 1, "failures": 2, "pipeline": 3}[case])
    kw = {"reset": {"reset_at": 7}, "failures": {"p": 0.02},
          "pipeline": {"pipeline": True}}.get(case, {})
    a, cert = _run(monkeypatch, X, C0, True, **kw)
    b, _ = _run(monkeypatch, X, C0, False, **kw)
    if case != "pipeline":
        assert cert > 0, "no row was resolved by the gap screen"
    for (la, Ca, sa), (lb, Cb, sb) in zip(a, b):
        assert torch.equal(la, lb)
        assert torch.equal(Ca, Cb)
        assert sa == sb


def test_screen_wide_band_inertia_close_to_fp64_path(monkeypatch):
    """The fp32 screen settles wide bands whose membership is certain
    (recheck_fast_kernel) and writes their min-vs-label correction from its
    fp32 distances, where the fp64 re-check (SQ_SCREEN=0) uses fp64 ones:
    labels and centres are identical, and the iteration inertia stays within
    a stated tolerance of the fp64 path's (1e-6 relative: fp32 rounding of
    the corrections of the screen-settled rows)."""
    X, C0 = _data(n=80000, d=64, k=96, seed=3, spread=1.2)
    res = {}
    for scr in ("1", "0"):
        monkeypatch.setenv("SQ_SCREEN", scr)
        res[scr], _ = _run(monkeypatch, X, C0, False, iters=8, delta=2.0)
    for (la, ca, va), (lb, cb, vb) in zip(res["1"], res["0"]):
        assert torch.equal(la, lb)
        assert torch.equal(ca, cb)
        assert abs(va[0] - vb[0]) <= 1e-6 * abs(vb[0]), (va, vb)
