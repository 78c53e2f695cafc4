"""List form of the incremental M-step (csrc/kmeans.hip
delta_hist_list_kernel / delta_scatter_list_kernel): after a filtered E-step
only the rows on its three disjoint row lists (unpruned rows, the filter's
own multi rows, list B) are walked.  Labels, centres, the iteration scalars
and the fixed-point cluster statistics are bit-identical to the full walk
over all rows, with gap records on, across a centre reset and pipelined."""
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


def _run(monkeypatch, X, C0, lists, records, iters=14, reset_at=None, pipeline=False):
    monkeypatch.setenv("SQ_DELTA_LISTS", "1" if lists else "0")
    monkeypatch.setenv("SQ_MULTI_RECORDS", "1" if records else "0")
    monkeypatch.setenv("SQ_ESTEP_BOUNDS", "1")
    monkeypatch.setenv("SQ_MSTEP_INCREMENTAL", "1")
    monkeypatch.setenv("SQ_ESTEP_KEEP_MAX", "1.0")   # always filter
    Xt = torch.from_numpy(X).cuda()
    eng = LloydEngine(Xt, C0.shape[0], delta=2.0, intermediate_error=True,
                      true_tomography=False, seed=5)
    assert eng.fast and eng.certified and eng.bounds and eng.incremental
    eng.set_centers(torch.from_numpy(C0).cuda())
    eng.pipeline = pipeline
    out = []
    for it in range(iters):
        if reset_at is not None and it == reset_at:
            eng.set_centers(eng.centers().clone() * 1.01)
        labels, sc = eng.step()
        vals = sc.tolist()[:2]
        torch.cuda.synchronize()
        out.append((labels.clone().cpu(), eng.centers().clone().cpu(), vals))
    eng.pipeline = False
    eng.drop_pending()
    stats = (eng.sums.clone().cpu(), eng.counts.clone().cpu(), eng.qsum.clone().cpu(),
             eng.prev_labels[:eng.n].clone().cpu())
    return out, stats, getattr(eng, "delta_list_steps", 0)


@pytest.mark.parametrize("case", ["plain", "records", "reset", "pipeline"])
def test_delta_lists_bit_identical(monkeypatch, case):
    X, C0 = _data(seed={"plain": 0, "records": 1, "reset": 2, "pipeline": 3}[case])
    rec = case != "plain"
    kw = {"reset": {"reset_at": 7}, "pipeline": {"pipeline": True}}.get(case, {})
    a, sa, used = _run(monkeypatch, X, C0, True, rec, **kw)
    b, sb, unused = _run(monkeypatch, X, C0, False, rec, **kw)
    assert used >= 5 and unused == 0
    for (la, Ca, va), (lb, Cb, vb) in zip(a, b):
        assert torch.equal(la, lb)
        assert torch.equal(Ca, Cb)
        assert va == vb
    for ta, tb in zip(sa, sb):
        assert torch.equal(ta, tb)
