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


@pytest.mark.parametrize("delta,d", [(0.0, 64), (0.5, 256), (3.0, 100)])
def test_incremental_mstep_bit_identical(cuda, delta, d):
    X, _ = make_blobs(60000, d, centers=40, cluster_std=1.5, random_state=0)
    Xt = torch.tensor(X, dtype=torch.float32, device=cuda)
    k = 48
    C0 = Xt[torch.as_tensor(np.random.RandomState(1).choice(60000, k, replace=False), device=cuda)]
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
