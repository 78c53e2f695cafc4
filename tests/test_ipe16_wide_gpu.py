"""The certified fp16 IPE screen for wide rows (d_pad > 256, up to 1024:
MNIST's d = 784 and d = 1000; ``MnistTrial.py:10-28``, ``Utility.py:697-737``).

Above d_pad 256 a row set's fp16 A fragments no longer fit in VGPRs next to
the sweep's epilogue state, so the sweep's values come from a separate MFMA
pass (``ipe16_values_kernel``: the same operands, k-step order and
instruction from zero) and the sweep reads them (``Ipe16.gv``).

* the values pass is bit-identical to the resident-fragment sweep: forced on
  at d_pad <= 256 (``SQ_IPE16_GV=1``), two E-steps (argmin hints, then the
  screen with the row skip) give the same labels and estimates;
* law at d = 784 / 1000 against the full sampler (fp32 fused kernel, pruning
  off): many near centroids, and a far band whose pairs fire;
* a q-means IPE trajectory at the MNIST shape runs the screen (no fp32
  fallback outside dense rows) and follows the fp32 kernel's inertia."""
import numpy as np
import pytest
import torch

from sq_learn_amd.ops import kmeans as K

from test_ipe16_gpu import _fire_case, _row_and_centroids, _run16, _run_full, _same_law
from test_ipe16_skip_gpu import _blobs, _two_steps

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("d", [64, 256])
def test_values_pass_bit_identical_to_resident_sweep(cuda, monkeypatch, d):
    X, C = _blobs(3, d=d, k=40)
    Xt, Ct = torch.tensor(X, device=cuda), torch.tensor(C, device=cuda)
    outs = []
    for gv in ("0", "1"):
        monkeypatch.setenv("SQ_IPE16_GV", gv)
        st = torch.zeros((2, 8), dtype=torch.int64, device=cuda)
        out, eng = _two_steps(Xt, Ct, 0.25, 13, 5, True, stats=st)
        assert eng.gv == (gv == "1")
        outs.append((out, st.tolist()))
    (oa, sa), (ob, sb) = outs
    assert sa == sb, (sa, sb)
    assert sa[1][7] > 0, sa        # the second step's row skip engaged
    for (la, ma), (lb, mb) in zip(oa, ob):
        assert np.array_equal(la, lb) and np.array_equal(ma, mb)


@pytest.mark.parametrize("d", [784, 1000])
def test_wide_rows_match_full_sampler_law_many_centroids(cuda, d):
    x, C = _row_and_centroids(12, d, 40, 1.0)
    n = 300_000
    X = torch.tensor(np.tile(x, (n, 1)), device=cuda)
    Ct = torch.tensor(C, device=cuda)
    st = torch.zeros(8, dtype=torch.int64, device=cuda)
    la, ma, eng = _run16(X, Ct, 0.1, 13, 1, stats_t=st)
    assert eng.gv and eng.last_dense == 0, st.tolist()
    lb, mb = _run_full(X, Ct, 0.1, 13, 2)
    assert _same_law(la, ma, lb, mb) > 1e-4


@pytest.mark.parametrize("d", [784, 1000])
def test_wide_rows_fire_path_matches_full_sampler_law(cuda, d):
    x, C = _fire_case(d=d, K_=301)
    # the d = 96 case's norms (|x|^2 ~ 96: the estimation noise ~ eps |x.c|
    # stays below the competitors' distance), every pair shifted along x
    # (distances unchanged: the competitors' directions are orthogonal to x)
    xs = (x * np.sqrt(96.0 / float(x @ x))).astype(np.float32)
    C = (C + (xs - x)[None]).astype(np.float32)
    x = xs
    n = 300_000
    X = torch.tensor(np.tile(x, (n, 1)), device=cuda)
    Ct = torch.tensor(C, device=cuda)
    hint = torch.zeros(n, dtype=torch.int32, device=cuda)
    st = torch.zeros(8, dtype=torch.int64, device=cuda)
    la, ma, eng = _run16(X, Ct, 0.25, 13, 5, hint=hint, stats_t=st, ht=9e-4)
    s = st.tolist()
    assert eng.gv and eng.last_dense < 1e-3 * n and s[0] == 0, s
    assert s[1] > 0.05 * n and s[4] > 0.05 * n, s
    lb, mb = _run_full(X, Ct, 0.25, 13, 6)
    assert _same_law(la, ma, lb, mb, min_cells=2) > 1e-4


def test_mnist_shape_trajectory_uses_the_screen(cuda, monkeypatch):
    """70k x 784, k = 10 (MNIST's shape): the IPE Lloyd steps run the fp16
    screen (values pass), the fp32 kernel only for dense rows, and the
    inertia follows the fp32 kernel's trajectory within the law's noise."""
    from sq_learn_amd.models._data import Data, gather_rows
    from sq_learn_amd.models.cluster._lloyd import LloydEngine
    from sq_learn_amd.parallel.comm import Comm
    from sq_learn_amd.utils.datasets import make_blobs_device
    n, d, k = 70_000, 784, 10
    X, _ = make_blobs_device(n, d, centers=k, cluster_std=4.0, seed=4, device=cuda,
                             dtype=torch.float32)
    C0 = gather_rows(Data(X, n, 0, Comm(None), "sharded"),
                     np.random.RandomState(4).choice(n, k, replace=False))
    out = {}
    for use16 in ("0", "1"):
        monkeypatch.setenv("SQ_IPE16", use16)
        eng = LloydEngine(X, k, delta=0.5, true_distance_estimate=True, intermediate_error=True,
                          seed=3)
        eng.set_centers(C0)
        out[use16] = [eng.step()[1].tolist()[0] for _ in range(4)]
        if use16 == "1":
            st16 = eng._ipe16
            assert st16 is not None and st16.gv and st16.last_dense < 0.05 * n
    a, b = np.array(out["0"]), np.array(out["1"])
    assert np.all(np.abs(a - b) <= 2e-3 * a), (a, b)
