"""Pipelined Lloyd steps (``LloydEngine.pipeline``): the next iteration's
E-step is enqueued right after the M-step, before the host reads the
iteration's scalars.  Same kernels, same Philox keys, same stream order - so
per-iteration scalars, returned labels and the final centroids must be
BIT-identical to the unpipelined loop, and a loop that stops (dropping the
speculative E-step) must leave a final E-step identical too.  (Scalar 3, the
Hamerly filter's kept count, is a scheduling diagnostic: the adaptive filter
decides on the host's view of it, which lags by one step when pipelined.)  QMeans.fit
runs pipelined without checkpoints: its result must equal a fit whose loop
is forced unpipelined."""
import numpy as np
import pytest
import torch

from sq_learn_amd.models.cluster import QMeans
from sq_learn_amd.models.cluster._lloyd import LloydEngine
from sq_learn_amd.utils.datasets import make_blobs

pytestmark = pytest.mark.gpu


def _run(Xt, C0, k, delta, pipeline, steps):
    eng = LloydEngine(Xt, k, delta=delta, intermediate_error=delta > 0, seed=11,
                      gemm_precision="fp32")
    eng.set_centers(C0)
    eng.pipeline = pipeline
    scal, labs = [], []
    for _ in range(steps):
        labels, sc = eng.step()
        scal.append(sc.tolist())
        labs.append(labels.clone())
    eng.pipeline = False
    eng.drop_pending()
    fin_lab, fin_mind, fin_in = eng.estep()
    return scal, labs, eng.centers().clone(), fin_lab.clone(), float(fin_in.sum())


@pytest.mark.parametrize("delta,d", [(0.5, 256), (0.0, 64), (1.0, 100)])
def test_pipelined_steps_bit_identical(cuda, delta, d):
    X, _ = make_blobs(40000, d, centers=32, cluster_std=2.0, random_state=2)
    Xt = torch.tensor(X, dtype=torch.float32, device=cuda)
    k = 40
    C0 = Xt[torch.as_tensor(np.random.RandomState(5).choice(Xt.shape[0], k, replace=False),
                            device=cuda)]
    a = _run(Xt, C0, k, delta, False, 9)
    b = _run(Xt, C0, k, delta, True, 9)
    # inertia / shift / overflow per step
    assert [s[:3] for s in a[0]] == [s[:3] for s in b[0]]
    for la, lb in zip(a[1], b[1]):
        assert torch.equal(la, lb)
    assert torch.equal(a[2], b[2])                        # centroids
    assert torch.equal(a[3], b[3]) and a[4] == b[4]       # final E-step after the loop


def test_qmeans_fit_pipelined_equals_unpipelined(cuda, monkeypatch):
    X, _ = make_blobs(30000, 128, centers=24, cluster_std=1.5, random_state=4)
    kw = dict(n_clusters=24, delta=0.5, true_distance_estimate=False, intermediate_error=True,
              true_tomography=False, n_init=1, max_iter=30, random_state=0, device="cuda:0")
    piped = QMeans(**kw).fit(X)
    # force the loop unpipelined: the engine ignores the flag when it is reset
    orig = LloydEngine.step

    def step_nopipe(self):
        self.pipeline = False
        return orig(self)

    monkeypatch.setattr(LloydEngine, "step", step_nopipe)
    plain = QMeans(**kw).fit(X)
    assert piped.n_iter_ == plain.n_iter_
    np.testing.assert_array_equal(np.asarray(piped.labels_), np.asarray(plain.labels_))
    np.testing.assert_array_equal(np.asarray(piped.cluster_centers_),
                                  np.asarray(plain.cluster_centers_))
    assert piped.inertia_ == plain.inertia_
