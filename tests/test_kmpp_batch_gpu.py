"""Batched k-means++ restarts (csrc/kmpp.hip ``sq_kmpp_batch``,
``ops.kmeans.KmppBatch``): the restarts' draws are taken up front in the
reference order (``_dmeans.py:153-247, 1285-1306``: the Lloyd loop never
draws from random_state), then all restarts advance through their centres
together.  Centres, ids and the RandomState afterwards must equal sequential
``kmeans_plusplus`` calls, with the screens on and off; a q-means fit with
n_init = 3 gives the same result either way."""
import numpy as np
import pytest
import torch

from sq_learn_amd.models._data import Data
from sq_learn_amd.models.cluster import _init as I
from sq_learn_amd.parallel.comm import Comm

pytestmark = pytest.mark.gpu


def _data(cuda, n=120_000, d=64, blobs=40, seed=0):
    rs = np.random.RandomState(seed)
    G = rs.uniform(-4, 4, (blobs, d))
    X = (G[rs.randint(blobs, size=n)] + rs.randn(n, d)).astype(np.float32)
    Xt = torch.from_numpy(X).to(cuda)
    return Data(Xt, n, 0, Comm(None), "sharded")


# (the pruned cases run the fused screen / bound: t = 5 -> 8 columns per
# restart; k = 3000: t = 10 -> 16 columns, one restart per MFMA block; R = 16
# x 8 = 128 columns, the limit)
@pytest.mark.parametrize("prune,d,k,R,n", [(True, 64, 48, 4, 120_000), (False, 64, 48, 4, 120_000),
                                           (True, 256, 48, 4, 120_000),
                                           (True, 128, 48, 16, 60_000),
                                           (True, 64, 3000, 3, 40_000)])
def test_batched_restarts_equal_sequential(cuda, prune, d, k, R, n):
    data = _data(cuda, d=d, n=n)
    rs1 = np.random.RandomState(7)
    seq = [I.kmeans_plusplus(data, k, rs1, prune=prune) for _ in range(R)]
    rs2 = np.random.RandomState(7)
    bat = I.kmeans_plusplus_restarts(data, k, rs2, R, prune=prune)
    assert bat is not None and len(bat) == R
    for (C, ids), Cb in zip(seq, bat):
        assert torch.equal(C, Cb)
    assert rs1.random_sample() == rs2.random_sample()


def test_qmeans_fit_n_init_batched_matches_sequential(cuda, monkeypatch):
    from sq_learn_amd.models.cluster import qmeans as Q
    data = _data(cuda, n=60_000, d=32, blobs=20, seed=1)
    X = data.X
    kw = dict(n_clusters=16, delta=0.5, true_distance_estimate=False, intermediate_error=True,
              init="k-means++", n_init=3, max_iter=8, random_state=5, device=str(cuda))
    a = Q.QMeans(**kw).fit(X)
    monkeypatch.setattr(Q, "kmeans_plusplus_restarts", lambda *a_, **k_: None)
    b = Q.QMeans(**kw).fit(X)
    assert len(a.fit_restart_inertias_) == 3
    assert a.fit_restart_inertias_ == b.fit_restart_inertias_
    assert np.array_equal(a.labels_, b.labels_)
    assert a.inertia_ == b.inertia_


@pytest.mark.parametrize("env", ["SQ_KMPP_FUSED", "SQ_KMPP_PAIRS"])
def test_fused_passes_equal_per_restart_passes(cuda, monkeypatch, env):
    """SQ_KMPP_FUSED=0 (per-restart screen / bound) and SQ_KMPP_PAIRS=0 (the
    exact pass over every trial of a listed row) give the same centres."""
    data = _data(cuda, n=100_000, d=96, blobs=30, seed=3)
    a = I.kmeans_plusplus_restarts(data, 64, np.random.RandomState(11), 6)
    monkeypatch.setenv(env, "0")
    b = I.kmeans_plusplus_restarts(data, 64, np.random.RandomState(11), 6)
    for Ca, Cb in zip(a, b):
        assert torch.equal(Ca, Cb)
