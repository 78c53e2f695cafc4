"""Failure-probability model and iteration-level
checkpoint / resume (§5.4) on the CPU path."""
import numpy as np
import pytest
import torch

from sq_learn_amd.cluster import QMeans
from sq_learn_amd.models.cluster._lloyd import LloydEngine
from sq_learn_amd.ops.failure import failure_inject_
from sq_learn_amd.runtime.rng import RngKey
from sq_learn_amd.utils.datasets import make_blobs


def _inject(n, k, p, R, offset=0, seed=3):
    lab = torch.zeros(n, dtype=torch.int64)
    cnt = torch.zeros(2, dtype=torch.int64)
    failure_inject_(lab, k, p, R, RngKey(seed, "failure", 7), offset, cnt)
    return lab, cnt


@pytest.mark.parametrize("p,R", [(0.3, 1), (0.3, 3), (0.05, 2)])
def test_failure_rates(p, R):
    n, k = 200_000, 16
    lab, cnt = _inject(n, k, p, R)
    corrupted = int(cnt[1])
    exp = n * p ** R
    assert abs(corrupted - exp) < 5 * np.sqrt(exp * (1 - p ** R)) + 1
    exp_attempts = n * (1 - p ** R) / (1 - p)
    assert abs(int(cnt[0]) - exp_attempts) < 0.01 * exp_attempts
    # outliers are uniform over the centroids (label 0 is also the "true" label here)
    moved = lab[lab != 0]
    if moved.numel() > 1000:
        h = torch.bincount(moved, minlength=k)[1:].double()
        assert (h.max() / h.mean()).item() < 1.3


def test_failure_zero_and_shard_invariance():
    lab, cnt = _inject(1000, 8, 0.0, 1)
    assert (lab == 0).all() and int(cnt[1]) == 0
    full, _ = _inject(5000, 8, 0.4, 2)
    a, _ = _inject(2000, 8, 0.4, 2, offset=0)
    b, _ = _inject(3000, 8, 0.4, 2, offset=2000)
    assert torch.equal(full, torch.cat([a, b]))


def test_qmeans_failure_policies():
    X, _ = make_blobs(n_samples=3000, centers=5, n_features=4, random_state=0)
    kw = dict(n_clusters=5, n_init=1, max_iter=10, delta=0.2, random_state=0,
              true_distance_estimate=False, intermediate_error=False, tol=0.0)
    ign = QMeans(failure_prob=0.2, failure_policy="ignore", **kw).fit(X)
    res = QMeans(failure_prob=0.2, failure_policy="resample", failure_max_attempts=3, **kw).fit(X)
    assert ign.n_failed_rows_ > res.n_failed_rows_ > 0
    assert res.n_estimations_ > ign.n_estimations_
    clean = QMeans(**kw).fit(X)
    assert clean.n_failed_rows_ == 0
    # corrupted assignments degrade the fit; resampling recovers most of it
    assert res.inertia_ <= ign.inertia_ * 1.05
    with pytest.raises(ValueError):
        QMeans(failure_prob=1.5).fit(X)


class _Crash(RuntimeError):
    pass


def _fit_with_crash(X, ckdir, crash_at, **kw):
    """Fit, raising inside the engine after ``crash_at`` iterations."""
    orig = LloydEngine.step
    calls = {"n": 0}

    def step(self):
        calls["n"] += 1
        if calls["n"] > crash_at:
            raise _Crash()
        return orig(self)

    LloydEngine.step = step
    try:
        with pytest.raises(_Crash):
            QMeans(checkpoint_dir=ckdir, **kw).fit(X)
    finally:
        LloydEngine.step = orig


@pytest.mark.parametrize("crash_at", [5, 17])
def test_checkpoint_resume_is_bit_identical(tmp_path, crash_at):
    X, _ = make_blobs(n_samples=2000, centers=6, n_features=5, cluster_std=2.5, random_state=1)
    kw = dict(n_clusters=6, n_init=2, max_iter=12, delta=0.3, tol=0.0, random_state=4,
              true_distance_estimate=False, intermediate_error=True, true_tomography=False,
              checkpoint_every=2)
    ref = QMeans(**kw).fit(X)
    ckdir = str(tmp_path / "ck")
    _fit_with_crash(X, ckdir, crash_at, **kw)
    resumed = QMeans(checkpoint_dir=ckdir, **kw).fit(X)
    assert hasattr(resumed, "resumed_from_")
    np.testing.assert_array_equal(resumed.cluster_centers_, ref.cluster_centers_)
    np.testing.assert_array_equal(resumed.labels_, ref.labels_)
    assert resumed.inertia_ == ref.inertia_
    # a completed fit leaves no checkpoint behind
    import os
    assert not [f for f in os.listdir(ckdir) if f.endswith(".pt")]


def test_checkpoint_mismatch_starts_over(tmp_path):
    X, _ = make_blobs(n_samples=500, centers=3, n_features=3, random_state=2)
    kw = dict(n_clusters=3, n_init=1, max_iter=8, delta=0.1, tol=0.0, random_state=0,
              true_distance_estimate=False, checkpoint_every=1)
    ckdir = str(tmp_path / "ck")
    _fit_with_crash(X, ckdir, 2, **kw)
    with pytest.warns(UserWarning, match="does not match"):
        m = QMeans(checkpoint_dir=ckdir, **{**kw, "n_clusters": 4}).fit(X)
    assert not hasattr(m, "resumed_from_")


def test_checkpoint_rejects_mixed_generations(tmp_path):
    """A crash between the rank-file and state-file writes leaves new rank
    files beside the previous state: load() must refuse the mix."""
    import torch
    from sq_learn_amd.utils.checkpoint import Checkpointer
    from sq_learn_amd.parallel.comm import Comm
    ck = Checkpointer(str(tmp_path), Comm(None), tag="t", every=1)
    ck.save({"restart": 0, "it": 3, "C": torch.zeros(2)}, {"lab": torch.zeros(3)})
    assert ck.load() is not None
    # simulate: rank file of the next generation written, state file not
    orig = ck._atomic_save
    calls = []

    def only_rank(obj, path):
        calls.append(path)
        if path == ck._rank_path():
            orig(obj, path)
    ck._atomic_save = only_rank
    ck.save({"restart": 0, "it": 6, "C": torch.ones(2)}, {"lab": torch.ones(3)})
    ck._atomic_save = orig
    assert ck.load() is None
