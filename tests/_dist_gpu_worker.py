"""Worker of tests/test_distributed_gpu.py: one rank of a torchrun job whose
ranks ALL run on cuda:0 with the gloo backend (SQ_DIST_BACKEND=gloo - the
one-GPU rehearsal of the RCCL path: the same sharded code, the collectives
staged through host memory).  Every case fits the full data in this process
(world 1) and the row-sharded data (world W, uneven shards) and records how
far apart they are; rank 0 writes the results as JSON for the test to assert.

usage: torchrun ... _dist_gpu_worker.py OUT_JSON
"""
import json
import os
import sys
import traceback
import warnings

import numpy as np
import torch


def _bounds(n, world):
    # deliberately uneven shards (not shard_bounds): 2 ranks 40/60 %, 3 ranks
    # 20/50/30 %
    fr = {1: [1.0], 2: [0.4, 0.6], 3: [0.2, 0.5, 0.3]}[world]
    cuts = [0]
    for f in fr[:-1]:
        cuts.append(cuts[-1] + int(round(f * n)))
    cuts.append(n)
    return cuts


def main(out_path):
    warnings.simplefilter("ignore")
    from sq_learn_amd.parallel.comm import init_distributed
    from sq_learn_amd.parallel.sharding import ShardedArray
    comm = init_distributed()
    assert comm.world_size > 1 and comm.backend == "gloo", (comm.world_size, comm.backend)
    dev = os.environ.get("SQ_TEST_DEVICE", "cuda:0")   # cpu: dry run of the logic
    if dev.startswith("cuda"):
        torch.cuda.set_device(0)
    rank, world = comm.rank, comm.world_size

    # which engine configuration ran (the fast certified path must be the one
    # under test, not a generic fallback)
    from sq_learn_amd.models.cluster import _lloyd
    seen = []
    orig_init = _lloyd.LloydEngine.__init__

    def spy(self, *a, **kw):
        orig_init(self, *a, **kw)
        seen.append(dict(fast=bool(self.fast), certified=bool(getattr(self, "certified", False)),
                         bounds=bool(getattr(self, "bounds", False)),
                         incremental=bool(getattr(self, "incremental", False)),
                         relocate=bool(self.relocate_empty), n=int(self.n)))
    _lloyd.LloydEngine.__init__ = spy

    def shard(X):
        cuts = _bounds(X.shape[0], world)
        s0, s1 = cuts[rank], cuts[rank + 1]
        return ShardedArray(torch.as_tensor(X[s0:s1]).contiguous(), X.shape[0], s0, comm)

    def gather_labels(lab):
        t = torch.as_tensor(np.asarray(lab).astype(np.int64))
        return torch.cat(comm.all_gather_varlen(t)).numpy()

    def tonp(a):
        return a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)

    def rel(a, b):
        a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
        return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))

    from sq_learn_amd.utils.datasets import make_blobs
    res = {}
    X, _ = make_blobs(12011, 32, centers=48, cluster_std=3.0, random_state=7)
    X = X.astype(np.float32)
    Xs = shard(X)

    from sq_learn_amd.models.cluster import QMeans, KMeans
    for init in ("k-means++", "random", "k-means||"):
        kw = dict(n_clusters=48, delta=0.5, true_distance_estimate=False, intermediate_error=True,
                  true_tomography=False, random_state=3, n_init=2, max_iter=25, init=init,
                  device=dev)
        seen.clear()
        ref = QMeans(**kw).fit(X)
        ref_cfg = list(seen)
        seen.clear()
        got = QMeans(**kw).fit(Xs)
        got_cfg = list(seen)
        full = gather_labels(got.labels_)
        res["qmeans_" + init] = dict(
            labels_equal=bool(np.array_equal(full, ref.labels_)),
            centers_bitwise=bool(np.array_equal(got.cluster_centers_, ref.cluster_centers_)),
            centers_rel=rel(got.cluster_centers_, ref.cluster_centers_),
            inertia_rel=abs(got.inertia_ - ref.inertia_) / ref.inertia_,
            n_iter=[int(got.n_iter_), int(ref.n_iter_)],
            cond_rel=abs(got.condition_number - ref.condition_number) / ref.condition_number,
            muA_rel=abs(got.muA - ref.muA) / ref.muA,
            cfg_ref=ref_cfg[-1], cfg_got=got_cfg[-1])

    # the reference DEFAULT distance mode: IPE (fused csrc/ipe.hip kernel,
    # row-keyed hazard streams and label hints), k-means++ init
    kw = dict(n_clusters=24, delta=0.5, true_distance_estimate=True, intermediate_error=True,
              true_tomography=False, random_state=5, n_init=1, max_iter=6, tol=0.0,
              init="k-means++", device=dev)
    ref = QMeans(**kw).fit(X)
    got = QMeans(**kw).fit(Xs)
    res["qmeans_ipe"] = dict(
        labels_equal=bool(np.array_equal(gather_labels(got.labels_), ref.labels_)),
        centers_bitwise=bool(np.array_equal(got.cluster_centers_, ref.cluster_centers_)),
        inertia_rel=abs(got.inertia_ - ref.inertia_) / ref.inertia_,
        n_iter=[int(got.n_iter_), int(ref.n_iter_)])

    # wide rows: the certified filter at d_pad 512 / 1024 (d = 300, 784) and
    # the exact fp64 rows kernel beyond it (d = 1100) under k-means||
    for d_w, init_w in ((300, "k-means++"), (784, "random"), (1100, "k-means||")):
        Xw, _ = make_blobs(4001, d_w, centers=16, cluster_std=2.0, random_state=d_w)
        Xw = Xw.astype(np.float32)
        kw = dict(n_clusters=16, delta=0.5, true_distance_estimate=False, intermediate_error=True,
                  true_tomography=False, random_state=2, n_init=1, max_iter=8, init=init_w,
                  device=dev)
        seen.clear()
        ref = QMeans(**kw).fit(Xw)
        ref_cfg = list(seen)
        seen.clear()
        got = QMeans(**kw).fit(shard(Xw))
        got_cfg = list(seen)
        res[f"qmeans_d{d_w}"] = dict(
            labels_equal=bool(np.array_equal(gather_labels(got.labels_), ref.labels_)),
            centers_bitwise=bool(np.array_equal(got.cluster_centers_, ref.cluster_centers_)),
            inertia_rel=abs(got.inertia_ - ref.inertia_) / ref.inertia_,
            n_iter=[int(got.n_iter_), int(ref.n_iter_)],
            cfg_ref=ref_cfg[-1], cfg_got=got_cfg[-1])

    # classical KMeans (fp32 certified E-step + empty-cluster relocation):
    # two far initial centres own no rows at the first E-step
    rng = np.random.RandomState(0)
    Xr = np.vstack([rng.randn(3000, 8) + 6 * (i % 3) for i in range(3)] +
                   [rng.randn(5, 8) * 0.1 + 40.0]).astype(np.float32)
    init = np.vstack([Xr[0], Xr[3000], Xr[6000], np.full(8, 500.0), np.full(8, -500.0)])
    seen.clear()
    ref = KMeans(n_clusters=5, init=init, n_init=1, max_iter=30, device=dev).fit(Xr)
    ref_cfg = list(seen)
    seen.clear()
    got = KMeans(n_clusters=5, init=init, n_init=1, max_iter=30, device=dev).fit(shard(Xr))
    got_cfg = list(seen)
    res["kmeans_relocate"] = dict(
        labels_equal=bool(np.array_equal(gather_labels(got.labels_), ref.labels_)),
        centers_bitwise=bool(np.array_equal(got.cluster_centers_, ref.cluster_centers_)),
        centers_rel=rel(got.cluster_centers_, ref.cluster_centers_),
        inertia_rel=abs(got.inertia_ - ref.inertia_) / ref.inertia_,
        n_iter=[int(got.n_iter_), int(ref.n_iter_)],
        distinct=int(len(np.unique(ref.labels_))),
        cfg_ref=ref_cfg[-1] if ref_cfg else None, cfg_got=got_cfg[-1] if got_cfg else None)

    # CholeskyQR2 sigma_min on the fp64 Gram kernel (two passes, two d x d
    # all-reduces), centred and not
    from sq_learn_amd.models._data import as_data, sigma_min, global_mean_var
    Z = (rng.randn(9001, 24) @ rng.randn(24, 24)).astype(np.float32)
    d1 = as_data(Z, device=dev)
    dW = as_data(shard(Z), device=dev)
    m1, _ = global_mean_var(d1)
    mW, _ = global_mean_var(dW)
    res["sigma_min"] = dict(plain_rel=abs(sigma_min(dW) - sigma_min(d1)) / sigma_min(d1),
                            centred_rel=abs(sigma_min(dW, mW) - sigma_min(d1, m1)) / sigma_min(d1, m1))

    # qPCA full (Gram) and randomized, quantum extras with Gaussian and true
    # (long-vector, rank-split multinomial) tomography of the left vectors
    from sq_learn_amd.models.decomposition import QPCA
    Zq = (rng.randn(6007, 20) @ rng.randn(20, 20)).astype(np.float32)
    for solver, tt in (("full", False), ("full", True), ("randomized", False),
                       ("randomized", True)):
        kw = dict(n_components=4, svd_solver=solver, random_state=0, device=dev)
        fk = dict(eps=1e-3, theta_major=1e-6, delta=0.3, estimate_all=True, true_tomography=tt)
        if solver == "randomized":
            kw["quantum_truncated"] = True
        # tensor input: the left vectors stay device tensors (numpy input
        # returns them as numpy and takes the host RNG, like the reference)
        ref = QPCA(**kw).fit(torch.as_tensor(Zq).to(dev), **fk)
        got = QPCA(**kw).fit(shard(Zq), **fk)
        left = tonp(got.estimate_left_sv)
        fullL = torch.cat(comm.all_gather_varlen(torch.as_tensor(left.T).contiguous())).T.numpy()
        Ug = torch.cat(comm.all_gather_varlen(
            torch.as_tensor(tonp(got.left_sv).T).contiguous())).T.numpy()
        refL = tonp(ref.estimate_left_sv)
        res[f"qpca_{solver}_{'true' if tt else 'gauss'}"] = dict(
            sv_rel=rel(tonp(got.singular_values_), tonp(ref.singular_values_)),
            comp_absdiff=float(np.max(np.abs(np.abs(tonp(got.components_)) - np.abs(tonp(ref.components_))))),
            left_err=[float(v) for v in np.linalg.norm(fullL - Ug, axis=1)],
            left_shape=list(fullL.shape),
            # Gaussian tomography draws Philox element (i, global column):
            # the same noise as the single-process fit (up to the left
            # vectors' own rounding)
            left_vs_ref=float(np.max(np.abs(np.abs(fullL) - np.abs(refL)))),
            muA_rel=abs(got.muA - ref.muA) / ref.muA)

    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(dict(world=world, results=res), f, indent=1)


if __name__ == "__main__":
    try:
        main(sys.argv[1])
    except Exception:
        traceback.print_exc()
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(1)
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
