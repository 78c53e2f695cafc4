#!/usr/bin/env python
"""Headline benchmark: q-means Lloyd-iteration throughput on 10M x 256,
k = 1024, row-sharded over N MI355X GPUs (BASELINE.json config 3), plus the
q-means fit wall-clock and the qPCA wall-clocks (configs 2/5) as extras.

One step = one full q-means iteration of the reference's delta-means path
(``_dmeans.py:534-671`` with ``delta > 0``, ``true_distance_estimate=False``,
``intermediate_error=True``, Gaussian tomography) at REFERENCE PRECISION:
fp32 data, the certified E-step (csrc/estep_f32.hip: fp16 MFMA filter with a
rigorous error bound + fp64 re-check of the candidates -> the fp64 delta-band
labels of ``_dmeans.py:742-751``; crowded rows through the fp32-faithful
3-pass kernel), the segmented centroid reduce that also yields the exact fp64
min distances, one packed RCCL all-reduce, centroid finalise with
truncated-normal tomography noise, convergence scalars read back to the host.
Nothing is skipped inside the timed region.

Strong scaling: the 10M rows are split across ranks (each rank generates its
own shard in HBM from the global Philox stream - same dataset for every N).

    python bench.py [--gpus N --steps K --warmup W]
    (N > 1 without torchrun: re-launched under torch.distributed.run, one
     process per GPU, before any GPU call)
"""

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

BASELINE_SAMPLES_PER_S = 3.7e3   # reference q-means iteration, 8-core Xeon


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", dest="n", type=int, default=10_000_000)
    ap.add_argument("--features", dest="d", type=int, default=256)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--delta", type=float, default=0.5)
    ap.add_argument("--blobs", type=int, default=1024)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="fp32: reference precision (default); bf16: fast approximate E-step")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--no-qpca", action="store_true")
    ap.add_argument("--no-fit", action="store_true")
    ap.add_argument("--fit-iters", type=int, default=10)
    ap.add_argument("--ipe-steps", type=int, default=3,
                    help="timed steady-state Lloyd steps of the IPE (true_distance_estimate) "
                         "extra, after its first two (separately timed) steps; 0 = skip")
    ap.add_argument("--ipe-warm", type=int, default=3,
                    help="untimed IPE steps between the second step and the timed ones")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--no-hard", action="store_true", help="skip the overlapping-blobs extra")
    ap.add_argument("--no-mnist", action="store_true", help="skip the 70k x 784 (config 4) extra")
    ap.add_argument("--no-share8", action="store_true", help="skip the N = 8 per-GPU share extra")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="skip the qPCA -> q-means pipeline (config 5) extra")
    ap.add_argument("--pipeline-rows", type=int, default=50_000_000)
    return ap.parse_args(argv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawn(a):
    """--gpus N > 1 outside torchrun: run N ranks under torch.distributed.run
    (one process per GPU) as a child and exit with its code.  No GPU call has
    been made in this process."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def _max_over_ranks(comm, dev, v):
    t = torch.tensor([float(v)], dtype=torch.float64, device=dev)
    comm.all_reduce_(t, op="max")
    return float(t.item())


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def _qpca_extra(extra, name, sa, comm, dev, solver, n_components=16, true_tomography=False):
    """Wall-clock of a QPCA fit with the quantum extras of ``_qPCA.py:357-465``
    (CPE singular values, Theorem 11 top-k extraction + tomography of the
    right AND the n-long left singular vectors; on the randomized path via
    ``quantum_truncated=True``, BASELINE config 2); one untimed warm fit of
    the same call first (every kernel of the path already loaded).  Never
    breaks the line."""
    try:
        from sq_learn_amd.models.decomposition import QPCA
        qt = solver != "full"
        q = QPCA(n_components=n_components, svd_solver=solver, random_state=0, device=dev).fit(sa)
        theta = 0.5 * float(q.singular_values_[n_components - 1])

        def fit():
            q = QPCA(n_components=n_components, svd_solver=solver, random_state=0, device=dev,
                     quantum_truncated=qt)
            q.fit(sa, eps=1e-3, theta_major=theta, delta=0.1, estimate_all=True,
                  true_tomography=true_tomography)
            return q

        fit()
        _sync(dev)
        comm.barrier()
        t0 = time.perf_counter()
        q = fit()
        _sync(dev)
        assert q.topk == n_components and q.estimate_left_sv is not None
        _sync(dev)
        comm.barrier()
        extra[name] = _max_over_ranks(comm, dev, time.perf_counter() - t0)
    except Exception as e:  # qPCA must not break the headline line
        extra[name + "_error"] = repr(e)[:200]


def _ipe_extra(extra, a, X, comm, dev, start, C0):
    """Lloyd throughput with the reference's DEFAULT distance mode,
    true_distance_estimate=True (``_dmeans.py:753-772``): every (row,
    centroid) distance is |x|^2 + |c|^2 - 2 IPE(x, c), IPE = median of 13
    amplitude estimations, drawn from its exact law.  The certified fp16
    screen (csrc/ipe16.hip: hint pair in full, fp16 MFMA band
    classification + per-pair certificate, row skip by Hamerly-style bounds,
    canonical fp32 dots and samplers only for near / fired pairs; rows it
    cannot certify through the fp32 kernel of csrc/ipe.hip).  Same data, k
    and delta as the headline.  First and second steps timed on their own;
    then ``--ipe-warm`` untimed steps and ``--ipe-steps`` timed ones (the
    steady state, like the headline's warmup)."""
    try:
        from sq_learn_amd.models.cluster._lloyd import LloydEngine
        eng = LloydEngine(X, a.k, delta=a.delta, true_distance_estimate=True,
                          intermediate_error=True, true_tomography=False, seed=a.seed, comm=comm,
                          row_offset=start, gemm_precision="fp32")
        eng.set_centers(C0)
        _sync(dev)
        comm.barrier()
        t0 = time.perf_counter()
        eng.step()[1].tolist()    # no label hints yet: the first-sweep hints
        _sync(dev)
        comm.barrier()
        extra["ipe_first_step_ms"] = _max_over_ranks(comm, dev, (time.perf_counter() - t0) * 1e3)
        # the second step: label hints from the first, still far from converged
        t0 = time.perf_counter()
        eng.step()[1].tolist()
        _sync(dev)
        comm.barrier()
        extra["ipe_second_step_ms"] = _max_over_ranks(comm, dev, (time.perf_counter() - t0) * 1e3)
        for _ in range(a.ipe_warm):
            eng.step()[1].tolist()
        _sync(dev)
        comm.barrier()
        t0 = time.perf_counter()
        for _ in range(a.ipe_steps):
            eng.step()[1].tolist()
        _sync(dev)
        comm.barrier()
        el = _max_over_ranks(comm, dev, time.perf_counter() - t0)
        extra["ipe_samples_iter_per_s"] = a.n * a.ipe_steps / el
        extra["ipe_ms_per_step"] = el / a.ipe_steps * 1e3
        extra["ipe_pairs_per_s"] = a.n * a.k * a.ipe_steps / el
        # one more (untimed) step with the screens' pair counters: the fp16
        # band screen (csrc/ipe16.hip) and the fp32 kernel of its dense rows
        eng.ipe_stats = torch.zeros(5, dtype=torch.int64, device=dev)
        eng.ipe16_stats = torch.zeros(8, dtype=torch.int64, device=dev)
        eng.step()[1].tolist()
        st = eng.ipe_stats.double()
        comm.all_reduce_(st)
        s16 = eng.ipe16_stats.double()
        comm.all_reduce_(s16)
        tot = float(a.n) * a.k
        extra["ipe_screen"] = {
            "listed_near_per_row": float(s16[0]) / a.n, "fired_per_row": float(s16[1]) / a.n,
            "full_sampler_per_row": (float(s16[6]) + float(st[1])) / a.n,
            "fired_exact_branch": int(s16[2]) + int(st[3]),
            "dense_row_frac": float(s16[3]) / a.n, "no_band_row_frac": float(s16[5]) / a.n,
            "dense_rows_fp32_screened_frac": float(st[0]) / tot}
        eng.ipe_stats = eng.ipe16_stats = None
        del eng
        torch.cuda.empty_cache()
    except Exception as e:
        extra["ipe_error"] = repr(e)[:200]


def _share8_extra(extra, a, X, comm, dev, C0):
    """The per-GPU share of an 8-GPU run (rows n / 8) stepped on this GPU:
    the same pipelined, pruned, incremental headline iteration on the first
    n / 8 rows from the headline's initial centres (the N = 8 run's centres
    come from the global init: rank 0's rows with the global trajectory's
    centres, not a separate 1.25M-row problem with its own init) - the N = 8
    per-rank compute cost; the all-reduce is a no-op here."""
    try:
        from sq_learn_amd.models.cluster._lloyd import LloydEngine
        m = a.n // 8
        Xs = X[:m]
        eng = LloydEngine(Xs, a.k, delta=a.delta, true_distance_estimate=False,
                          intermediate_error=True, true_tomography=False, seed=a.seed, comm=comm,
                          row_offset=0, gemm_precision=a.dtype)
        eng.set_centers(C0)
        eng.pipeline = True
        for _ in range(max(a.warmup, 3)):
            eng.step()[1].tolist()
        _sync(dev)
        t0 = time.perf_counter()
        steps = max(a.steps, 10)
        for _ in range(steps):
            eng.step()[1].tolist()
        _sync(dev)
        extra["share8_rows"] = m
        extra["share8_ms_per_step"] = (time.perf_counter() - t0) / steps * 1e3
        eng.pipeline = False
        eng.drop_pending()
        del eng
        torch.cuda.empty_cache()
    except Exception as e:
        extra["share8_error"] = repr(e)[:200]


def _hard_extra(extra, a, comm, dev, unpruned=True):
    """A hard regime for the certified E-step: 1024 strongly overlapping
    blobs (centres in [-0.1, 0.1]^d, spread 0.4: a mean delta-band of ~3
    members, ~60 % multi-candidate rows) so that most rows have several
    centroids within delta of their minimum.  Reports the steady-state
    and unpruned ms per step, the first iteration, the dense / multi-candidate
    row fractions of the last step and the mean delta-band size (fp64, on a
    4096-row sample).  Rows: a.n / 5 (2M at the default)."""
    try:
        from sq_learn_amd.parallel.comm import shard_bounds
        from sq_learn_amd.utils.datasets import make_blobs_device
        from sq_learn_amd.models.cluster._lloyd import LloydEngine
        from sq_learn_amd.models._data import Data, gather_rows
        n = max(a.n // 5, 4096)
        s0, s1 = shard_bounds(n, comm.rank, comm.world_size)
        X, _ = make_blobs_device(n, a.d, centers=a.blobs, cluster_std=0.4, center_box=(-0.1, 0.1),
                                 seed=a.seed + 1, device=dev, dtype=torch.float32,
                                 row_range=(s0, s1))
        data = Data(X, n, s0, comm, "sharded")
        rs = np.random.RandomState(a.seed + 1)
        C0 = gather_rows(data, rs.choice(n, a.k, replace=False))
        eng = LloydEngine(X, a.k, delta=a.delta, true_distance_estimate=False,
                          intermediate_error=True, true_tomography=False, seed=a.seed, comm=comm,
                          row_offset=s0, gemm_precision="fp32")
        eng.set_centers(C0)

        def timed(steps):
            _sync(dev)
            comm.barrier()
            t0 = time.perf_counter()
            for _ in range(steps):
                eng.step()[1].tolist()
            _sync(dev)
            comm.barrier()
            return _max_over_ranks(comm, dev, (time.perf_counter() - t0) / steps * 1e3)

        extra["hard_first_iter_ms"] = timed(1)
        for _ in range(4):
            eng.step()[1].tolist()
        extra["hard_ms_per_step"] = timed(5)
        kf = getattr(eng, "_kept_frac", None)
        if kf is not None:
            extra["hard_filter_kept_frac"] = round(float(kf), 4)
        cnt = eng.buf.counts.tolist()
        tot = torch.tensor([float(cnt[1]), float(cnt[2])], dtype=torch.float64, device=dev)
        comm.all_reduce_(tot)
        extra["hard_dense_row_frac"] = float(tot[0]) / n
        extra["hard_multi_row_frac"] = float(tot[1]) / n
        if unpruned and getattr(eng, "bounds", False):
            # the same iterations (1 .. 10 from the same centres) with the
            # Hamerly bounds off, on a fresh engine: like for like
            C_last = eng.centers().clone()
            eng2 = LloydEngine(X, a.k, delta=a.delta, true_distance_estimate=False,
                               intermediate_error=True, true_tomography=False, seed=a.seed,
                               comm=comm, row_offset=s0, gemm_precision="fp32")
            eng2.bounds = False
            eng2.set_centers(C0)
            eng_b, eng = eng, eng2
            timed(1)
            for _ in range(4):
                eng.step()[1].tolist()
            extra["hard_unpruned_ms_per_step"] = timed(5)
            cnt = eng.buf.counts.tolist()
            tot = torch.tensor([float(cnt[1]), float(cnt[2])], dtype=torch.float64, device=dev)
            comm.all_reduce_(tot)
            extra["hard_unpruned_dense_row_frac"] = float(tot[0]) / n
            extra["hard_unpruned_multi_row_frac"] = float(tot[1]) / n
            extra["hard_unpruned_same_centres"] = bool(torch.equal(eng.centers(), C_last))
            del eng
            eng = eng_b
        if comm.rank == 0:
            m = min(4096, s1 - s0)
            Xs = X[:m].double()
            C = eng.centers().double()
            D = ((Xs * Xs).sum(1)[:, None] + (C * C).sum(1)[None, :] - 2.0 * Xs @ C.T)
            band = (D <= D.min(1, keepdim=True).values + a.delta).sum(1).double()
            extra["hard_mean_band_size"] = float(band.mean())
        extra["hard_rows"] = n
        del eng, X
        torch.cuda.empty_cache()
    except Exception as e:
        extra["hard_error"] = repr(e)[:200]


def _mnist_extra(extra, a, comm, dev):
    """BASELINE config 4 shape (MNIST 70k x 784, k = 10; synthetic blobs of
    that shape): wall-clock of the classical KMeans (k-means++, certified
    fp32 E-step at d_pad = 1024) and PCA (50 components, CholeskyQR2 on the
    fp64-MFMA Gram kernels) fits, and the q-means Lloyd step (delta-means +
    tomography noise) on the same matrix."""
    try:
        from sq_learn_amd.parallel.comm import shard_bounds
        from sq_learn_amd.parallel.sharding import ShardedArray
        from sq_learn_amd.utils.datasets import make_blobs_device
        from sq_learn_amd.models.cluster import KMeans, QMeans
        from sq_learn_amd.models.decomposition import PCA
        n, d, k = 70_000, 784, 10
        s0, s1 = shard_bounds(n, comm.rank, comm.world_size)
        X, _ = make_blobs_device(n, d, centers=k, cluster_std=4.0, center_box=(0.0, 8.0),
                                 seed=a.seed + 7, device=dev, dtype=torch.float32,
                                 row_range=(s0, s1))
        sa = ShardedArray(X, n, s0, comm)

        def wall(fn):
            fn()   # warm (kernel load, workspace allocation)
            _sync(dev)
            comm.barrier()
            t0 = time.perf_counter()
            r = fn()
            _sync(dev)
            comm.barrier()
            return _max_over_ranks(comm, dev, time.perf_counter() - t0), r

        t, km = wall(lambda: KMeans(n_clusters=k, n_init=1, max_iter=30, random_state=0,
                                    device=dev).fit(sa))
        extra["mnist70kx784_kmeans_fit_s"] = t
        extra["mnist70kx784_kmeans_n_iter"] = int(km.n_iter_)
        t, _ = wall(lambda: PCA(n_components=50, random_state=0, device=dev).fit(sa))
        extra["mnist70kx784_pca50_fit_s"] = t
        t, qm = wall(lambda: QMeans(n_clusters=k, delta=a.delta, true_distance_estimate=False,
                                    intermediate_error=True, true_tomography=False, n_init=1,
                                    max_iter=20, tol=0.0, random_state=0, device=dev).fit(sa))
        extra["mnist70kx784_qmeans_fit_s"] = t
        extra["mnist70kx784_qmeans_lloyd_ms_per_step"] = round(
            1e3 * getattr(qm, "fit_phase_s_", {}).get("lloyd_s", float("nan")) / max(qm.n_iter_, 1), 4)
        # the reference default distance mode (IPE) at this shape: d_pad 896
        # runs the certified fp16 screen with its values pass (ops.kmeans.
        # Ipe16.gv), the fp32 IPE kernel only for the screen's dense rows
        t, qm = wall(lambda: QMeans(n_clusters=k, delta=a.delta, true_distance_estimate=True,
                                    intermediate_error=True, true_tomography=False, n_init=1,
                                    max_iter=20, tol=0.0, random_state=0, device=dev).fit(sa))
        extra["mnist70kx784_qmeans_ipe_fit_s"] = t
        extra["mnist70kx784_qmeans_ipe_lloyd_ms_per_step"] = round(
            1e3 * getattr(qm, "fit_phase_s_", {}).get("lloyd_s", float("nan")) / max(qm.n_iter_, 1), 4)
        from sq_learn_amd.models.cluster._lloyd import LloydEngine
        eng = LloydEngine(X, k, delta=a.delta, true_distance_estimate=True,
                          intermediate_error=True, true_tomography=False, seed=a.seed, comm=comm,
                          row_offset=s0)
        eng.set_centers(torch.as_tensor(qm.cluster_centers_, dtype=torch.float32, device=dev))
        for _ in range(3):
            eng.step()[1].tolist()
        i16 = getattr(eng, "_ipe16", None)
        extra["mnist70kx784_ipe16_screen"] = bool(i16 is not None and i16.gv)
        extra["mnist70kx784_ipe16_dense_row_frac"] = (
            round(i16.last_dense / max(X.shape[0], 1), 6) if i16 is not None else None)
        del eng
        del X, sa
        torch.cuda.empty_cache()
        if comm.world_size == 1:
            # the reference's driver (MnistTrial.py): qPCA(61) -> quantum
            # representation (tomography, error 0.8) -> 7-NN, 10-fold CV
            sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                            "examples"))
            from mnist_pipeline import run as mnist_run
            r = mnist_run(device=str(dev), classic=False)
            for kk in ("qpca_fit_s", "transform_s", "cv_s", "total_s", "accuracy"):
                extra[f"mnist_pipeline_{kk}"] = round(r[kk], 4)
            torch.cuda.empty_cache()
    except Exception as e:
        extra["mnist_error"] = repr(e)[:200]


def _pipeline_extra(extra, a, comm, dev):
    """BASELINE config 5: qPCA -> q-means on 50M x 128 (bf16, low rank + tail)
    with failure-probability resampling (benchmarks/pipeline_bench.py
    run_pipeline): per-stage seconds."""
    try:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "benchmarks"))
        from pipeline_bench import run_pipeline
        res = run_pipeline(comm, dev, a.pipeline_rows)
        tag = f"pipeline_{a.pipeline_rows // 1_000_000}Mx128"
        for kk, v in res.items():
            extra[f"{tag}_{kk}"] = round(v, 4) if isinstance(v, float) else v
        torch.cuda.empty_cache()
    except Exception as e:
        extra["pipeline_error"] = repr(e)[:200]


def _fit_extra(extra, a, sa, comm, dev, init, ipe=False, name=None, n_init=1):
    """Wall-clock of a whole QMeans.fit (prelude: eta, mu(A), condition
    number; centring; initialisation; ``fit_iters`` Lloyd iterations with
    tol = 0; final E-step) on the same matrix (BASELINE: fit wall-clock at a
    fixed max_iter).  ``ipe``: the reference's DEFAULT distance mode
    (``true_distance_estimate=True``, ``_dmeans.py:1016-1039``)."""
    name = name or f"fit_wall_s_{init.replace('|', 'par').replace('+', 'pp')}_{a.fit_iters}it"
    try:
        from sq_learn_amd.models.cluster import QMeans
        kw = dict(n_clusters=a.k, delta=a.delta, true_distance_estimate=bool(ipe),
                  intermediate_error=True, true_tomography=False, init=init, n_init=n_init,
                  max_iter=a.fit_iters, tol=0.0, random_state=a.seed, device=dev,
                  gemm_precision=a.dtype)
        _sync(dev)
        comm.barrier()
        t0 = time.perf_counter()
        est = QMeans(**kw).fit(sa)
        _sync(dev)
        comm.barrier()
        extra[name] = _max_over_ranks(comm, dev, time.perf_counter() - t0)
        extra[name + "_n_iter"] = int(est.n_iter_)
        extra[name + "_inertia"] = float(est.inertia_)
        for ph, v in getattr(est, "fit_phase_s_", {}).items():
            extra[name + "_" + ph] = round(v, 4)
    except Exception as e:
        extra[name + "_error"] = repr(e)[:200]


def main(argv=None):
    a = parse(argv)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return _spawn(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")

    from sq_learn_amd.parallel.comm import init_distributed, shard_bounds, Comm
    from sq_learn_amd.utils.datasets import make_blobs_device
    from sq_learn_amd.models.cluster._lloyd import LloydEngine
    from sq_learn_amd.models._data import Data, gather_rows

    gpu = a.device == "cuda"
    comm = init_distributed(backend=None if gpu else "gloo") if world > 1 else Comm(None)
    rank = comm.rank
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if gpu:
        dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32

    start, stop = shard_bounds(a.n, rank, comm.world_size)
    X, _ = make_blobs_device(a.n, a.d, centers=a.blobs, cluster_std=1.0, seed=a.seed, device=dev,
                             dtype=dtype, row_range=(start, stop))
    data = Data(X, a.n, start, comm, "sharded")
    rs = np.random.RandomState(a.seed)
    init_idx = rs.choice(a.n, a.k, replace=False)
    C0 = gather_rows(data, init_idx)

    eng = LloydEngine(X, a.k, delta=a.delta, true_distance_estimate=False, intermediate_error=True,
                      true_tomography=False, seed=a.seed, comm=comm, row_offset=start,
                      gemm_precision=a.dtype)
    eng.set_centers(C0)

    def step():
        labels, sc = eng.step()
        return sc.tolist()          # convergence read-back, as in fit()

    # as in QMeans.fit: the next iteration's E-step is enqueued before the
    # read-back (LloydEngine.pipeline)
    eng.pipeline = True

    for _ in range(a.warmup):
        step()
    comm.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    last = None
    for _ in range(a.steps):
        last = step()
    _sync(dev)
    comm.barrier()
    elapsed = _max_over_ranks(comm, dev, time.perf_counter() - t0)
    ms_per_step = elapsed / a.steps * 1e3
    value = a.n * a.steps / elapsed

    extra = {"inertia_last": last[0] if last else None, "rows_per_gpu": stop - start,
             "delta": a.delta, "k": a.k, "d": a.d,
             "precision": ("certified fp64 delta-band labels (fp16 MFMA filter + fp64 re-check)"
                           if a.dtype == "fp32" else "bf16 operands (approximate band edges)")}
    eng.pipeline = False
    eng.drop_pending()
    if eng.fast and gpu:
        cnt = eng.buf.counts.tolist()
        extra["overflow_rows_last"], extra["dense_rows_last"] = int(cnt[0]), int(cnt[1])
        extra["multi_rows_last"] = int(cnt[2])   # rows re-checked over their candidate sets
        if len(cnt) > 5 and getattr(eng, "mrec", None) is not None:
            # multi rows whose gap record was moved by the shifts (fp16 row)
            # and, of those, resolved without the fp32 screen
            extra["gap_rows_last"], extra["gap_resolved_last"] = int(cnt[5]), int(cnt[4])
        xf = getattr(eng.buf, "exact_flag", None)
        if xf is not None and cnt[2] > 0:   # of which the fp32 screen left to the fp64 pass
            extra["multi_fp64_rows_last"] = int((xf[:int(cnt[2])] != 0).sum())
        # per-phase ms of 3 more (untimed) iterations, CUDA events per phase
        ph = {}
        for _ in range(3):
            for kk, v in eng.step_phases().items():
                ph[kk] = ph.get(kk, 0.0) + v / 3.0
        extra["phase_ms"] = {kk: round(v, 4) for kk, v in ph.items()}
        # the regimes behind the steady-state number: the same iteration with
        # the Hamerly pruning off (every row through the filter sweep) and the
        # first iteration after (re)setting the centres (no valid bounds, the
        # full incremental M-step start)
        if getattr(eng, "bounds", False):
            eng.bounds = False
            step()
            _sync(dev)
            comm.barrier()
            t0 = time.perf_counter()
            for _ in range(3):
                step()
            _sync(dev)
            comm.barrier()
            extra["unpruned_ms_per_step"] = _max_over_ranks(
                comm, dev, (time.perf_counter() - t0) / 3 * 1e3)
            eng.bounds = True
        eng.set_centers(C0)
        _sync(dev)
        comm.barrier()
        t0 = time.perf_counter()
        step()
        _sync(dev)
        comm.barrier()
        extra["first_iter_ms"] = _max_over_ranks(comm, dev, (time.perf_counter() - t0) * 1e3)

    del eng
    if gpu:
        torch.cuda.empty_cache()
    if gpu and comm.world_size == 1 and a.n >= 8 * 4096 and not a.no_share8:
        _share8_extra(extra, a, X, comm, dev, C0)
    if a.ipe_steps > 0 and gpu:
        _ipe_extra(extra, a, X, comm, dev, start, C0)
    if gpu and not a.no_hard:
        _hard_extra(extra, a, comm, dev)
    if gpu and not a.no_mnist:
        _mnist_extra(extra, a, comm, dev)
    from sq_learn_amd.parallel.sharding import ShardedArray
    sa = ShardedArray(X, a.n, start, comm)
    if not a.no_fit:
        for init in ("random", "k-means||", "k-means++"):
            _fit_extra(extra, a, sa, comm, dev, init)
        if gpu and a.ipe_steps > 0:
            # the reference defaults: k-means++ init + IPE ("l2-sampled")
            # distances, n_init = 1, fit_iters iterations, tol = 0
            _fit_extra(extra, a, sa, comm, dev, "k-means++", ipe=True,
                       name="fit_wall_s_refdefault")
            # ... at the reference's default n_init = 10 (best of 10 restarts,
            # _dmeans.py:1285-1306)
            _fit_extra(extra, a, sa, comm, dev, "k-means++", ipe=True,
                       name="fit_wall_s_refdefault_ninit10", n_init=10)
    if not a.no_qpca and gpu:
        # qPCA wall-clock (BASELINE metric part 2) on the same 10M x 256 matrix
        _qpca_extra(extra, "qpca_10Mx256_full_fit_s", sa, comm, dev, "full")
        _qpca_extra(extra, "qpca_10Mx256_full_truetomo_fit_s", sa, comm, dev, "full",
                    true_tomography=True)
        _qpca_extra(extra, "qpca_10Mx256_randomized_fit_s", sa, comm, dev, "randomized")
        _qpca_extra(extra, "qpca_10Mx256_randomized_truetomo_fit_s", sa, comm, dev, "randomized",
                    true_tomography=True)
        del X, sa
        torch.cuda.empty_cache()
        # BASELINE config 2: qPCA 1M x 512 bf16 (low-rank + tail), full and randomized
        from sq_learn_amd.utils.datasets import make_low_rank_device
        n2, d2 = 1_000_000, 512
        s2, e2 = shard_bounds(n2, rank, comm.world_size)
        X2 = make_low_rank_device(n2, d2, effective_rank=32, tail_strength=0.3, seed=a.seed,
                                  device=dev, dtype=torch.bfloat16, row_range=(s2, e2))
        sa2 = ShardedArray(X2, n2, s2, comm)
        _qpca_extra(extra, "qpca_1Mx512_full_fit_s", sa2, comm, dev, "full")
        _qpca_extra(extra, "qpca_1Mx512_randomized_fit_s", sa2, comm, dev, "randomized")
        _qpca_extra(extra, "qpca_1Mx512_randomized_truetomo_fit_s", sa2, comm, dev, "randomized",
                    true_tomography=True)
        del X2, sa2
        torch.cuda.empty_cache()
    if gpu and not a.no_pipeline:
        _pipeline_extra(extra, a, comm, dev)

    if rank == 0:
        out = {
            "metric": "q-means fit samples/sec (Lloyd samples*iterations/s, delta-means + tomography noise)",
            "value": value,
            "unit": "samples*iter/s",
            "n_gpus": comm.world_size,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": value / BASELINE_SAMPLES_PER_S,
            "dtype": a.dtype,
            "data": f"synthetic (on-device make_blobs, Philox-keyed, {a.blobs} blobs)",
            "config": {"model": f"q-means k={a.k} delta={a.delta} ({a.n} x {a.d} synthetic)",
                       "global_batch": a.n, "seq_len": a.d,
                       "parallelism": f"dp{comm.world_size}"},
            "extra": extra,
        }
        if "ipe_samples_iter_per_s" in extra:
            # the reference's DEFAULT distance mode (true_distance_estimate=True)
            out["co_headline"] = {
                "metric": "q-means IPE (true_distance_estimate) samples*iter/s",
                "value": extra["ipe_samples_iter_per_s"], "unit": "samples*iter/s",
                "ms_per_step": extra.get("ipe_ms_per_step")}
        print(json.dumps(out), flush=True)
    if comm.distributed:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
