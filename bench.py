#!/usr/bin/env python
"""Headline benchmark: q-means Lloyd-iteration throughput on 10M x 256,
k = 1024, row-sharded over N MI355X GPUs (BASELINE.json config 3), plus the
qPCA wall-clock on the same matrix (config 2/metric part 2) as an extra.

One step = one full q-means iteration of the reference's delta-means path
(``_dmeans.py:534-671`` with ``delta > 0``, ``true_distance_estimate=False``,
``intermediate_error=True``, Gaussian tomography): fused MFMA distance +
delta-band E-step, segmented centroid reduce, one packed RCCL all-reduce,
centroid finalise with truncated-normal tomography noise, convergence
scalars read back to the host.  Nothing is skipped inside the timed region.

Strong scaling: the 10M rows are split across ranks (each rank generates its
own shard in HBM from the global Philox stream - same dataset for every N).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N --steps K --warmup W
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

BASELINE_SAMPLES_PER_S = 3.7e3   # reference q-means iteration, 8-core Xeon


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--delta", type=float, default=0.5)
    ap.add_argument("--blobs", type=int, default=1024)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-qpca", action="store_true")
    ap.add_argument("--seed", type=int, default=2024)
    return ap.parse_args()


def _qpca_extra(extra, name, sa, comm, dev, solver, n_components=16):
    """Wall-clock of a QPCA fit with the quantum extras of ``_qPCA.py:357-465``
    (CPE singular values, Theorem 11 top-k extraction + Gaussian tomography);
    one untimed warm fit first.  Never breaks the headline line."""
    try:
        from sq_learn_amd.models.decomposition import QPCA
        q = QPCA(n_components=n_components, svd_solver=solver, random_state=0, device=dev).fit(sa)
        theta = 0.5 * float(q.singular_values_[n_components - 1])
        torch.cuda.synchronize()
        comm.barrier()
        t0 = time.perf_counter()
        q = QPCA(n_components=n_components, svd_solver=solver, random_state=0, device=dev)
        q.fit(sa, eps=1e-3, theta_major=theta, delta=0.1, estimate_all=True,
              true_tomography=False)
        torch.cuda.synchronize()
        comm.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        comm.all_reduce_(el, op="max")
        extra[name] = float(el.item())
    except Exception as e:  # qPCA must not break the headline line
        extra[name + "_error"] = repr(e)[:200]


def main():
    a = parse()
    from sq_learn_amd.parallel.comm import init_distributed, shard_bounds, Comm
    from sq_learn_amd.utils.datasets import make_blobs_device
    from sq_learn_amd.models.cluster._lloyd import LloydEngine
    from sq_learn_amd.models._data import Data, gather_rows

    world = int(os.environ.get("WORLD_SIZE", "1"))
    comm = init_distributed() if world > 1 else Comm(None)
    rank = comm.rank
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
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
                      gemm_precision="bf16")
    eng.set_centers(C0)

    def step():
        labels, sc = eng.step()
        return sc.tolist()          # convergence read-back, as in fit()

    for _ in range(a.warmup):
        step()
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = None
    for _ in range(a.steps):
        last = step()
    torch.cuda.synchronize()
    comm.barrier()
    t1 = time.perf_counter()
    el = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    comm.all_reduce_(el, op="max")
    elapsed = float(el.item())
    ms_per_step = elapsed / a.steps * 1e3
    value = a.n * a.steps / elapsed
    ovf = int(last[2]) if last else 0

    extra = {"inertia_last": last[0] if last else None, "overflow_rows_last": ovf,
             "rows_per_gpu": stop - start, "delta": a.delta, "k": a.k, "d": a.d}
    if not a.no_qpca:
        del eng
        torch.cuda.empty_cache()
        from sq_learn_amd.parallel.sharding import ShardedArray
        # qPCA wall-clock (BASELINE metric part 2) on the same 10M x 256 matrix
        _qpca_extra(extra, "qpca_10Mx256_full_fit_s", ShardedArray(X, a.n, start, comm), comm,
                    dev, "full")
        del X
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
            "data": "synthetic (on-device make_blobs, Philox-keyed, 1024 blobs)",
            "config": {"model": f"q-means k={a.k} delta={a.delta} (10M x 256 synthetic)",
                       "global_batch": a.n, "seq_len": a.d,
                       "parallelism": f"dp{comm.world_size}"},
            "extra": extra,
        }
        print(json.dumps(out), flush=True)
    if comm.distributed:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
