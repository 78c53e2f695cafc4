"""Row-sharded data parallelism on CPU with gloo (world_size 2 and 3): a sharded
fit must reproduce the single-process fit (counter-based RNG keyed by global
row -> identical draws; SURVEY.md §4 implication 3, the analogue of the
reference's thread-count invariance test test_k_means.py:840-852)."""
import os
import socket
import tempfile
import traceback

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir, case):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                init_method=f"tcp://127.0.0.1:{port}")
        import warnings
        warnings.simplefilter("ignore")
        from sq_learn_amd.parallel import Comm, shard_rows
        from sq_learn_amd.utils.datasets import make_blobs
        comm = Comm(dist.group.WORLD)
        X, y = make_blobs(900, 6, centers=5, cluster_std=1.0, random_state=7)
        sa = shard_rows(X, comm=comm)
        if case == "qmeans":
            from sq_learn_amd.models.cluster import QMeans
            for init in ("random", "k-means++"):
                kw = dict(n_clusters=5, delta=0.8, true_distance_estimate=False,
                          intermediate_error=True, true_tomography=False, random_state=3,
                          n_init=2, init=init, device="cpu")
                ref = QMeans(**kw).fit(X)
                got = QMeans(**kw).fit(sa)
                np.testing.assert_allclose(got.cluster_centers_, ref.cluster_centers_, rtol=1e-9, atol=1e-9)
                loc = torch.as_tensor(got.labels_.astype(np.int64))
                full = torch.cat(comm.all_gather_varlen(loc)).numpy()
                np.testing.assert_array_equal(full, ref.labels_)
                assert abs(got.inertia_ - ref.inertia_) <= 1e-9 * ref.inertia_
                assert got.n_iter_ == ref.n_iter_
                assert abs(got.muA - ref.muA) < 1e-9 * ref.muA
                assert abs(got.condition_number - ref.condition_number) < 1e-6 * ref.condition_number
        elif case == "ipe":
            from sq_learn_amd.models.cluster import QMeans
            Xs = X[:120]
            sa2 = shard_rows(Xs, comm=comm)
            kw = dict(n_clusters=3, delta=0.3, true_distance_estimate=True, random_state=1,
                      n_init=1, max_iter=3, init="random", device="cpu", compute_prelude=False)
            ref = QMeans(**kw).fit(Xs)
            got = QMeans(**kw).fit(sa2)
            loc = torch.as_tensor(got.labels_.astype(np.int64))
            full = torch.cat(comm.all_gather_varlen(loc)).numpy()
            np.testing.assert_array_equal(full, ref.labels_)
        elif case == "kmeans":
            from sq_learn_amd.models.cluster import KMeans
            ref = KMeans(n_clusters=5, random_state=0, n_init=1, device="cpu").fit(X)
            got = KMeans(n_clusters=5, random_state=0, n_init=1, device="cpu").fit(sa)
            np.testing.assert_allclose(got.cluster_centers_, ref.cluster_centers_, rtol=1e-9)
            assert abs(got.inertia_ - ref.inertia_) <= 1e-9 * ref.inertia_
        elif case == "pca":
            from sq_learn_amd.models.decomposition import PCA, QPCA
            from sq_learn_amd.models.decomposition._svd import full_svd
            from sq_learn_amd.models._data import as_data, global_mean_var
            rng = np.random.RandomState(0)
            Z = rng.randn(600, 8) @ rng.randn(8, 8) + 3.0
            sz = shard_rows(Z, comm=comm)
            # Gram path (forced) on shards vs exact SVD of the full matrix
            d = as_data(sz)
            mean, _ = global_mean_var(d)
            res = full_svd(d, mean, 4, method="gram")
            S = np.linalg.svd(Z - Z.mean(0), compute_uv=False)
            np.testing.assert_allclose(res.S, S, rtol=1e-8)
            U = torch.cat(comm.all_gather_varlen(res.U_local)).numpy()
            Uf, Sf, Vf = np.linalg.svd(Z - Z.mean(0), full_matrices=False)
            np.testing.assert_allclose(np.abs(U), np.abs(Uf[:, :4]), atol=1e-8)
            # randomized path
            p = PCA(n_components=3, svd_solver="randomized", random_state=0, device="cpu").fit(sz)
            np.testing.assert_allclose(p.singular_values_, S[:3], rtol=1e-6)
            q = QPCA(n_components=3, svd_solver="full", random_state=0, device="cpu").fit(
                sz, eps=0.01, theta_major=1e-3, delta=0.1, estimate_all=True, true_tomography=False)
            qr = QPCA(n_components=3, svd_solver="full", random_state=0, device="cpu").fit(
                Z, eps=0.01, theta_major=1e-3, delta=0.1, estimate_all=True, true_tomography=False)
            np.testing.assert_allclose(q.singular_values_, qr.singular_values_, rtol=1e-8)
            np.testing.assert_allclose(q.estimate_s_values, qr.estimate_s_values, rtol=1e-12)
            assert abs(q.muA - qr.muA) < 1e-9 * qr.muA
            # Gaussian tomography of the row-sharded left vectors draws the
            # Philox element (vector, GLOBAL row): the unsharded tensor fit's
            # noise, element for element
            qt = QPCA(n_components=3, svd_solver="full", random_state=0, device="cpu").fit(
                torch.as_tensor(Z), eps=0.01, theta_major=1e-3, delta=0.1, estimate_all=True,
                true_tomography=False)
            left = torch.as_tensor(np.asarray(q.estimate_left_sv))
            fullL = torch.cat(comm.all_gather_varlen(left.T.contiguous())).T.numpy()
            np.testing.assert_allclose(np.abs(fullL), np.abs(np.asarray(qt.estimate_left_sv)),
                                       atol=1e-10)
        elif case == "relocate":
            # empty-cluster relocation across shards: per-shard top-e + all-gather
            from sq_learn_amd.models.cluster import KMeans
            rng = np.random.RandomState(0)
            Xr = np.vstack([rng.randn(300, 2), rng.randn(300, 2) + [8, 8], [[30.0, -30.0]],
                            [[-25.0, 20.0]]])
            init = np.array([[0.0, 0.0], [8.0, 8.0], [500.0, 500.0], [-500.0, 500.0]])
            ref = KMeans(n_clusters=4, init=init, n_init=1, device="cpu").fit(Xr)
            got = KMeans(n_clusters=4, init=init, n_init=1, device="cpu").fit(
                shard_rows(Xr, comm=comm))
            np.testing.assert_allclose(got.cluster_centers_, ref.cluster_centers_, atol=1e-9)
        elif case == "tomography":
            # long-vector tomography of row-sharded vectors (qPCA left singular
            # vectors): same law as the single-process draw, stopping rule
            # evaluated on the GLOBAL error
            from scipy import stats
            from sq_learn_amd.parallel.comm import shard_bounds
            from sq_learn_amd.quantum.device import tomography_long
            from sq_learn_amd.runtime.rng import RngKey
            rng = np.random.RandomState(3)
            n = 1500
            A = torch.tensor(rng.standard_normal((2, n)))
            Vn = (A / A.norm(dim=1, keepdim=True)).numpy()
            s0, s1 = shard_bounds(n, comm.rank, comm.world_size)
            e_sh, e_one = [], []
            for rep in range(25):
                key = RngKey(rep, "tomography", 1)
                loc = tomography_long(A[:, s0:s1], None, key, N=60000, incremental_measure=False,
                                      comm=comm, n_global=n)
                full = torch.cat(comm.all_gather_varlen(loc.T.contiguous())).T.numpy()
                e_sh += list(np.linalg.norm(full - Vn, axis=1))
                one = tomography_long(A, None, RngKey(rep, "tomography", 2), N=60000,
                                      incremental_measure=False).numpy()
                e_one += list(np.linalg.norm(one - Vn, axis=1))
            assert stats.ks_2samp(e_sh, e_one).pvalue > 1e-4
            for rep in range(3):
                loc = tomography_long(A[:, s0:s1], 0.4, RngKey(rep, "tomography", 3), comm=comm,
                                      n_global=n)
                full = torch.cat(comm.all_gather_varlen(loc.T.contiguous())).T.numpy()
                assert np.all(np.linalg.norm(full - Vn, axis=1) <= 0.4)
            # qPCA randomized path with the quantum extras on sharded data
            from sq_learn_amd.models.decomposition import QPCA
            Z = rng.randn(1200, 10) @ rng.randn(10, 10)
            sz = shard_rows(Z, comm=comm)
            q = QPCA(n_components=3, svd_solver="randomized", random_state=0, device="cpu",
                     quantum_truncated=True).fit(sz, eps=1e-3, theta_major=1e-6, delta=0.3,
                                                 estimate_all=True, true_tomography=True)
            left = torch.as_tensor(q.estimate_left_sv)
            fullL = torch.cat(comm.all_gather_varlen(left.T.contiguous())).T.numpy()
            Ut = torch.cat(comm.all_gather_varlen(torch.as_tensor(q.left_sv).T.contiguous())).T.numpy()
            assert fullL.shape == (3, 1200)
            assert np.all(np.linalg.norm(fullL - Ut, axis=1) <= 0.3)   # N = 36 n ln n / delta^2 shots
            assert np.all(np.abs(np.linalg.norm(fullL, axis=1) - 1) < 0.2)
        elif case == "resume":
            # sharded fit with failures, crashed mid-fit on every rank, then
            # resumed from the per-rank checkpoint: identical to an
            # uninterrupted single-process fit
            from sq_learn_amd.models.cluster import QMeans
            from sq_learn_amd.models.cluster._lloyd import LloydEngine
            kw = dict(n_clusters=5, delta=0.5, true_distance_estimate=False, random_state=2,
                      n_init=2, max_iter=10, tol=0.0, device="cpu", failure_prob=0.1,
                      failure_policy="resample", failure_max_attempts=2, checkpoint_every=3)
            ref = QMeans(**kw).fit(X)
            ck = os.path.join(outdir, "ck")
            orig = LloydEngine.step
            calls = {"n": 0}

            def crashing(self):
                calls["n"] += 1
                if calls["n"] > 13:
                    raise KeyboardInterrupt
                return orig(self)
            LloydEngine.step = crashing
            try:
                QMeans(checkpoint_dir=ck, **kw).fit(sa)
                raise AssertionError("expected the simulated crash")
            except KeyboardInterrupt:
                pass
            finally:
                LloydEngine.step = orig
            got = QMeans(checkpoint_dir=ck, **kw).fit(sa)
            assert got.resumed_from_ == (1, 3)
            np.testing.assert_allclose(got.cluster_centers_, ref.cluster_centers_, rtol=1e-9,
                                       atol=1e-9)
            loc = torch.as_tensor(got.labels_.astype(np.int64))
            full = torch.cat(comm.all_gather_varlen(loc)).numpy()
            np.testing.assert_array_equal(full, ref.labels_)
            assert got.n_failed_rows_ > 0
        with open(os.path.join(outdir, f"ok{rank}"), "w") as f:
            f.write("ok")
    except Exception:
        with open(os.path.join(outdir, f"err{rank}"), "w") as f:
            f.write(traceback.format_exc())
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("case,world", [("qmeans", 2), ("qmeans", 3), ("kmeans", 2), ("pca", 2),
                                        ("ipe", 2), ("resume", 2), ("tomography", 2),
                                        ("relocate", 3)])
def test_sharded_matches_single_process(case, world):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d, case), nprocs=world, join=True)
        errs = [open(os.path.join(d, f)).read() for f in os.listdir(d) if f.startswith("err")]
        assert not errs, errs[0]
        assert len([f for f in os.listdir(d) if f.startswith("ok")]) == world
