"""Multi-rank rehearsal of the GPU fast path: the
row-sharded fit at world 2 and 3 - every rank a FRESH child process of
``torch.distributed.run``, all ranks on cuda:0, gloo collectives
(SQ_DIST_BACKEND=gloo) - against the single-process fit of the same data.

The analogue of the reference's thread-count invariance test
(``sklearn/cluster/tests/test_k_means.py:840-852``).  What is pinned:

* q-means (certified fp16-filter + fp64 re-check E-step, Hamerly pruning,
  incremental fixed-point M-step) with k-means++, random and k-means||
  initialisation: labels and centroids BIT-IDENTICAL (fixed-point centroid
  sums, draws keyed by global row), same iteration count; the inertia is an
  fp64 sum whose association follows the shard boundaries (<= 1e-12 rel);
* classical KMeans with empty-cluster relocation (per-shard top-e +
  all-gather): bit-identical labels and centroids;
* q-means with the reference's default IPE distances (fused kernel, hazard
  streams keyed by global row, previous-label hints) and with wide rows
  (d = 300 / 784 through the certified filter, d = 1100 through the exact
  fp64 rows kernel under k-means||): bit-identical labels and centroids;
* CholeskyQR2 sigma_min on the fp64-MFMA Gram, centred and not, and the
  full and randomized qPCA spectra (fp64 end to end): fp64 sums over
  shards, <= 1e-9 rel;
* tomography of the row-sharded left singular vectors: Gaussian noise
  keyed by (vector, GLOBAL column) - the single-process draw; true
  tomography (rank-split multinomial) within its delta guarantee.
"""
import json
import os
import socket
import subprocess
import sys
import tempfile

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res.json")
        env = dict(os.environ)
        env["SQ_DIST_BACKEND"] = "gloo"
        env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
        env.setdefault("OMP_NUM_THREADS", "2")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
               f"--master-port={_free_port()}", os.path.join(HERE, "_dist_gpu_worker.py"), out]
        p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=200)
        assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-6000:])
        with open(out) as f:
            return json.load(f)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gpu_fast_path_matches_single_process(world):
    r = _run(world)
    assert r["world"] == world
    res = r["results"]
    print(json.dumps(res, indent=1))
    for init in ("k-means++", "random", "k-means||"):
        q = res["qmeans_" + init]
        # the certified, pruned, incremental engine is what ran
        for cfg in (q["cfg_ref"], q["cfg_got"]):
            assert cfg["fast"] and cfg["certified"] and cfg["bounds"] and cfg["incremental"], cfg
        assert q["labels_equal"], (init, q)
        assert q["centers_bitwise"], (init, q)
        assert q["n_iter"][0] == q["n_iter"][1], (init, q)
        assert q["inertia_rel"] <= 1e-12, (init, q)
        assert q["cond_rel"] <= 1e-10 and q["muA_rel"] <= 1e-12, (init, q)
    q = res["qmeans_ipe"]
    assert q["labels_equal"] and q["centers_bitwise"], q
    assert q["n_iter"][0] == q["n_iter"][1] and q["inertia_rel"] <= 1e-12, q
    for d_w, fast in ((300, True), (784, True), (1100, False)):
        q = res[f"qmeans_d{d_w}"]
        assert q["cfg_got"]["fast"] == fast and q["cfg_ref"]["fast"] == fast, (d_w, q)
        assert q["labels_equal"] and q["centers_bitwise"], (d_w, q)
        assert q["n_iter"][0] == q["n_iter"][1] and q["inertia_rel"] <= 1e-12, (d_w, q)
    km = res["kmeans_relocate"]
    assert km["cfg_got"]["fast"] and km["cfg_got"]["relocate"], km
    assert km["distinct"] == 5, km      # both far centres were relocated
    assert km["labels_equal"] and km["centers_bitwise"], km
    assert km["n_iter"][0] == km["n_iter"][1] and km["inertia_rel"] <= 1e-12, km
    sm = res["sigma_min"]
    assert sm["plain_rel"] <= 1e-10 and sm["centred_rel"] <= 1e-10, sm
    for key in ("qpca_full_gauss", "qpca_full_true", "qpca_randomized_gauss",
                "qpca_randomized_true"):
        q = res[key]
        # both paths are fp64 end to end (full: the fp64-MFMA Gram +
        # CholeskyQR2; randomized: fp64 xw / xtx power iterations and
        # CholeskyQR2 on tsgemm64): the shard sums differ only in fp64
        # summation order
        assert q["sv_rel"] <= 1e-9, (key, q)
        assert q["comp_absdiff"] <= 1e-6, (key, q)
        assert q["left_shape"] == [4, 6007], (key, q)
        assert max(q["left_err"]) <= 0.3 + 1e-9, (key, q)     # the delta guarantee
        assert q["muA_rel"] <= 1e-10, (key, q)
        if key.endswith("gauss"):
            # same Philox elements as the unsharded draw
            assert q["left_vs_ref"] <= (1e-5 if "full" in key else 1e-4), (key, q)
