"""bench.py contract on CPU: ``--gpus 2`` without torchrun re-launches itself
under torch.distributed.run (2 gloo ranks) and prints one JSON line with the
driver's keys; ``--gpus`` must equal WORLD_SIZE."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--device", "cpu", "--rows", "4096", "--features", "16", "--k", "8", "--blobs", "8",
         "--steps", "2", "--warmup", "1", "--no-qpca", "--fit-iters", "3"]


def _run(args, env_extra=None, timeout=300):
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT,
                          env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                          timeout=timeout)


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus", [1, 2])
def test_bench_entry_runs_n_ranks(gpus):
    r = _run(["--gpus", str(gpus)] + SMALL)
    assert r.returncode == 0, r.stderr[-3000:]
    o = _line(r.stdout)
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in o
    assert o["n_gpus"] == gpus and o["steps"] == 2 and o["warmup"] == 1
    assert o["config"]["parallelism"] == f"dp{gpus}" and o["dtype"] == "fp32"
    assert o["value"] > 0 and o["extra"]["rows_per_gpu"] == 4096 // gpus
    fit = [k for k in o["extra"] if k.startswith("fit_wall_s") and not k.endswith("_error")
           and not k.endswith("_n_iter")]
    assert fit, o["extra"]


def test_bench_rejects_world_size_mismatch():
    r = _run(["--gpus", "2"] + SMALL, env_extra={"WORLD_SIZE": "1"})
    assert r.returncode != 0
    assert "WORLD_SIZE" in (r.stderr + r.stdout)
