"""Task parallelism: independent fits (cross-validation folds, search
candidates, one-vs-rest / multi-output members, ensemble members) fanned
out over worker threads and the node's GPUs.

The reference hands such tasks to joblib (``Parallel(n_jobs)(delayed(f)(...)
for ...)``, e.g. ``model_selection/_validation.py:267``,
``_search.py:795``), usually to worker processes.  Here a task is a fit of
an estimator whose heavy work is either HIP kernels or the host-native
library (ctypes calls, GIL released), so THREADS suffice and keep every
task in the process that owns the GPUs - no pickling of data or models, no
process re-exec on a GPU host.  With more than one visible GPU and a
GPU-resolving config, task ``i`` runs pinned to GPU ``i mod n_gpus``
(``torch.cuda.device`` + config ``device='cuda:<i>'`` for that task only):
one fold or candidate per GPU, the 288 GB of each HBM holding its own
copy of the training split.  Results come back in task order; the first
failing task's exception (in task order) is re-raised.

    from sq_learn_amd.parallel.tasks import Parallel
    from sq_learn_amd.utils.fixes import delayed
    scores = Parallel(n_jobs=4)(delayed(fit_and_score)(clone(est), f) for f in folds)
"""

import os
from concurrent.futures import ThreadPoolExecutor

from .._config import get_config
from ..utils.fixes import _FuncWrapper


def effective_n_jobs(n_jobs=None):
    """joblib's convention: None -> 1, -1 -> all CPUs, -k -> CPUs + 1 - k."""
    if n_jobs is None or n_jobs == 0:
        return 1
    n_jobs = int(n_jobs)
    if n_jobs < 0:
        return max(1, (os.cpu_count() or 1) + 1 + n_jobs)
    return n_jobs


def _gpu_slots(devices):
    """GPU indices the tasks rotate over (empty: no pinning)."""
    if devices is not None:
        return list(devices)
    dev = str(get_config().get("device", "auto"))
    if dev not in ("auto", "cuda", "gpu", "hip"):
        return []          # an explicit device (cpu / cuda:<i>) is left alone
    try:
        import torch
        n = torch.cuda.device_count() if torch.cuda.is_available() else 0
    except Exception:
        n = 0
    return list(range(n)) if n > 1 else []


class Parallel:
    """Run ``(function, args, kwargs)`` tasks on ``n_jobs`` threads, task i
    pinned to GPU ``devices[i % len(devices)]`` when several GPUs are in
    play (``devices=None``: every visible GPU when the config resolves to
    the GPU; ``devices=()``: no pinning)."""

    def __init__(self, n_jobs=None, *, devices=None, verbose=0, pre_dispatch=None,
                 backend=None, prefer=None, require=None):
        self.n_jobs = n_jobs
        self.devices = devices
        self.verbose = verbose

    @staticmethod
    def _run(task, gpu):
        fn, args, kwargs = task
        if gpu is None:
            return fn(*args, **kwargs)
        import torch
        with torch.cuda.device(gpu):
            if isinstance(fn, _FuncWrapper):
                return fn.call_with({"device": f"cuda:{gpu}"}, *args, **kwargs)
            from .._config import config_context
            with config_context(device=f"cuda:{gpu}"):
                return fn(*args, **kwargs)

    def __call__(self, iterable):
        tasks = list(iterable)
        n = min(effective_n_jobs(self.n_jobs), max(len(tasks), 1))
        if n <= 1:
            return [self._run(t, None) for t in tasks]
        slots = _gpu_slots(self.devices)
        gpus = [slots[i % len(slots)] if slots else None for i in range(len(tasks))]
        with ThreadPoolExecutor(max_workers=n, thread_name_prefix="sq-task") as ex:
            futures = [ex.submit(self._run, t, g) for t, g in zip(tasks, gpus)]
            return [f.result() for f in futures]


__all__ = ["Parallel", "effective_n_jobs"]
