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

import contextlib
import os
import threading
from concurrent.futures import ThreadPoolExecutor

from .._config import get_config
from ..utils.fixes import _FuncWrapper

# ------------------------------------------------------------- backends
# A backend turns a list of task thunks into results.  'threading' (the
# default: worker threads, task i pinned to GPU i mod n_gpus) and
# 'sequential' are built in; joblib's process backends ('loky',
# 'multiprocessing') map to 'threading' - the heavy work of a task is HIP
# kernels or the ctypes host library with the GIL released, and a process
# backend would re-exec workers on a GPU host.  register_parallel_backend adds
# a backend from a factory returning a concurrent.futures-style executor
# (``submit`` + ``shutdown``), e.g. a ProcessPoolExecutor for pure-python
# CPU tasks.
_BACKENDS = {}
_DEFAULT = {"name": "threading"}
_LOCAL = threading.local()


def register_parallel_backend(name, factory, make_default=False):
    """Register ``factory(n_jobs) -> executor`` under ``name`` (reference
    ``utils/__init__.py:50``, joblib's register_parallel_backend)."""
    if not callable(factory):
        raise TypeError("factory must be callable")
    _BACKENDS[str(name)] = factory
    if make_default:
        _DEFAULT["name"] = str(name)


def _active():
    stack = getattr(_LOCAL, "stack", None)
    return stack[-1] if stack else (_DEFAULT["name"], None, {})


@contextlib.contextmanager
def parallel_backend(backend, n_jobs=-1, inner_max_num_threads=None, **backend_params):
    """Context manager selecting the task backend and its default n_jobs for
    the ``Parallel`` calls inside it (reference ``utils/__init__.py:49``,
    joblib's parallel_backend): ``Parallel(n_jobs=None)`` then uses
    ``n_jobs``.  Thread-local, nestable."""
    name = str(backend)
    if name not in ("threading", "sequential", "loky", "multiprocessing") and name not in _BACKENDS:
        raise ValueError(f"Invalid backend: {backend!r}")
    stack = getattr(_LOCAL, "stack", None)
    if stack is None:
        stack = _LOCAL.stack = []
    stack.append((name, n_jobs, dict(backend_params)))
    try:
        yield name, n_jobs
    finally:
        stack.pop()


def effective_n_jobs(n_jobs=None):
    """joblib's convention: None -> the active backend's n_jobs (1 outside a
    parallel_backend context), -1 -> all CPUs, -k -> CPUs + 1 - k."""
    if n_jobs is None:
        name, ctx_jobs, _ = _active()
        if name == "sequential":
            return 1
        n_jobs = ctx_jobs
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
        self.backend = None if backend in (None, "loky", "multiprocessing") else str(backend)

    @staticmethod
    def _run(task, gpu, ctx=None):
        if ctx is not None:
            # the caller's parallel_backend stack, so a nested Parallel inside
            # a worker sees the same backend / n_jobs (the stack is thread-local)
            prev = getattr(_LOCAL, "stack", None)
            _LOCAL.stack = list(ctx)
            try:
                return Parallel._run(task, gpu)
            finally:
                _LOCAL.stack = prev
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
        name = self.backend or _active()[0]
        n = min(effective_n_jobs(self.n_jobs), max(len(tasks), 1))
        if n <= 1 or name == "sequential":
            return [self._run(t, None) for t in tasks]
        # task i -> GPU i mod n_gpus (+ per-task device config), for the
        # built-in threading backend and registered executors alike
        slots = _gpu_slots(self.devices)
        gpus = [slots[i % len(slots)] if slots else None for i in range(len(tasks))]
        ctx = list(getattr(_LOCAL, "stack", None) or [])
        if name in _BACKENDS:
            ex = _BACKENDS[name](n)
            try:
                futures = [ex.submit(Parallel._run, t, g, ctx) for t, g in zip(tasks, gpus)]
                return [f.result() for f in futures]
            finally:
                ex.shutdown(wait=True)
        with ThreadPoolExecutor(max_workers=n, thread_name_prefix="sq-task") as ex:
            futures = [ex.submit(self._run, t, g, ctx) for t, g in zip(tasks, gpus)]
            return [f.result() for f in futures]


__all__ = ["Parallel", "effective_n_jobs", "parallel_backend", "register_parallel_backend"]
