"""Global configuration for sq_learn_amd.

Mirrors the reference's ``sklearn/_config.py:6-150`` (``get_config`` /
``set_config`` / ``config_context``) and adds the framework knobs that the
MI355X build needs: the compute device, the GEMM precision
policy for the fused distance kernels and the default counter-RNG seed.

Like newer scikit-learn the config is THREAD-LOCAL: each thread starts from
the process defaults and ``set_config`` / ``config_context`` change only the
calling thread's view.  Task-parallel workers (``sq_learn_amd.parallel.tasks``:
cross-validation folds, search candidates, one-vs-rest members, fanned out
over threads and GPUs) therefore get the dispatching thread's config
explicitly - ``utils.fixes.delayed`` captures it at dispatch and restores
it in the worker (reference ``utils/fixes.py:205-222``) - and each worker can
be pinned to its own GPU through the ``device`` key without touching the
other threads.
"""

import os
import threading
from contextlib import contextmanager

_global_config = {
    # --- reference keys (sklearn/_config.py:6-11) ---
    "assume_finite": bool(os.environ.get("SQ_ASSUME_FINITE", os.environ.get("SKLEARN_ASSUME_FINITE", False))),
    "working_memory": int(os.environ.get("SQ_WORKING_MEMORY", os.environ.get("SKLEARN_WORKING_MEMORY", 1024))),
    "print_changed_only": True,
    "display": "text",
    # --- MI355X framework keys ---
    # 'auto' -> cuda (HIP) when a GPU is visible, else cpu
    "device": os.environ.get("SQ_DEVICE", "auto"),
    # precision of the q-means / k-means distance GEMMs on GPU:
    #   'fp32' : fp32-faithful (default) - fused E-step on an fp16 hi/lo split
    #            (3 MFMA products, fp32 accumulation, csrc/estep_f32.hip),
    #            overflow rows re-selected in fp64
    #   'bf16' : bf16 operands, fp32 accumulation (MFMA 32x32x16): ~2x faster,
    #            band edges only bf16-accurate (2^-9 per operand)
    "gemm_precision": os.environ.get("SQ_GEMM_PRECISION", "fp32"),
    # default seed of the counter-based (Philox) stochastic layer when an
    # estimator is given random_state=None
    "seed": int(os.environ.get("SQ_SEED", 0x5EED)),
    # structured per-iteration logging (sq_learn_amd.utils.tracing)
    "log_iterations": bool(int(os.environ.get("SQ_LOG_ITERATIONS", "0"))),
}
_lock = threading.Lock()
_threadlocal = threading.local()


def _config():
    """This thread's mutable config (created from the process defaults)."""
    cfg = getattr(_threadlocal, "config", None)
    if cfg is None:
        with _lock:
            cfg = _threadlocal.config = dict(_global_config)
    return cfg


def get_config():
    """Return a copy of the current (thread's) configuration."""
    return dict(_config())


def set_config(assume_finite=None, working_memory=None, print_changed_only=None,
               display=None, device=None, gemm_precision=None, seed=None,
               log_iterations=None):
    """Set the configuration of the calling thread (reference:
    ``sklearn/_config.py:30``); threads started afterwards by the task layer
    receive it through ``utils.fixes.delayed``."""
    cfg = _config()
    if assume_finite is not None:
        cfg["assume_finite"] = assume_finite
    if working_memory is not None:
        cfg["working_memory"] = working_memory
    if print_changed_only is not None:
        cfg["print_changed_only"] = print_changed_only
    if display is not None:
        cfg["display"] = display
    if device is not None:
        cfg["device"] = device
    if gemm_precision is not None:
        if gemm_precision not in ("bf16", "fp32"):
            raise ValueError("gemm_precision must be 'bf16' or 'fp32'")
        cfg["gemm_precision"] = gemm_precision
    if seed is not None:
        cfg["seed"] = int(seed)
    if log_iterations is not None:
        cfg["log_iterations"] = bool(log_iterations)


@contextmanager
def config_context(**new_config):
    """Temporarily change the global config (reference ``_config.py:86``)."""
    old = get_config()
    set_config(**new_config)
    try:
        yield
    finally:
        set_config(**old)
