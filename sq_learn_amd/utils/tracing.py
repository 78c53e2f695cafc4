"""Tracing and structured iteration logging.

* :func:`range` - a roctx range (via torch's nvtx shim, which maps to roctx
  on ROCm) around a phase, so ``rocprofv3 --marker-trace`` / timeline views
  show E-step / M-step / all-reduce / noise; a no-op unless ``SQ_TRACE=1``.
* :class:`IterationLog` - per-iteration records (iteration, inertia, shift,
  wall ms, bytes all-reduced) emitted through ``logging`` instead of the
  reference's unconditional ``print`` (``_dmeans.py:652``).
"""

import contextlib
import logging
import os
import time

logger = logging.getLogger("sq_learn_amd")
_ENABLED = os.environ.get("SQ_TRACE", "0") == "1"


def enable(flag=True):
    global _ENABLED
    _ENABLED = bool(flag)


@contextlib.contextmanager
def range(name):  # noqa: A001 - mirrors nvtx/roctx naming
    if not _ENABLED:
        yield
        return
    try:
        import torch
        torch.cuda.nvtx.range_push(name)
        pushed = True
    except Exception:  # pragma: no cover
        pushed = False
    try:
        yield
    finally:
        if pushed:
            import torch
            torch.cuda.nvtx.range_pop()


class IterationLog:
    def __init__(self, name, verbose=0, comm=None):
        self.name = name
        self.verbose = verbose
        self.comm = comm
        self.records = []
        self._t = time.perf_counter()

    def record(self, **fields):
        now = time.perf_counter()
        fields["ms"] = (now - self._t) * 1e3
        self._t = now
        if self.comm is not None:
            fields["bytes_allreduced"] = self.comm.bytes_reduced
        self.records.append(fields)
        if self.verbose:
            msg = ", ".join(f"{k}={v:.6g}" if isinstance(v, float) else f"{k}={v}"
                            for k, v in fields.items())
            logger.info("%s: %s", self.name, msg)
            if self.verbose > 1:
                print(f"{self.name}: {msg}")
