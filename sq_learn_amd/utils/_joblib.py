"""Reference-layout path ``utils/_joblib.py``: joblib's public names when
joblib is installed (the reference vendors or requires it); this package's
own fan-out is ``parallel/tasks.py`` (threads, one GPU per task), with the
config-propagating ``delayed`` of ``utils/fixes.py``."""
from .fixes import delayed  # noqa: F401
from ..parallel.tasks import effective_n_jobs  # noqa: F401

try:  # pragma: no cover - depends on the environment
    import joblib
    from joblib import (Memory, Parallel, cpu_count, dump, hash, load,  # noqa: F401
                        parallel_backend, register_parallel_backend)
    from joblib import __version__  # noqa: F401
    logger = joblib.logger
except ImportError:  # joblib absent: the task layer's Parallel stands in
    joblib = None
    from ..parallel.tasks import Parallel  # noqa: F401

__all__ = ["parallel_backend", "register_parallel_backend", "cpu_count", "Parallel", "Memory",
           "delayed", "effective_n_jobs", "hash", "logger", "dump", "load", "joblib",
           "__version__"]
