"""Config-propagating task wrapper (reference ``utils/fixes.py:205-222``).

``delayed(f)(*args, **kw)`` returns the task triple ``(wrapper, args, kw)``;
the wrapper snapshots the DISPATCHING thread's configuration and re-applies
it around the call in whatever worker runs it (the configuration is
thread-local, ``_config.py``), optionally with per-task overrides - the task
layer pins each worker to its own GPU through ``device``."""

import functools

from .._config import config_context, get_config


class _FuncWrapper:
    """Call ``function`` under the configuration captured at construction."""

    def __init__(self, function):
        self.function = function
        self.config = get_config()
        functools.update_wrapper(self, function)

    def call_with(self, overrides, *args, **kwargs):
        cfg = dict(self.config)
        cfg.update(overrides or {})
        with config_context(**cfg):
            return self.function(*args, **kwargs)

    def __call__(self, *args, **kwargs):
        return self.call_with(None, *args, **kwargs)


def delayed(function):
    """Capture a call of ``function`` as a (wrapper, args, kwargs) task."""
    @functools.wraps(function)
    def delayed_function(*args, **kwargs):
        return _FuncWrapper(function), args, kwargs
    return delayed_function


__all__ = ["delayed"]


# numpy / scipy names the reference re-exports from its fixes module
from numpy import linspace  # noqa: E402,F401
from numpy.ma import MaskedArray  # noqa: E402,F401
from scipy.stats import loguniform  # noqa: E402,F401
