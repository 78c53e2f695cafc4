"""Reference-layout private module paths.

Code written against the reference sometimes imports from its private
modules (``from sklearn.ensemble._forest import ...``,
``from sklearn.utils._testing import ...``).  This package groups the same
names differently (a flat ``compose`` module, one ``_extra`` file per
family), so each such path is registered in ``sys.modules`` as an alias of
the module that actually holds the names - the module object itself, no
copies or wrappers.  Called at the end of the owning module, so an alias
exists as soon as its parent is imported, and
``import sq_learn_amd.compose._target`` resolves through ``sys.modules``
even where the parent is a plain module."""

import importlib
import sys


def alias_submodules(parent, *subs, target=None):
    """Register ``parent.<sub>`` for each sub as the module ``target``
    (default: the parent module itself) and bind it as an attribute."""
    pmod = sys.modules[parent]
    mod = pmod if target is None else importlib.import_module(target)
    for s in subs:
        sys.modules.setdefault(f"{parent}.{s}", mod)
        if not hasattr(pmod, s):
            setattr(pmod, s, mod)
