"""Reference-layout path of the ``deprecated`` decorator
(``utils/deprecation.py``; implemented in ``utils/_misc.py``)."""
from ._misc import deprecated

__all__ = ["deprecated"]
