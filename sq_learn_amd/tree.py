"""Reference-layout import path (``sklearn.tree``)."""
from .models.tree import *  # noqa: F401,F403
from .models.tree import __all__  # noqa: F401
