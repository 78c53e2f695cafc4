"""Reference-layout import path (``sklearn.manifold``)."""
from .models.manifold import *  # noqa: F401,F403
from .models.manifold import __all__  # noqa: F401
