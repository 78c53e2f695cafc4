"""Reference-layout import path (``sklearn.manifold``)."""
from .models.manifold import *  # noqa: F401,F403
from .models.manifold import __all__  # noqa: F401

from .utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
