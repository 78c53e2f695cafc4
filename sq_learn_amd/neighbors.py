"""Reference-layout import path (``sklearn.neighbors``)."""
from .models.neighbors import *  # noqa: F401,F403
from .models.neighbors import __all__  # noqa: F401

from .utils._aliases import alias_submodules  # noqa: E402
alias_submodules(__name__, "_lof")

from .utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
