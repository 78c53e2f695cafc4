"""Reference-layout import path (``sklearn.tree``)."""
from .models.tree import *  # noqa: F401,F403
from .models.tree import __all__  # noqa: F401

from .utils._aliases import alias_submodules  # noqa: E402
alias_submodules(__name__, "_classes", target="sq_learn_amd.models.tree._classes")

from .utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
