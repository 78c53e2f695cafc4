"""Reference-layout import path (``sklearn.neural_network``)."""
from .models.neural_network import *  # noqa: F401,F403
from .models.neural_network import __all__  # noqa: F401

from .utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
