"""Reference-layout import path (``sklearn.neural_network``)."""
from .models.neural_network import *  # noqa: F401,F403
from .models.neural_network import __all__  # noqa: F401
