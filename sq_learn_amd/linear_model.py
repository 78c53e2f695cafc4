"""Reference-layout import path (``sklearn.linear_model``)."""
from .models.linear_model import *  # noqa: F401,F403
from .models.linear_model import __all__  # noqa: F401
