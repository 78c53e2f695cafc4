"""Reference-layout import path (``sklearn.ensemble``)."""
from .models.ensemble import *  # noqa: F401,F403
from .models.ensemble import __all__  # noqa: F401
