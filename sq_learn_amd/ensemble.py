"""Reference-layout import path (``sklearn.ensemble``)."""
from .models.ensemble import *  # noqa: F401,F403
from .models.ensemble import __all__  # noqa: F401

from .utils._aliases import alias_submodules  # noqa: E402
alias_submodules(__name__, "_bagging", "_forest", "_iforest", "_weight_boosting")

from .utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
