"""Reference-layout import path (``sklearn.linear_model``)."""
from .models.linear_model import *  # noqa: F401,F403
from .models.linear_model import __all__  # noqa: F401
from .models.linear_model._lm_extra import GeneralizedLinearRegressor  # noqa: F401,E402

from .utils._aliases import alias_submodules  # noqa: E402
alias_submodules(__name__, "_glm")

from .utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
