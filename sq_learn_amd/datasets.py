"""Reference-layout import path (``sklearn.datasets``): synthetic generators."""
from .utils.datasets import (make_blobs, make_blobs_device, make_classification,  # noqa: F401
                             make_low_rank_device, make_low_rank_matrix)
from .utils.svmlight import dump_svmlight_file, load_svmlight_file, load_svmlight_files  # noqa: F401
from .utils.datasets_extra import *  # noqa: F401,F403,E402
from .utils.datasets_extra import __all__ as _extra_all  # noqa: E402,F401

from .utils._aliases import alias_submodules  # noqa: E402
alias_submodules(__name__, "_openml")

from .utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
