"""Reference-layout import path (``sklearn.QuantumUtility.Utility``): the
quantum-simulation routines (host oracle + batched device samplers).

``from sq_learn_amd.QuantumUtility import Utility`` mirrors the reference's
``from sklearn.QuantumUtility import Utility``.
"""
from . import quantum as Utility  # noqa: F401
from .quantum import *  # noqa: F401,F403

from .utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
