"""QuantumUtility error model (reference ``sklearn/QuantumUtility``).

``from sq_learn_amd.quantum import *`` gives the reference's public names
(``QuantumState``, ``tomography``, ``amplitude_estimation``,
``phase_estimation``, ``consistent_phase_estimation``, ``ipe``, ``best_mu``,
...) with exact semantics (NumPy oracle, :mod:`.reference`); the batched
device versions live in :mod:`.device` and :mod:`sq_learn_amd.ops.random`;
the analytic quantum running-time formulas in :mod:`.cost_model`.
"""

from .reference import *  # noqa: F401,F403
from .reference import __all__ as _ref_all
from . import device, fejer, cost_model  # noqa: F401

__all__ = list(_ref_all) + ["device", "fejer", "cost_model"]
