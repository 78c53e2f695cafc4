"""Least-squares SVMs: classical LSSVC and quantum-simulated QLSSVC."""
from .lssvm import LSSVC, QLSSVC, conjugate_gradient

__all__ = ["LSSVC", "QLSSVC", "conjugate_gradient"]
