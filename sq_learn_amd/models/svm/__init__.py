"""Least-squares SVMs: classical LSSVC and quantum-simulated QLSSVC."""
from ._liblinear import LinearSVC, LinearSVR
from ._libsvm import SVC, SVR, NuSVC, NuSVR, OneClassSVM
from .lssvm import LSSVC, QLSSVC, conjugate_gradient

__all__ = ["LSSVC", "QLSSVC", "conjugate_gradient", "SVC", "NuSVC", "SVR", "NuSVR",
           "OneClassSVM", "LinearSVC", "LinearSVR"]
