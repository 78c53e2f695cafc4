"""Reference-layout import path (``sklearn.random_projection``)."""
from .kernel_approximation import (GaussianRandomProjection, SparseRandomProjection,  # noqa: F401
                                   johnson_lindenstrauss_min_dim)
from .kernel_approximation import _BaseRandomProjection as BaseRandomProjection  # noqa: E402,F401
