"""GLM distributions (reference ``sklearn/_loss``)."""
from .glm_distribution import (ExponentialDispersionModel, GammaDistribution,  # noqa: F401
                               InverseGaussianDistribution, NormalDistribution,
                               PoissonDistribution, TweedieDistribution)
