"""Manifold learning (reference ``sklearn.manifold``)."""
from ._embed import (MDS, TSNE, Isomap, LocallyLinearEmbedding, locally_linear_embedding,
                     smacof, trustworthiness)
from ._spectral import SpectralEmbedding, spectral_embedding

__all__ = ["SpectralEmbedding", "spectral_embedding", "TSNE", "trustworthiness", "Isomap",
           "LocallyLinearEmbedding", "locally_linear_embedding", "MDS", "smacof"]
