"""Manifold learning (reference ``sklearn.manifold``)."""
from ._spectral import SpectralEmbedding, spectral_embedding

__all__ = ["SpectralEmbedding", "spectral_embedding"]
