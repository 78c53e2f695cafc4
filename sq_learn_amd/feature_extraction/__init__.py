"""Feature extraction (reference ``sklearn.feature_extraction``): the
hashing trick, dict vectorisation, text vectorisers and image patches."""
from . import image, text  # noqa: F401
from ._dict_vectorizer import DictVectorizer  # noqa: F401
from ._hash import FeatureHasher  # noqa: F401
from ._stop_words import ENGLISH_STOP_WORDS  # noqa: F401
from .image import grid_to_graph, img_to_graph  # noqa: F401

__all__ = ["DictVectorizer", "image", "img_to_graph", "grid_to_graph", "text",
           "FeatureHasher"]
