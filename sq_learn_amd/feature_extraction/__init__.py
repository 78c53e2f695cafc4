"""Feature extraction (reference ``sklearn.feature_extraction``): the
hashing trick (``FeatureHasher``)."""
from ._hash import FeatureHasher  # noqa: F401
