"""Reference-layout import path (``sklearn.neighbors``)."""
from .models.neighbors import KNeighborsClassifier, KNeighborsRegressor, NearestNeighbors  # noqa: F401
