"""HIP-backed compute ops (GPU tensors) with torch twins (CPU tensors)."""
from . import _native  # noqa: F401
