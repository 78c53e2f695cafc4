"""Makes ``IterativeImputer`` importable from ``impute`` (reference
``experimental/enable_iterative_imputer.py``; here it always is)."""
from .. import impute
from ..impute import IterativeImputer

setattr(impute, "IterativeImputer", IterativeImputer)
if "IterativeImputer" not in impute.__all__:
    impute.__all__ += ["IterativeImputer"]
