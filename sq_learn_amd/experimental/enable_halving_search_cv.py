"""Makes the successive-halving searches importable from
``model_selection`` (reference ``experimental/enable_halving_search_cv.py``;
here they always are)."""
from .. import model_selection
from ..model_selection import HalvingGridSearchCV, HalvingRandomSearchCV

setattr(model_selection, "HalvingGridSearchCV", HalvingGridSearchCV)
setattr(model_selection, "HalvingRandomSearchCV", HalvingRandomSearchCV)
for _name in ("HalvingGridSearchCV", "HalvingRandomSearchCV"):
    if _name not in model_selection.__all__:
        model_selection.__all__ += [_name]
