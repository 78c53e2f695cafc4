"""No-op kept for import compatibility (reference
``experimental/enable_hist_gradient_boosting.py``): the histogram gradient
boosting estimators are regular members of ``ensemble``."""
import warnings

warnings.warn("Since version 1.0, it is not needed to import enable_hist_gradient_boosting "
              "anymore. HistGradientBoostingClassifier and HistGradientBoostingRegressor are "
              "now stable and can be normally imported from sq_learn_amd.ensemble.")
