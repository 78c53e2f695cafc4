"""Importable experimental-feature switches (reference ``experimental/``).

Every feature they used to gate is a regular estimator here, so importing a
switch only makes the estimator reachable under the same names as in the
reference (``enable_iterative_imputer`` -> ``impute.IterativeImputer``,
``enable_halving_search_cv`` -> ``model_selection.Halving*SearchCV``);
``enable_hist_gradient_boosting`` is a no-op with the reference's warning.
"""
