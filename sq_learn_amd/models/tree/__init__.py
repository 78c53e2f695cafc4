"""Decision trees (reference ``sklearn.tree``)."""
from ._classes import (BaseDecisionTree, DecisionTreeClassifier, DecisionTreeRegressor, ExtraTreeClassifier,
                       ExtraTreeRegressor)
from ._export import export_graphviz, export_text, plot_tree
from ._tree import Tree

__all__ = ["BaseDecisionTree", "DecisionTreeClassifier", "DecisionTreeRegressor", "ExtraTreeClassifier",
           "ExtraTreeRegressor", "export_graphviz", "export_text", "plot_tree", "Tree"]
