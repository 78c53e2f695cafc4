"""Tree export (reference ``tree/_export.py``: ``export_text`` :825,
``export_graphviz``, ``plot_tree``)."""

import numpy as np

from ...base import is_classifier
from ...utils.validation import check_is_fitted
from ._tree import TREE_LEAF, TREE_UNDEFINED


def _subtree_depth(tree, node):
    depths, stack = [], [(node, 1)]
    while stack:
        n, d = stack.pop()
        if tree.children_left[n] == TREE_LEAF:
            depths.append(d)
        else:
            stack.append((tree.children_left[n], d + 1))
            stack.append((tree.children_right[n], d + 1))
    return max(depths)


def export_text(decision_tree, *, feature_names=None, max_depth=10, spacing=3, decimals=2,
                show_weights=False):
    """Text report of the rules of a fitted decision tree."""
    check_is_fitted(decision_tree)
    tree_ = decision_tree.tree_
    clf = is_classifier(decision_tree)
    class_names = decision_tree.classes_ if clf else None
    if max_depth < 0:
        raise ValueError("max_depth bust be >= 0, given %d" % max_depth)
    if feature_names is not None and len(feature_names) != tree_.n_features:
        raise ValueError("feature_names must contain %d elements, got %d"
                         % (tree_.n_features, len(feature_names)))
    if spacing <= 0:
        raise ValueError("spacing must be > 0, given %d" % spacing)
    if decimals < 0:
        raise ValueError("decimals must be >= 0, given %d" % decimals)
    value_fmt = ("{}{} weights: {}\n" if show_weights else "{}{}{}\n") if clf else "{}{} value: {}\n"
    if feature_names:
        names = [feature_names[i] if i != TREE_UNDEFINED else None for i in tree_.feature]
    else:
        names = ["feature_{}".format(i) for i in tree_.feature]
    out = []

    def add_leaf(value, class_name, indent):
        val = ""
        if show_weights or not clf:
            val = "[" + ", ".join("{1:.{0}f}".format(decimals, v) for v in value) + "]"
        if clf:
            val += " class: " + str(class_name)
        out.append(value_fmt.format(indent, "", val))

    def rec(node, depth):
        indent = ("|" + " " * spacing) * depth
        indent = indent[:-spacing] + "-" * spacing
        value = tree_.value[node][0] if tree_.n_outputs == 1 else tree_.value[node].T[0]
        class_name = np.argmax(value)
        if tree_.n_classes[0] != 1 and tree_.n_outputs == 1:
            class_name = class_names[class_name]
        if depth <= max_depth + 1:
            if tree_.feature[node] != TREE_UNDEFINED:
                name = names[node]
                thr = "{1:.{0}f}".format(decimals, tree_.threshold[node])
                out.append("{} {} <= {}\n".format(indent, name, thr))
                rec(tree_.children_left[node], depth + 1)
                out.append("{} {} >  {}\n".format(indent, name, thr))
                rec(tree_.children_right[node], depth + 1)
            else:
                add_leaf(value, class_name, indent)
        else:
            sd = _subtree_depth(tree_, node)
            if sd == 1:
                add_leaf(value, class_name, indent)
            else:
                out.append("{} {}\n".format(indent, "truncated branch of depth %d" % sd))

    rec(0, 1)
    return "".join(out)


def export_graphviz(decision_tree, out_file=None, *, max_depth=None, feature_names=None,
                    class_names=None, label="all", filled=False, leaves_parallel=False,
                    impurity=True, node_ids=False, proportion=False, rotate=False,
                    rounded=False, special_characters=False, precision=3, fontname="helvetica"):
    """DOT description of a fitted tree (returned as a string when
    ``out_file`` is None)."""
    check_is_fitted(decision_tree)
    t = decision_tree.tree_
    crit = getattr(decision_tree, "criterion", "impurity")
    lines = ["digraph Tree {",
             'node [shape=box%s, fontname="%s"] ;' % (", style=\"rounded\"" if rounded else "",
                                                       fontname),
             'edge [fontname="%s"] ;' % fontname]
    if rotate:
        lines.append("rankdir=LR ;")

    def node_label(i):
        parts = []
        if node_ids:
            parts.append("node #%d" % i)
        if t.children_left[i] != TREE_LEAF:
            f = t.feature[i]
            fname = feature_names[f] if feature_names is not None else "x[%d]" % f
            parts.append("%s <= %s" % (fname, round(float(t.threshold[i]), precision)))
        if impurity:
            parts.append("%s = %s" % (crit, round(float(t.impurity[i]), precision)))
        if proportion:
            parts.append("samples = %s%%" % round(100.0 * t.n_node_samples[i]
                                                  / t.n_node_samples[0], 1))
        else:
            parts.append("samples = %d" % t.n_node_samples[i])
        v = t.value[i]
        if t.n_outputs == 1:
            v = v[0]
        if proportion and t.n_classes[0] != 1:
            v = v / max(v.sum(), 1e-300)
        parts.append("value = %s" % np.array2string(np.round(v, precision), separator=", "))
        if class_names is not None and t.n_classes[0] != 1 and t.n_outputs == 1:
            cn = class_names[int(np.argmax(v))] if class_names is not True else "y[%d]" % int(
                np.argmax(v))
            parts.append("class = %s" % cn)
        return "\\n".join(parts)

    stack = [(0, -1, 0)]
    while stack:
        i, parent, depth = stack.pop()
        if max_depth is not None and depth > max_depth:
            lines.append('%d [label="(...)"] ;' % i)
        else:
            lines.append('%d [label="%s"] ;' % (i, node_label(i)))
            if t.children_left[i] != TREE_LEAF:
                stack.append((t.children_right[i], i, depth + 1))
                stack.append((t.children_left[i], i, depth + 1))
        if parent >= 0:
            lines.append("%d -> %d ;" % (parent, i))
    lines.append("}")
    dot = "\n".join(lines)
    if out_file is None:
        return dot
    if isinstance(out_file, str):
        with open(out_file, "w", encoding="utf-8") as f:
            f.write(dot)
    else:
        out_file.write(dot)
    return None


def plot_tree(decision_tree, *, max_depth=None, feature_names=None, class_names=None,
              label="all", filled=False, impurity=True, node_ids=False, proportion=False,
              rounded=False, precision=3, ax=None, fontsize=None):
    """Matplotlib rendering (layered layout: leaves spread left to right)."""
    import matplotlib.pyplot as plt
    check_is_fitted(decision_tree)
    t = decision_tree.tree_
    ax = ax or plt.gca()
    ax.set_axis_off()
    xs, counter = {}, [0]

    def place(i, depth):
        if t.children_left[i] == TREE_LEAF or (max_depth is not None and depth >= max_depth):
            xs[i] = (counter[0], depth)
            counter[0] += 1
            return xs[i][0]
        a = place(t.children_left[i], depth + 1)
        b = place(t.children_right[i], depth + 1)
        xs[i] = ((a + b) / 2.0, depth)
        return xs[i][0]

    place(0, 0)
    width = max(counter[0], 1)
    depth_max = max(d for _, d in xs.values()) + 1
    anns = []
    for i, (x, d) in xs.items():
        txt = "samples = %d" % t.n_node_samples[i]
        if t.children_left[i] != TREE_LEAF and i in xs:
            f = t.feature[i]
            fname = feature_names[f] if feature_names is not None else "x[%d]" % f
            txt = "%s <= %s\n" % (fname, round(float(t.threshold[i]), precision)) + txt
        anns.append(ax.annotate(txt, ((x + 0.5) / width, 1 - (d + 0.5) / depth_max),
                                ha="center", va="center", fontsize=fontsize,
                                bbox=dict(boxstyle="round" if rounded else "square", fc="w")))
    return anns
