"""Fitted-tree container and native growth/inference glue (reference
``tree/_tree.pyx``: ``Tree`` arrays, ``apply``, ``predict``,
``decision_path``, ``compute_feature_importances``, cost-complexity pruning
``_cost_complexity_prune`` / ``ccp_pruning_path`` / ``_build_pruned_tree``
at ``_tree.pyx:1294-1650``).

Growth runs in the host-native builder (``csrc/host/tree.cpp``, one OpenMP
thread per tree for forests); inference runs natively too: the host
``sqh_forest_apply`` for numpy inputs and the HIP ``forest_apply`` kernel
(``csrc/forest.hip``) when the rows live on a GPU.
"""

import ctypes

import numpy as np
import scipy.sparse as sp
import torch

from ...ops import _host

CRITERIA = {"gini": 0, "entropy": 1, "log_loss": 1, "squared_error": 2, "mse": 2,
            "friedman_mse": 3, "absolute_error": 4, "mae": 4, "poisson": 5}
RAND_R_MAX = 0x7FFFFFFF
TREE_LEAF = -1
TREE_UNDEFINED = -2


class Tree:
    """Array-of-structures view of one fitted binary tree (same attribute
    names as the reference's ``sklearn.tree._tree.Tree``)."""

    def __init__(self, n_features, n_classes, n_outputs):
        self.n_features = int(n_features)
        self.n_classes = np.asarray(n_classes, dtype=np.intp).reshape(-1)
        self.n_outputs = int(n_outputs)
        self.max_n_classes = int(self.n_classes.max()) if self.n_classes.size else 1
        self.node_count = 0
        self.max_depth = 0
        empty_i = np.zeros(0, dtype=np.intp)
        self.children_left = empty_i
        self.children_right = empty_i
        self.feature = empty_i
        self.threshold = np.zeros(0)
        self.impurity = np.zeros(0)
        self.n_node_samples = empty_i
        self.weighted_n_node_samples = np.zeros(0)
        self.value = np.zeros((0, self.n_outputs, self.max_n_classes))

    @property
    def capacity(self):
        return self.node_count

    @property
    def n_leaves(self):
        return int(np.sum(self.children_left == TREE_LEAF))

    def _set_arrays(self, left, right, feature, threshold, impurity, n_node, wn, value,
                    max_depth):
        self.children_left = left
        self.children_right = right
        self.feature = feature
        self.threshold = threshold
        self.impurity = impurity
        self.n_node_samples = n_node
        self.weighted_n_node_samples = wn
        self.value = value.reshape(len(left), self.n_outputs, -1)
        self.node_count = len(left)
        self.max_depth = int(max_depth)

    # ------------------------------------------------------------- inference
    def apply(self, X):
        """Leaf id of each row."""
        return forest_apply([self], X)[:, 0]

    def predict(self, X):
        return self.value.take(self.apply(X), axis=0)

    def decision_path(self, X):
        """CSR indicator (n_samples, node_count) of the nodes each row visits."""
        X = _dense_f32(X)
        n = X.shape[0]
        node = np.zeros(n, dtype=np.intp)
        rows, cols = [np.arange(n)], [node.copy()]
        active = np.arange(n)
        while active.size:
            cur = node[active]
            internal = self.children_left[cur] != TREE_LEAF
            active, cur = active[internal], cur[internal]
            if not active.size:
                break
            go_left = X[active, self.feature[cur]].astype(np.float64) <= self.threshold[cur]
            nxt = np.where(go_left, self.children_left[cur], self.children_right[cur])
            node[active] = nxt
            rows.append(active)
            cols.append(nxt)
        r = np.concatenate(rows)
        c = np.concatenate(cols)
        order = np.lexsort((c, r))
        return sp.csr_matrix((np.ones(len(r), dtype=np.intp), (r[order], c[order])),
                             shape=(n, self.node_count))

    def compute_feature_importances(self, normalize=True):
        imp = np.zeros(self.n_features)
        left, right = self.children_left, self.children_right
        wn, im = self.weighted_n_node_samples, self.impurity
        inner = np.where(left != TREE_LEAF)[0]
        if inner.size:
            dec = (wn[inner] * im[inner] - wn[left[inner]] * im[left[inner]]
                   - wn[right[inner]] * im[right[inner]])
            np.add.at(imp, self.feature[inner], dec)
        if self.node_count and wn[0] > 0:
            imp /= wn[0]
        if normalize:
            s = imp.sum()
            if s > 0.0:
                imp /= s
        return imp


def _dense_f32(X):
    if isinstance(X, torch.Tensor):
        X = X.detach().cpu().numpy()
    if sp.issparse(X):
        X = X.toarray()
    return np.ascontiguousarray(X, dtype=np.float32)


# ------------------------------------------------------------------- growth
def build_trees(X, y, sample_weights, n_classes, params, seeds, n_threads=0):
    """Grow ``len(seeds)`` trees natively (OpenMP over trees).

    X: (n, d) float32; y: (n, n_outputs) float64 (class codes for
    classification); sample_weights: None or (n_trees, n) float64;
    n_classes: per-output class counts (ones for regression); params: dict
    with criterion, splitter, max_depth, min_samples_split, min_samples_leaf,
    max_features, max_leaf_nodes, min_weight_leaf, min_impurity_decrease.
    Returns a list of ``Tree``.
    """
    lib = _host.lib()
    Xc = np.asfortranarray(X, dtype=np.float32)
    n, d = Xc.shape
    y = np.ascontiguousarray(y, dtype=np.float64)
    if y.ndim == 1:
        y = y[:, None]
    n_outputs = y.shape[1]
    n_classes = np.ascontiguousarray(n_classes, dtype=np.int64).reshape(-1)
    classif = params["criterion"] in ("gini", "entropy", "log_loss")
    max_nc = int(n_classes.max()) if classif else 1
    prm = np.array([CRITERIA[params["criterion"]], 1 if params["splitter"] == "random" else 0,
                    params["max_depth"], params["min_samples_split"], params["min_samples_leaf"],
                    params["max_features"], params["max_leaf_nodes"], params["min_weight_leaf"],
                    params["min_impurity_decrease"]], dtype=np.float64)
    seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
    T = len(seeds)
    sw = None
    if sample_weights is not None:
        sw = np.ascontiguousarray(sample_weights, dtype=np.float64).reshape(T, n)
    handles = (ctypes.c_void_p * T)()
    lib.sqh_forest_build(Xc.ctypes.data, y.ctypes.data, _host.ptr(sw), n, d, n_outputs,
                         n_classes.ctypes.data, max_nc, prm.ctypes.data, seeds.ctypes.data, T,
                         int(n_threads), ctypes.cast(handles, ctypes.c_void_p))
    out = []
    sizes = np.zeros(3, dtype=np.int64)
    for h in handles:
        lib.sqh_tree_sizes(h, sizes.ctypes.data)
        m, depth, stride = (int(v) for v in sizes)
        left, right, feat = (np.empty(m, dtype=np.int64) for _ in range(3))
        thr, imp, wn = np.empty(m), np.empty(m), np.empty(m)
        nn = np.empty(m, dtype=np.int64)
        val = np.empty(m * stride)
        lib.sqh_tree_copy(h, left.ctypes.data, right.ctypes.data, feat.ctypes.data,
                          thr.ctypes.data, imp.ctypes.data, nn.ctypes.data, wn.ctypes.data,
                          val.ctypes.data)
        lib.sqh_tree_free(h)
        t = Tree(d, n_classes if classif else np.ones(n_outputs, dtype=np.intp), n_outputs)
        t._set_arrays(left.astype(np.intp), right.astype(np.intp), feat.astype(np.intp),
                      thr, imp, nn.astype(np.intp), wn, val, depth)
        out.append(t)
    return out


# ---------------------------------------------------------------- inference
def stack_trees(trees):
    """Concatenated node arrays of several trees + per-tree node offsets."""
    offs = np.zeros(len(trees), dtype=np.int64)
    acc = 0
    for i, t in enumerate(trees):
        offs[i] = acc
        acc += t.node_count

    def cat(name, dt):
        return np.ascontiguousarray(np.concatenate([getattr(t, name) for t in trees]), dtype=dt)

    return (cat("children_left", np.int64), cat("children_right", np.int64),
            cat("feature", np.int64), cat("threshold", np.float64), offs)


def forest_apply_host(trees, X):
    """(n, n_trees) leaf ids, host-native traversal."""
    X = _dense_f32(X)
    n, d = X.shape
    left, right, feat, thr, offs = stack_trees(trees)
    out = np.empty((n, len(trees)), dtype=np.int64)
    _host.lib().sqh_forest_apply(left.ctypes.data, right.ctypes.data, feat.ctypes.data,
                                 thr.ctypes.data, offs.ctypes.data, len(trees), X.ctypes.data,
                                 n, d, out.ctypes.data)
    return out.astype(np.intp)


def forest_apply_device(trees, X):
    """(n, n_trees) leaf ids of GPU rows with the HIP traversal kernel."""
    from ...ops import forest as _fops
    left, right, feat, thr, offs = stack_trees(trees)
    leaves = _fops.forest_apply(X, left, right, feat, thr, offs)
    return leaves.cpu().numpy().astype(np.intp)


def forest_apply(trees, X):
    if isinstance(X, torch.Tensor) and X.is_cuda:
        return forest_apply_device(trees, X)
    return forest_apply_host(trees, X)


# ------------------------------------------------------------------ pruning
def _parents(tree):
    parent = np.full(tree.node_count, -1, dtype=np.intp)
    inner = np.where(tree.children_left != TREE_LEAF)[0]
    parent[tree.children_left[inner]] = inner
    parent[tree.children_right[inner]] = inner
    return parent


def _cost_complexity_prune(tree, stop_alpha=None):
    """Weakest-link pruning (reference ``_tree.pyx:1294-1470``).  Returns
    (leaves_in_subtree mask, alphas, impurities)."""
    m = tree.node_count
    wn, imp = tree.weighted_n_node_samples, tree.impurity
    left, right = tree.children_left, tree.children_right
    r_node = wn * imp / wn[0]
    parent = _parents(tree)
    is_leaf = left == TREE_LEAF
    leaves = is_leaf.copy()
    r_branch = np.zeros(m)
    n_leaves = np.zeros(m, dtype=np.intp)
    for leaf in np.where(is_leaf)[0]:
        r_branch[leaf] = r_node[leaf]
        cur = r_node[leaf]
        node = leaf
        while node != 0:
            p = parent[node]
            r_branch[p] += cur
            n_leaves[p] += 1
            node = p
    candidate = ~is_leaf
    in_subtree = np.ones(m, dtype=bool)
    alphas, imps = [0.0], [r_branch[0]]
    while candidate[0]:
        idx = np.where(candidate)[0]
        sub_alpha = (r_node[idx] - r_branch[idx]) / (n_leaves[idx] - 1)
        j = int(np.argmin(sub_alpha))   # first minimum = the reference's strict '<' scan
        eff, pruned = float(sub_alpha[j]), int(idx[j])
        if stop_alpha is not None and stop_alpha < eff:
            break
        stack = [pruned]
        while stack:
            node = stack.pop()
            if not in_subtree[node]:
                continue
            candidate[node] = False
            leaves[node] = False
            in_subtree[node] = False
            if left[node] != TREE_LEAF:
                stack.append(left[node])
                stack.append(right[node])
        leaves[pruned] = True
        in_subtree[pruned] = True
        n_pruned = n_leaves[pruned] - 1
        n_leaves[pruned] = 0
        r_diff = r_node[pruned] - r_branch[pruned]
        r_branch[pruned] = r_node[pruned]
        node = parent[pruned]
        while node != -1:
            n_leaves[node] -= n_pruned
            r_branch[node] += r_diff
            node = parent[node]
        alphas.append(eff)
        imps.append(r_branch[0])
    return leaves, np.asarray(alphas), np.asarray(imps)


def ccp_pruning_path(tree):
    _, alphas, imps = _cost_complexity_prune(tree)
    return {"ccp_alphas": alphas, "impurities": imps}


def build_pruned_tree_ccp(tree, ccp_alpha):
    """Copy of ``tree`` with the weakest-link subtrees below ``ccp_alpha``
    collapsed; node order is the depth-first (left first) preorder."""
    leaves, _, _ = _cost_complexity_prune(tree, stop_alpha=ccp_alpha)
    order, parent_new, is_left, depth = [], [], [], []
    stack = [(0, -1, False, 0)]
    while stack:
        node, par, il, dep = stack.pop()
        order.append(node)
        parent_new.append(par)
        is_left.append(il)
        depth.append(dep)
        new_id = len(order) - 1
        if not leaves[node]:
            stack.append((tree.children_right[node], new_id, False, dep + 1))
            stack.append((tree.children_left[node], new_id, True, dep + 1))
    order = np.asarray(order)
    m = len(order)
    left = np.full(m, TREE_LEAF, dtype=np.intp)
    right = np.full(m, TREE_LEAF, dtype=np.intp)
    for new_id in range(1, m):
        (left if is_left[new_id] else right)[parent_new[new_id]] = new_id
    leaf_new = leaves[order]
    feat = np.where(leaf_new, TREE_UNDEFINED, tree.feature[order])
    thr = np.where(leaf_new, float(TREE_UNDEFINED), tree.threshold[order])
    out = Tree(tree.n_features, tree.n_classes, tree.n_outputs)
    out._set_arrays(left, right, feat.astype(np.intp), thr, tree.impurity[order].copy(),
                    tree.n_node_samples[order].copy(),
                    tree.weighted_n_node_samples[order].copy(), tree.value[order].copy(),
                    max(depth) if depth else 0)
    return out
