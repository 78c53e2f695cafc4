"""The reference's q-means estimator functions, AST-extracted verbatim from
``/root/reference/sklearn/cluster/_dmeans.py`` (the module
itself cannot be imported - it needs ``matlab.engine`` and the compiled
Cython extensions).  Extracted: ``labels_estimation`` (:732-777),
``select_labels`` (:2252-2257), ``_centers_update`` (:780-830), ``wrapper``
(:725-727).  They run against the reference's own ``QuantumUtility/
Utility.py`` (``ipe``, ``tomography``) and scikit-learn's ``row_norms``.
Nothing is copied into the framework: the source is read at test time."""
import ast
import importlib.util
import itertools
import os
import random
import warnings

import numpy as np

DMEANS = "/root/reference/sklearn/cluster/_dmeans.py"
UTILITY = "/root/reference/sklearn/QuantumUtility/Utility.py"
FUNCS = ("labels_estimation", "select_labels", "_centers_update", "wrapper")


def available():
    return os.path.exists(DMEANS) and os.path.exists(UTILITY)


def load_utility():
    import matplotlib
    matplotlib.use("Agg")
    spec = importlib.util.spec_from_file_location("_ref_utility_dm", UTILITY)
    mod = importlib.util.module_from_spec(spec)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        spec.loader.exec_module(mod)
    return mod


def load():
    """Namespace with the extracted reference functions."""
    import scipy as sc
    import scipy.spatial  # noqa: F401  (sc.spatial.distance.cdist)
    from sklearn.utils.extmath import row_norms
    U = load_utility()
    tree = ast.parse(open(DMEANS).read())
    keep = [node for node in tree.body if isinstance(node, ast.FunctionDef) and node.name in FUNCS]
    assert {f.name for f in keep} == set(FUNCS), [f.name for f in keep]
    mod = ast.Module(body=keep, type_ignores=[])
    ns = {"np": np, "sc": sc, "random": random, "itertools": itertools, "row_norms": row_norms,
          "ipe": U.ipe, "tomography": U.tomography}
    exec(compile(mod, DMEANS, "exec"), ns)
    return ns, U
