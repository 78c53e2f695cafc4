"""Remaining dataset generators and the bundled toy datasets (reference
``datasets/_samples_generator.py`` and ``datasets/_base.py``).

Generators consume the NumPy RandomState stream in the reference's order
so the same ``random_state`` yields the same arrays.  Toy datasets ship as
the reference's CSV files under ``sq_learn_amd/_data`` (public data, no
network needed) and load as ``Bunch`` objects (optionally pandas frames).
"""

import array
import csv

import numbers
import os

import numpy as np
import scipy.sparse as sp
from scipy import linalg

from ._bunch import Bunch
from .validation import check_random_state

DATA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_data")


def _util_shuffle(*arrays, random_state=None):
    rs = check_random_state(random_state)
    idx = np.arange(len(arrays[0]))
    rs.shuffle(idx)
    out = [a[idx] for a in arrays]
    return out[0] if len(out) == 1 else out


# --------------------------------------------------------------- generators
def make_multilabel_classification(n_samples=100, n_features=20, *, n_classes=5, n_labels=2,
                                   length=50, allow_unlabeled=True, sparse=False,
                                   return_indicator="dense", return_distributions=False,
                                   random_state=None):
    if n_classes < 1:
        raise ValueError("'n_classes' should be an integer greater than 0. Got {} instead."
                         .format(n_classes))
    if length < 1:
        raise ValueError("'length' should be an integer greater than 0. Got {} instead."
                         .format(length))
    g = check_random_state(random_state)
    p_c = g.rand(n_classes)
    p_c /= p_c.sum()
    cum_c = np.cumsum(p_c)
    p_w_c = g.rand(n_features, n_classes)
    p_w_c /= np.sum(p_w_c, axis=0)

    def sample():
        y_size = n_classes + 1
        while (not allow_unlabeled and y_size == 0) or y_size > n_classes:
            y_size = g.poisson(n_labels)
        y = set()
        while len(y) != y_size:
            y.update(np.searchsorted(cum_c, g.rand(y_size - len(y))))
        y = list(y)
        n_words = 0
        while n_words == 0:
            n_words = g.poisson(length)
        if len(y) == 0:
            return g.randint(n_features, size=n_words), y
        cw = p_w_c.take(y, axis=1).sum(axis=1).cumsum()
        cw /= cw[-1]
        return np.searchsorted(cw, g.rand(n_words)), y

    ind = array.array("i")
    ptr = array.array("i", [0])
    Y = []
    for _ in range(n_samples):
        w, y = sample()
        ind.extend(w)
        ptr.append(len(ind))
        Y.append(y)
    X = sp.csr_matrix((np.ones(len(ind)), ind, ptr), shape=(n_samples, n_features))
    X.sum_duplicates()
    if not sparse:
        X = X.toarray()
    if return_indicator in (True, "sparse", "dense"):
        from ..preprocessing import MultiLabelBinarizer
        lb = MultiLabelBinarizer(sparse_output=(return_indicator == "sparse"))
        Y = lb.fit([range(n_classes)]).transform(Y)
    elif return_indicator is not False:
        raise ValueError("return_indicator must be either 'sparse', 'dense' or False.")
    if return_distributions:
        return X, Y, p_c, p_w_c
    return X, Y


def make_hastie_10_2(n_samples=12000, *, random_state=None):
    rs = check_random_state(random_state)
    X = rs.normal(size=(n_samples, 10)).reshape((n_samples, 10))
    y = ((X ** 2.0).sum(axis=1) > 9.34).astype(np.float64, copy=False)
    y[y == 0.0] = -1.0
    return X, y


def make_regression(n_samples=100, n_features=100, *, n_informative=10, n_targets=1, bias=0.0,
                    effective_rank=None, tail_strength=0.5, noise=0.0, shuffle=True, coef=False,
                    random_state=None):
    from .datasets import make_low_rank_matrix
    n_informative = min(n_features, n_informative)
    g = check_random_state(random_state)
    if effective_rank is None:
        X = g.randn(n_samples, n_features)
    else:
        X = make_low_rank_matrix(n_samples=n_samples, n_features=n_features,
                                 effective_rank=effective_rank, tail_strength=tail_strength,
                                 random_state=g)
    gt = np.zeros((n_features, n_targets))
    gt[:n_informative, :] = 100 * g.rand(n_informative, n_targets)
    y = X @ gt + bias
    if noise > 0.0:
        y += g.normal(scale=noise, size=y.shape)
    if shuffle:
        X, y = _util_shuffle(X, y, random_state=g)
        idx = np.arange(n_features)
        g.shuffle(idx)
        X[:, :] = X[:, idx]
        gt = gt[idx]
    y = np.squeeze(y)
    return (X, y, np.squeeze(gt)) if coef else (X, y)


def _two_sizes(n_samples):
    if isinstance(n_samples, numbers.Integral):
        return n_samples // 2, n_samples - n_samples // 2
    try:
        a, b = n_samples
    except ValueError as e:
        raise ValueError("`n_samples` can be either an int or a two-element tuple.") from e
    return a, b


def make_circles(n_samples=100, *, shuffle=True, noise=None, random_state=None, factor=0.8):
    if factor >= 1 or factor < 0:
        raise ValueError("'factor' has to be between 0 and 1.")
    n_out, n_in = _two_sizes(n_samples)
    g = check_random_state(random_state)
    lo = np.linspace(0, 2 * np.pi, n_out, endpoint=False)
    li = np.linspace(0, 2 * np.pi, n_in, endpoint=False)
    X = np.vstack([np.append(np.cos(lo), np.cos(li) * factor),
                   np.append(np.sin(lo), np.sin(li) * factor)]).T
    y = np.hstack([np.zeros(n_out, dtype=np.intp), np.ones(n_in, dtype=np.intp)])
    if shuffle:
        X, y = _util_shuffle(X, y, random_state=g)
    if noise is not None:
        X += g.normal(scale=noise, size=X.shape)
    return X, y


def make_moons(n_samples=100, *, shuffle=True, noise=None, random_state=None):
    n_out, n_in = _two_sizes(n_samples)
    g = check_random_state(random_state)
    X = np.vstack([np.append(np.cos(np.linspace(0, np.pi, n_out)),
                             1 - np.cos(np.linspace(0, np.pi, n_in))),
                   np.append(np.sin(np.linspace(0, np.pi, n_out)),
                             1 - np.sin(np.linspace(0, np.pi, n_in)) - 0.5)]).T
    y = np.hstack([np.zeros(n_out, dtype=np.intp), np.ones(n_in, dtype=np.intp)])
    if shuffle:
        X, y = _util_shuffle(X, y, random_state=g)
    if noise is not None:
        X += g.normal(scale=noise, size=X.shape)
    return X, y


def make_friedman1(n_samples=100, n_features=10, *, noise=0.0, random_state=None):
    if n_features < 5:
        raise ValueError("n_features must be at least five.")
    g = check_random_state(random_state)
    X = g.rand(n_samples, n_features)
    y = (10 * np.sin(np.pi * X[:, 0] * X[:, 1]) + 20 * (X[:, 2] - 0.5) ** 2 + 10 * X[:, 3]
         + 5 * X[:, 4] + noise * g.randn(n_samples))
    return X, y


def _friedman_X(g, n):
    X = g.rand(n, 4)
    X[:, 0] *= 100
    X[:, 1] *= 520 * np.pi
    X[:, 1] += 40 * np.pi
    X[:, 3] *= 10
    X[:, 3] += 1
    return X


def make_friedman2(n_samples=100, *, noise=0.0, random_state=None):
    g = check_random_state(random_state)
    X = _friedman_X(g, n_samples)
    y = (X[:, 0] ** 2 + (X[:, 1] * X[:, 2] - 1 / (X[:, 1] * X[:, 3])) ** 2) ** 0.5 \
        + noise * g.randn(n_samples)
    return X, y


def make_friedman3(n_samples=100, *, noise=0.0, random_state=None):
    g = check_random_state(random_state)
    X = _friedman_X(g, n_samples)
    y = np.arctan((X[:, 1] * X[:, 2] - 1 / (X[:, 1] * X[:, 3])) / X[:, 0]) \
        + noise * g.randn(n_samples)
    return X, y


def make_sparse_coded_signal(n_samples, *, n_components, n_features, n_nonzero_coefs,
                             random_state=None):
    g = check_random_state(random_state)
    D = g.randn(n_features, n_components)
    D /= np.sqrt(np.sum(D ** 2, axis=0))
    X = np.zeros((n_components, n_samples))
    for i in range(n_samples):
        idx = np.arange(n_components)
        g.shuffle(idx)
        idx = idx[:n_nonzero_coefs]
        X[idx, i] = g.randn(n_nonzero_coefs)
    Y = D @ X
    return tuple(map(np.squeeze, (Y, D, X)))


def make_sparse_uncorrelated(n_samples=100, n_features=10, *, random_state=None):
    g = check_random_state(random_state)
    X = g.normal(loc=0, scale=1, size=(n_samples, n_features))
    y = g.normal(loc=X[:, 0] + 2 * X[:, 1] - 2 * X[:, 2] - 1.5 * X[:, 3],
                 scale=np.ones(n_samples))
    return X, y


def make_spd_matrix(n_dim, *, random_state=None):
    g = check_random_state(random_state)
    A = g.rand(n_dim, n_dim)
    U, _, Vt = linalg.svd(A.T @ A, check_finite=False)
    return U @ (1.0 + np.diag(g.rand(n_dim))) @ Vt


def make_sparse_spd_matrix(dim=1, *, alpha=0.95, norm_diag=False, smallest_coef=0.1,
                           largest_coef=0.9, random_state=None):
    rs = check_random_state(random_state)
    chol = -np.eye(dim)
    aux = rs.rand(dim, dim)
    aux[aux < alpha] = 0
    aux[aux > alpha] = smallest_coef + (largest_coef - smallest_coef) * rs.rand(np.sum(aux > alpha))
    aux = np.tril(aux, k=-1)
    perm = rs.permutation(dim)
    aux = aux[perm].T[perm]
    chol += aux
    prec = chol.T @ chol
    if norm_diag:
        d = 1.0 / np.sqrt(np.diag(prec).reshape(1, prec.shape[0]))
        prec *= d
        prec *= d.T
    return prec


def make_swiss_roll(n_samples=100, *, noise=0.0, random_state=None):
    g = check_random_state(random_state)
    t = 1.5 * np.pi * (1 + 2 * g.rand(1, n_samples))
    X = np.concatenate((t * np.cos(t), 21 * g.rand(1, n_samples), t * np.sin(t)))
    X += noise * g.randn(3, n_samples)
    return X.T, np.squeeze(t)


def make_s_curve(n_samples=100, *, noise=0.0, random_state=None):
    g = check_random_state(random_state)
    t = 3 * np.pi * (g.rand(1, n_samples) - 0.5)
    X = np.concatenate((np.sin(t), 2.0 * g.rand(1, n_samples), np.sign(t) * (np.cos(t) - 1)))
    X += noise * g.randn(3, n_samples)
    return X.T, np.squeeze(t)


def make_gaussian_quantiles(*, mean=None, cov=1.0, n_samples=100, n_features=2, n_classes=3,
                            shuffle=True, random_state=None):
    if n_samples < n_classes:
        raise ValueError("n_samples must be at least n_classes")
    g = check_random_state(random_state)
    mean = np.zeros(n_features) if mean is None else np.array(mean)
    X = g.multivariate_normal(mean, cov * np.identity(n_features), (n_samples,))
    X = X[np.argsort(np.sum((X - mean[np.newaxis, :]) ** 2, axis=1))]
    step = n_samples // n_classes
    y = np.hstack([np.repeat(np.arange(n_classes), step),
                   np.repeat(n_classes - 1, n_samples - step * n_classes)])
    if shuffle:
        X, y = _util_shuffle(X, y, random_state=g)
    return X, y


def _shuffle_2d(data, random_state=None):
    g = check_random_state(random_state)
    r = g.permutation(data.shape[0])
    c = g.permutation(data.shape[1])
    return data[r][:, c], r, c


def make_biclusters(shape, n_clusters, *, noise=0.0, minval=10, maxval=100, shuffle=True,
                    random_state=None):
    g = check_random_state(random_state)
    n_rows, n_cols = shape
    consts = g.uniform(minval, maxval, n_clusters)
    rs_ = g.multinomial(n_rows, np.repeat(1.0 / n_clusters, n_clusters))
    cs_ = g.multinomial(n_cols, np.repeat(1.0 / n_clusters, n_clusters))
    rl = np.hstack([np.repeat(v, r) for v, r in zip(range(n_clusters), rs_)])
    cl = np.hstack([np.repeat(v, r) for v, r in zip(range(n_clusters), cs_)])
    out = np.zeros(shape, dtype=np.float64)
    for i in range(n_clusters):
        out[np.outer(rl == i, cl == i)] += consts[i]
    if noise > 0:
        out += g.normal(scale=noise, size=out.shape)
    if shuffle:
        out, ri, ci = _shuffle_2d(out, random_state)
        rl, cl = rl[ri], cl[ci]
    return (out, np.vstack([rl == c for c in range(n_clusters)]),
            np.vstack([cl == c for c in range(n_clusters)]))


def make_checkerboard(shape, n_clusters, *, noise=0.0, minval=10, maxval=100, shuffle=True,
                      random_state=None):
    g = check_random_state(random_state)
    nr, nc = (n_clusters if hasattr(n_clusters, "__len__") else (n_clusters, n_clusters))
    n_rows, n_cols = shape
    rs_ = g.multinomial(n_rows, np.repeat(1.0 / nr, nr))
    cs_ = g.multinomial(n_cols, np.repeat(1.0 / nc, nc))
    rl = np.hstack([np.repeat(v, r) for v, r in zip(range(nr), rs_)])
    cl = np.hstack([np.repeat(v, r) for v, r in zip(range(nc), cs_)])
    out = np.zeros(shape, dtype=np.float64)
    for i in range(nr):
        for j in range(nc):
            out[np.outer(rl == i, cl == j)] += g.uniform(minval, maxval)
    if noise > 0:
        out += g.normal(scale=noise, size=out.shape)
    if shuffle:
        out, ri, ci = _shuffle_2d(out, random_state)
        rl, cl = rl[ri], cl[ci]
    rows = np.vstack([rl == a for a in range(nr) for _ in range(nc)])
    cols = np.vstack([cl == b for _ in range(nr) for b in range(nc)])
    return out, rows, cols


# ------------------------------------------------------------ toy datasets
def _frame(data, target, feature_names, target_names):
    import pandas as pd
    X = pd.DataFrame(data, columns=list(feature_names))
    if target.ndim == 1:
        y = pd.Series(target, name=target_names[0] if len(target_names) == 1 else "target")
    else:
        y = pd.DataFrame(target, columns=list(target_names))
    return pd.concat([X, y], axis=1), X, y


def _load_csv(name):
    path = os.path.join(DATA_DIR, name)
    with open(path) as f:
        r = csv.reader(f)
        head = next(r)
        n, d = int(head[0]), int(head[1])
        names = np.array(head[2:])
        data = np.empty((n, d))
        target = np.empty((n,), dtype=int)
        for i, row in enumerate(r):
            data[i] = np.asarray(row[:-1], dtype=np.float64)
            target[i] = int(row[-1])
    return data, target, names, path


def _finish(data, target, feature_names, target_names, descr, path, return_X_y, as_frame,
            **extra):
    frame = None
    if as_frame:
        tn = ["target"] if target.ndim == 1 else list(target_names)
        frame, data, target = _frame(data, target, feature_names, tn)
    if return_X_y:
        return data, target
    return Bunch(data=data, target=target, frame=frame, target_names=target_names, DESCR=descr,
                 feature_names=feature_names, filename=path, **extra)


def load_iris(*, return_X_y=False, as_frame=False):
    data, target, tn, path = _load_csv("iris.csv")
    fn = ["sepal length (cm)", "sepal width (cm)", "petal length (cm)", "petal width (cm)"]
    return _finish(data, target, fn, tn, "Iris plants dataset (150 x 4, 3 classes).", path,
                   return_X_y, as_frame)


def load_wine(*, return_X_y=False, as_frame=False):
    data, target, tn, path = _load_csv("wine_data.csv")
    fn = ["alcohol", "malic_acid", "ash", "alcalinity_of_ash", "magnesium", "total_phenols",
          "flavanoids", "nonflavanoid_phenols", "proanthocyanins", "color_intensity", "hue",
          "od280/od315_of_diluted_wines", "proline"]
    return _finish(data, target, fn, tn, "Wine recognition dataset (178 x 13, 3 classes).",
                   path, return_X_y, as_frame)


def load_breast_cancer(*, return_X_y=False, as_frame=False):
    data, target, tn, path = _load_csv("breast_cancer.csv")
    base = ["radius", "texture", "perimeter", "area", "smoothness", "compactness", "concavity",
            "concave points", "symmetry", "fractal dimension"]
    fn = np.array(["mean " + b for b in base] + [b + " error" for b in base]
                  + ["worst " + b for b in base])
    return _finish(data, target, fn, tn, "Breast cancer wisconsin (diagnostic) dataset "
                   "(569 x 30, 2 classes).", path, return_X_y, as_frame)


def load_digits(*, n_class=10, return_X_y=False, as_frame=False):
    path = os.path.join(DATA_DIR, "digits.csv.gz")
    raw = np.loadtxt(path, delimiter=",")
    target = raw[:, -1].astype(int, copy=False)
    flat = raw[:, :-1]
    images = flat.view()
    images.shape = (-1, 8, 8)
    if n_class < 10:
        idx = target < n_class
        flat, target, images = flat[idx], target[idx], images[idx]
    fn = ["pixel_{}_{}".format(r, c) for r in range(8) for c in range(8)]
    if return_X_y and not as_frame:
        return flat, target
    out = _finish(flat, target, fn, np.arange(10), "Optical recognition of handwritten digits "
                  "(8x8 images).", path, return_X_y, as_frame)
    if isinstance(out, Bunch):
        out.images = images
    return out


def load_diabetes(*, return_X_y=False, as_frame=False):
    dp = os.path.join(DATA_DIR, "diabetes_data.csv.gz")
    data = np.loadtxt(dp)
    target = np.loadtxt(os.path.join(DATA_DIR, "diabetes_target.csv.gz"))
    fn = ["age", "sex", "bmi", "bp", "s1", "s2", "s3", "s4", "s5", "s6"]
    out = _finish(data, target, fn, None, "Diabetes dataset (442 x 10, regression).", dp,
                  return_X_y, as_frame)
    if isinstance(out, Bunch):
        out.pop("target_names", None)
        out.data_filename, out.target_filename = "diabetes_data.csv.gz", "diabetes_target.csv.gz"
    return out


def load_linnerud(*, return_X_y=False, as_frame=False):
    ex = os.path.join(DATA_DIR, "linnerud_exercise.csv")
    ph = os.path.join(DATA_DIR, "linnerud_physiological.csv")
    data = np.loadtxt(ex, skiprows=1)
    target = np.loadtxt(ph, skiprows=1)
    with open(ex) as f:
        fn = f.readline().split()
    with open(ph) as f:
        tn = f.readline().split()
    frame = None
    if as_frame:
        frame, data, target = _frame(data, target, fn, tn)
    if return_X_y:
        return data, target
    return Bunch(data=data, feature_names=fn, target=target, target_names=tn, frame=frame,
                 DESCR="Linnerud dataset (20 x 3 exercise, 3 physiological targets).",
                 data_filename=ex, target_filename=ph)


def load_boston(*, return_X_y=False):
    path = os.path.join(DATA_DIR, "boston_house_prices.csv")
    with open(path) as f:
        r = csv.reader(f)
        head = next(r)
        n, d = int(head[0]), int(head[1])
        fn = np.array(next(r))
        data = np.empty((n, d))
        target = np.empty((n,))
        for i, row in enumerate(r):
            data[i] = np.asarray(row[:-1], dtype=np.float64)
            target[i] = float(row[-1])
    if return_X_y:
        return data, target
    return Bunch(data=data, target=target, feature_names=fn[:-1],
                 DESCR="Boston house prices dataset (506 x 13, regression).", filename=path)


def get_data_home(data_home=None):
    data_home = data_home or os.environ.get("SCIKIT_LEARN_DATA",
                                            os.path.join("~", "scikit_learn_data"))
    data_home = os.path.expanduser(data_home)
    os.makedirs(data_home, exist_ok=True)
    return data_home


def clear_data_home(data_home=None):
    import shutil
    shutil.rmtree(get_data_home(data_home))


def load_files(container_path, *, description=None, categories=None, load_content=True,
               shuffle=True, encoding=None, decode_error="strict", random_state=0):
    """Text files organised one sub-folder per category."""
    folders = sorted(f for f in os.listdir(container_path)
                     if os.path.isdir(os.path.join(container_path, f)))
    if categories is not None:
        folders = [f for f in folders if f in categories]
    target, filenames = [], []
    for label, folder in enumerate(folders):
        fp = os.path.join(container_path, folder)
        docs = sorted(os.listdir(fp))
        target.extend(len(docs) * [label])
        filenames.extend(os.path.join(fp, d) for d in docs)
    filenames = np.array(filenames)
    target = np.array(target)
    if shuffle:
        rs = check_random_state(random_state)
        idx = np.arange(filenames.shape[0])
        rs.shuffle(idx)
        filenames, target = filenames[idx], target[idx]
    out = dict(filenames=filenames, target_names=folders, target=target, DESCR=description)
    if load_content:
        data = []
        for fn in filenames:
            with open(fn, "rb") as f:
                data.append(f.read())
        if encoding is not None:
            data = [d.decode(encoding, decode_error) for d in data]
        out["data"] = data
    return Bunch(**out)


def load_sample_images():
    """The two bundled sample photographs (``china.jpg``, ``flower.jpg``,
    427 x 640 x 3 uint8; CC-BY, see ``_data/images/README.txt``) as a Bunch
    with ``images``, ``filenames`` and ``DESCR`` (reference
    ``datasets/_base.py:1096``); decoded with Pillow."""
    from PIL import Image
    folder = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_data",
                          "images")
    files = sorted(os.path.join(folder, f) for f in os.listdir(folder) if f.endswith(".jpg"))
    images = []
    for f in files:
        with Image.open(f) as im:
            images.append(np.asarray(im.convert("RGB"), dtype=np.uint8))
    return Bunch(images=images, filenames=files,
                 DESCR="Two sample photographs (china.jpg, flower.jpg) for image processing "
                       "examples; Creative Commons BY 2.0 (README.txt next to the files).")


def load_sample_image(image_name):
    """One sample image by file name ('china.jpg' or 'flower.jpg') as a
    (height, width, 3) uint8 array (reference ``datasets/_base.py:1147``)."""
    data = load_sample_images()
    for name, img in zip(data.filenames, data.images):
        if name.endswith(image_name):
            return img
    raise AttributeError("Cannot find sample image: %s" % image_name)


def _fetch_unavailable(name):
    def f(*args, **kwargs):
        raise IOError("%s downloads its data from the internet, which is not available in this "
                      "deployment; place the files under get_data_home() and load them with "
                      "load_files / load_svmlight_file instead." % name)
    f.__name__ = name
    return f


fetch_20newsgroups = _fetch_unavailable("fetch_20newsgroups")
fetch_20newsgroups_vectorized = _fetch_unavailable("fetch_20newsgroups_vectorized")
fetch_california_housing = _fetch_unavailable("fetch_california_housing")
fetch_covtype = _fetch_unavailable("fetch_covtype")
fetch_kddcup99 = _fetch_unavailable("fetch_kddcup99")
fetch_lfw_pairs = _fetch_unavailable("fetch_lfw_pairs")
fetch_lfw_people = _fetch_unavailable("fetch_lfw_people")
fetch_olivetti_faces = _fetch_unavailable("fetch_olivetti_faces")
fetch_openml = _fetch_unavailable("fetch_openml")
fetch_rcv1 = _fetch_unavailable("fetch_rcv1")
fetch_species_distributions = _fetch_unavailable("fetch_species_distributions")

__all__ = [n for n in dir() if n.startswith(("make_", "load_", "fetch_"))] + [
    "get_data_home", "clear_data_home"]

