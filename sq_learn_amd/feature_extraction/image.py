"""Image feature extraction (reference ``feature_extraction/image.py``):
pixel-adjacency graphs and patch extraction / reconstruction."""

import numbers
from itertools import product

import numpy as np
from numpy.lib.stride_tricks import as_strided
from scipy import sparse

from ..base import BaseEstimator
from ..utils.validation import check_random_state

__all__ = ["PatchExtractor", "extract_patches_2d", "grid_to_graph", "img_to_graph",
           "reconstruct_from_patches_2d"]


def _make_edges_3d(n_x, n_y, n_z=1):
    v = np.arange(n_x * n_y * n_z).reshape((n_x, n_y, n_z))
    return np.hstack([np.vstack((v[:, :, :-1].ravel(), v[:, :, 1:].ravel())),
                      np.vstack((v[:, :-1].ravel(), v[:, 1:].ravel())),
                      np.vstack((v[:-1].ravel(), v[1:].ravel()))])


def _compute_gradient_3d(edges, img):
    flat = img.reshape(-1)
    return np.abs(flat[edges[0]] - flat[edges[1]])


def _mask_edges_weights(mask, edges, weights=None):
    inds = np.arange(mask.size)[mask.ravel()]
    keep = np.logical_and(np.isin(edges[0], inds), np.isin(edges[1], inds))
    edges = edges[:, keep]
    if weights is not None:
        weights = weights[keep]
    top = edges.max() if edges.size else 0
    order = np.searchsorted(np.flatnonzero(mask), np.arange(top + 1))
    edges = order[edges]
    return edges if weights is None else (edges, weights)


def _to_graph(n_x, n_y, n_z, mask=None, img=None, return_as=sparse.coo_matrix, dtype=None):
    edges = _make_edges_3d(n_x, n_y, n_z)
    if dtype is None:
        dtype = int if img is None else img.dtype
    if img is not None:
        img = np.atleast_3d(img)
        weights = _compute_gradient_3d(edges, img)
        if mask is not None:
            edges, weights = _mask_edges_weights(mask, edges, weights)
            diag = img.squeeze()[mask]
        else:
            diag = img.ravel()
        nv = diag.size
    else:
        if mask is not None:
            mask = np.asarray(mask, dtype=bool)
            edges = _mask_edges_weights(mask, edges)
            nv = int(np.sum(mask))
        else:
            nv = n_x * n_y * n_z
        weights = np.ones(edges.shape[1], dtype=dtype)
        diag = np.ones(nv, dtype=dtype)
    d = np.arange(nv)
    i = np.hstack((edges[0], edges[1], d))
    j = np.hstack((edges[1], edges[0], d))
    g = sparse.coo_matrix((np.hstack((weights, weights, diag)), (i, j)), (nv, nv), dtype=dtype)
    if return_as is np.ndarray:
        return g.toarray()
    return return_as(g)


def img_to_graph(img, *, mask=None, return_as=sparse.coo_matrix, dtype=None):
    """Pixel-to-pixel gradient connections (edge weight |I_a - I_b|)."""
    img = np.atleast_3d(img)
    return _to_graph(*img.shape, mask, img, return_as, dtype)


def grid_to_graph(n_x, n_y, n_z=1, *, mask=None, return_as=sparse.coo_matrix, dtype=int):
    """Pixel-to-pixel connectivity graph of a grid."""
    return _to_graph(n_x, n_y, n_z, mask=mask, return_as=return_as, dtype=dtype)


def _compute_n_patches(i_h, i_w, p_h, p_w, max_patches=None):
    total = (i_h - p_h + 1) * (i_w - p_w + 1)
    if not max_patches:
        return total
    if isinstance(max_patches, numbers.Integral):
        return min(max_patches, total)
    if isinstance(max_patches, numbers.Real) and 0 < max_patches < 1:
        return int(max_patches * total)
    raise ValueError("Invalid value for max_patches: %r" % max_patches)


def _extract_patches(arr, patch_shape=8, extraction_step=1):
    nd = arr.ndim
    if isinstance(patch_shape, numbers.Number):
        patch_shape = (patch_shape,) * nd
    if isinstance(extraction_step, numbers.Number):
        extraction_step = (extraction_step,) * nd
    istr = arr[tuple(slice(None, None, s) for s in extraction_step)].strides
    counts = (np.array(arr.shape) - np.array(patch_shape)) // np.array(extraction_step) + 1
    return as_strided(arr, shape=tuple(counts) + tuple(patch_shape),
                      strides=tuple(istr) + tuple(arr.strides))


def extract_patches_2d(image, patch_size, *, max_patches=None, random_state=None):
    """All (or ``max_patches`` random) ``patch_size`` patches of an image."""
    i_h, i_w = image.shape[:2]
    p_h, p_w = patch_size
    if p_h > i_h:
        raise ValueError("Height of the patch should be less than the height of the image.")
    if p_w > i_w:
        raise ValueError("Width of the patch should be less than the width of the image.")
    image = np.asarray(image)
    if image.dtype.kind not in "fiub":
        image = image.astype(np.float64)
    image = image.reshape((i_h, i_w, -1))
    nc = image.shape[-1]
    ext = _extract_patches(image, patch_shape=(p_h, p_w, nc), extraction_step=1)
    n = _compute_n_patches(i_h, i_w, p_h, p_w, max_patches)
    if max_patches:
        rng = check_random_state(random_state)
        i_s = rng.randint(i_h - p_h + 1, size=n)
        j_s = rng.randint(i_w - p_w + 1, size=n)
        patches = ext[i_s, j_s, 0]
    else:
        patches = ext
    patches = patches.reshape(-1, p_h, p_w, nc)
    return patches.reshape((n, p_h, p_w)) if patches.shape[-1] == 1 else patches


def reconstruct_from_patches_2d(patches, image_size):
    """Average overlapping patches back into an image."""
    i_h, i_w = image_size[:2]
    p_h, p_w = patches.shape[1:3]
    img = np.zeros(image_size)
    n_h, n_w = i_h - p_h + 1, i_w - p_w + 1
    for p, (i, j) in zip(patches, product(range(n_h), range(n_w))):
        img[i:i + p_h, j:j + p_w] += p
    ch = np.minimum(np.minimum(np.arange(i_h) + 1, p_h), i_h - np.arange(i_h))
    cw = np.minimum(np.minimum(np.arange(i_w) + 1, p_w), i_w - np.arange(i_w))
    cnt = np.outer(ch, cw).astype(float)
    return img / (cnt if img.ndim == 2 else cnt[:, :, None])


class PatchExtractor(BaseEstimator):
    """Extract patches from a collection of images."""

    def __init__(self, *, patch_size=None, max_patches=None, random_state=None):
        self.patch_size = patch_size
        self.max_patches = max_patches
        self.random_state = random_state

    def fit(self, X, y=None):
        return self

    def transform(self, X):
        self.random_state = check_random_state(self.random_state)
        n_img, i_h, i_w = X.shape[:3]
        X = np.reshape(X, (n_img, i_h, i_w, -1))
        nc = X.shape[-1]
        ps = (i_h // 10, i_w // 10) if self.patch_size is None else tuple(self.patch_size)
        n = _compute_n_patches(i_h, i_w, ps[0], ps[1], self.max_patches)
        shape = (n_img * n,) + ps + ((nc,) if nc > 1 else ())
        out = np.empty(shape)
        for k, im in enumerate(X):
            out[k * n:(k + 1) * n] = extract_patches_2d(im, ps, max_patches=self.max_patches,
                                                        random_state=self.random_state)
        return out

    def _more_tags(self):
        return {"X_types": ["3darray"]}
