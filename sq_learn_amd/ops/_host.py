"""Loader for the host-native library ``sq_learn_amd/_sq_host.so``
(``csrc/host/*.cpp``), bound with ctypes.

Same policy as the device layer (``_native.py``): the library is (re)built
in-tree when missing or stale and every op that has a host kernel calls it
- there is no Python re-implementation to fall back to.  ctypes releases
the GIL for the duration of each call.
"""

import ctypes
import os
import threading

import numpy as np

_lock = threading.Lock()
_lib = None

_P = ctypes.c_void_p
_LL = ctypes.c_longlong
_I = ctypes.c_int
_U = ctypes.c_uint32
_D = ctypes.c_double
_F = ctypes.c_float

_SIGS = {
    "sqh_murmur_i32": (None, [_P, _LL, _U, _P]),
    "sqh_mt_permutation_head": (_I, [_P, _P, _LL, _LL, _P]),
    "sqh_murmur_bytes": (None, [_P, _P, _LL, _U, _P]),
    "sqh_hash_features": (None, [_P, _P, _P, _LL, _LL, _I, _U, _P, _P]),
    "sqh_pava_f64": (None, [_P, _P, _LL]),
    "sqh_pava_f32": (None, [_P, _P, _LL]),
    "sqh_make_unique_f64": (_LL, [_P, _P, _P, _LL, _D, _P, _P, _P]),
    "sqh_make_unique_f32": (_LL, [_P, _P, _P, _LL, _F, _P, _P, _P]),
    "sqh_floyd_warshall": (None, [_P, _LL, _I]),
    "sqh_dijkstra": (None, [_P, _P, _P, _P, _P, _P, _LL, _I, _P]),
    "sqh_svml_parse": (_P, [_P, _LL, _I, _I, _I, _LL, _LL]),
    "sqh_svml_error": (ctypes.c_char_p, [_P]),
    "sqh_svml_sizes": (None, [_P, _P]),
    "sqh_svml_copy": (None, [_P, _P, _P, _P, _P, _P, _P]),
    "sqh_svml_free": (None, [_P]),
    "sqh_dbscan_inner": (None, [_P, _P, _P, _LL, _P]),
    "sqh_group_tiles": (_I, [_P, _LL, _I, _I, _P]),
    "sqh_expected_mutual_info": (_D, [_P, _LL, _P, _LL, _LL]),
    "sqh_sparse_manhattan": (None, [_P, _P, _P, _P, _P, _P, _LL, _LL, _P]),
    "sqh_cholesky_delete": (None, [_P, _LL, _LL, _LL]),
    "sqh_csr_poly": (_LL, [_P, _P, _P, _LL, _LL, _I, _I, _P, _P, _P]),
    "sqh_linkage": (_I, [_P, _LL, _I, _I, _P]),
    "sqh_tron": (_I, [_P, _LL, _LL, _P, _P, _I, _D, _D, _I, _P]),
    "sqh_tsne_bh_grad": (_D, [_P, _LL, _I, _P, _P, _P, _D, _D, _I, _P]),
    "sqh_enet_cd_dense": (None, [_P, _D, _D, _P, _P, _LL, _LL, _I, _D, _U, _I, _I, _P]),
    "sqh_enet_cd_gram": (None, [_P, _D, _D, _P, _P, _D, _LL, _I, _D, _U, _I, _I, _P]),
    "sqh_forest_build": (None, [_P, _P, _P, _LL, _LL, _I, _P, _LL, _P, _P, _I, _I, _P]),
    "sqh_tree_sizes": (None, [_P, _P]),
    "sqh_tree_copy": (None, [_P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "sqh_tree_free": (None, [_P]),
    "sqh_forest_apply": (None, [_P, _P, _P, _P, _P, _I, _P, _LL, _LL, _P]),
    "sqh_hgb_map_bins": (None, [_P, _LL, _I, _P, _P, _I, _P]),
    "sqh_hgb_grow": (_P, [_P, _LL, _I, _P, _P, _I, _P, _P, _P, _P, _P]),
    "sqh_hgb_copy_cat": (None, [_P, _P, _P]),
    "sqh_hgb_predict_cat": (None, [_P, _LL, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                   _I, _P]),
    "sqh_hgb_size": (_LL, [_P]),
    "sqh_hgb_copy": (None, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _LL]),
    "sqh_hgb_free": (None, [_P]),
    "sqh_svm_solve": (None, [_P, _LL, _P, _P, _P, _P, _LL, _D, _LL, _I, _I, _P, _P]),
    "sqh_svm_solve_rows": (None, [_P, _P, _P, _P, _LL, _LL, _I, _D, _D, _I, _LL, _P, _P, _P, _P,
                                  _LL, _D, _LL, _I, _I, _P, _P]),
    "sqh_svm_kernel_rows": (None, [_P, _P, _P, _P, _LL, _LL, _I, _D, _D, _I, _P, _LL, _P, _LL,
                                   _P]),
    "sqh_linear_svc_dual": (_I, [_P, _LL, _LL, _P, _P, _I, _D, _I, _P, _P, _P]),
    "sqh_linear_svr_dual": (_I, [_P, _LL, _LL, _P, _P, _I, _D, _D, _I, _P, _P]),
    "sqh_linear_mcsvm_cs": (_I, [_P, _LL, _LL, _P, _I, _P, _D, _I, _P, _P]),
    "sqh_sag": (_I, [_P, _P, _P, _LL, _LL, _I, _I, _D, _D, _D, _I, _D, _I, _D, _I, _U, _P, _P]),
    "sqh_mt_new": (_P, [_U]),
    "sqh_sgd_plain": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _U, _P]),
    "sqh_mt_free": (None, [_P]),
    "sqh_btree_build": (_P, [_P, _LL, _I, _I, _I, _D]),
    "sqh_btree_free": (None, [_P]),
    "sqh_btree_info": (None, [_P, _P]),
    "sqh_btree_copy": (None, [_P, _P, _P, _P, _P, _P, _P]),
    "sqh_btree_knn": (None, [_P, _P, _LL, _I, _P, _P, _I]),
    "sqh_btree_radius": (_P, [_P, _P, _LL, _P, _I, _I, _I, _P, _I]),
    "sqh_radius_copy": (None, [_P, _P, _P]),
    "sqh_radius_free": (None, [_P]),
    "sqh_cdnmf_update": (_D, [_P, _P, _P, _P, _LL, _LL]),
    "sqh_optics_order": (None, [_P, _LL, _LL, _P, _D, _D, _P, _P, _P]),
    "sqh_dirichlet_expectation_2d": (None, [_P, _LL, _LL, _P]),
    "sqh_lda_estep": (None, [_P, _P, _P, _LL, _I, _LL, _P, _D, _I, _D, _P, _P, _I]),
    "sqh_hgb_predict": (None, [_P, _LL, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P]),
}


def lib():
    """The loaded host library (built on first use if missing or stale)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            from .. import _build
            override = os.environ.get("SQ_HOST_LIB")   # e.g. the ASan build
            if override:
                h = ctypes.CDLL(override)
            else:
                if _build.host_needs_build():
                    _build.build_host()
                h = ctypes.CDLL(_build.host_path())
            for name, (res, args) in _SIGS.items():
                fn = getattr(h, name)
                fn.restype = res
                fn.argtypes = args
            _lib = h
    return _lib


def ptr(a):
    """Raw data pointer of a C-contiguous numpy array (None -> NULL)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "host kernels take C-contiguous arrays"
    return a.ctypes.data


def carray(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)
