"""Dataset generators and bundled toy datasets against scikit-learn
(reference sklearn/datasets/_samples_generator.py, _base.py).  Same
random_state -> same arrays.  make_sparse_spd_matrix follows the
reference's dense algorithm (sklearn>=1.3 changed it: parity unpinned)."""
import warnings

import numpy as np
import pytest

pytest.importorskip("sklearn")
import sklearn.datasets as S  # noqa: E402

import sq_learn_amd.datasets as M  # noqa: E402


def _same(a, b):
    a = a if isinstance(a, tuple) else (a,)
    b = b if isinstance(b, tuple) else (b,)
    assert len(a) == len(b)
    for x, y in zip(a, b):
        x = x.toarray() if hasattr(x, "toarray") else x
        y = y.toarray() if hasattr(y, "toarray") else y
        np.testing.assert_allclose(np.asarray(y, float), np.asarray(x, float), atol=1e-12)


@pytest.mark.parametrize("name,kw", [
    ("make_multilabel_classification", {}),
    ("make_multilabel_classification", dict(sparse=True, return_indicator="sparse",
                                            allow_unlabeled=False)),
    ("make_hastie_10_2", dict(n_samples=100)),
    ("make_regression", dict(n_samples=50, n_features=8, noise=1.0, coef=True)),
    ("make_regression", dict(n_samples=50, n_features=8, effective_rank=3, n_targets=2)),
    ("make_circles", dict(noise=0.1)), ("make_moons", dict(noise=0.1)),
    ("make_friedman1", dict(noise=0.5)), ("make_friedman2", {}), ("make_friedman3", {}),
    ("make_sparse_uncorrelated", {}), ("make_swiss_roll", dict(noise=0.1)),
    ("make_s_curve", dict(noise=0.1)), ("make_gaussian_quantiles", {})])
def test_generators(name, kw):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        _same(getattr(S, name)(random_state=0, **kw), getattr(M, name)(random_state=0, **kw))


def test_matrix_generators():
    _same(S.make_spd_matrix(5, random_state=0), M.make_spd_matrix(5, random_state=0))
    _same(S.make_biclusters((20, 10), 3, noise=0.5, random_state=0),
          M.make_biclusters((20, 10), 3, noise=0.5, random_state=0))
    _same(S.make_checkerboard((20, 10), (2, 3), noise=0.5, random_state=0),
          M.make_checkerboard((20, 10), (2, 3), noise=0.5, random_state=0))
    a = S.make_sparse_coded_signal(10, n_components=8, n_features=6, n_nonzero_coefs=3,
                                   random_state=0)
    b = M.make_sparse_coded_signal(10, n_components=8, n_features=6, n_nonzero_coefs=3,
                                   random_state=0)
    for x, y in zip(a, b):   # sklearn>=1.3 returns the transposed layout
        assert (x.shape == y.shape and np.allclose(x, y)) or np.allclose(x, y.T)
    p = M.make_sparse_spd_matrix(8, alpha=0.5, norm_diag=True, random_state=0)
    assert np.allclose(p, p.T) and np.all(np.linalg.eigvalsh(p) > 0)


@pytest.mark.parametrize("loader", ["load_iris", "load_wine", "load_breast_cancer", "load_digits",
                                    "load_diabetes", "load_linnerud"])
def test_toy_loaders(loader):
    a, b = getattr(S, loader)(), getattr(M, loader)()
    # sklearn>=1.1 re-derives the scaled diabetes features (~1e-5 drift)
    np.testing.assert_allclose(b.data, a.data, atol=2e-5)
    np.testing.assert_allclose(b.target, a.target)
    assert list(a.feature_names) == list(b.feature_names)
    fa, fb = getattr(S, loader)(as_frame=True).frame, getattr(M, loader)(as_frame=True).frame
    assert list(fa.columns) == list(fb.columns)
    X, y = getattr(M, loader)(return_X_y=True)
    assert X.shape[0] == y.shape[0]
