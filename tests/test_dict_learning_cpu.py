"""Sparse coding / dictionary learning / SparsePCA (reference
``decomposition/_dict_learning.py``, ``_sparse_pca.py``).  Batch paths match
sklearn exactly; the online (mini-batch) learner follows the reference 1.0
algorithm, which sklearn >= 1.1 replaced, so it is checked for behaviour
(parity unpinned)."""
import warnings

import numpy as np
import pytest

import sq_learn_amd.decomposition as Q

S = pytest.importorskip("sklearn.decomposition")


@pytest.fixture(scope="module")
def data():
    rng = np.random.RandomState(0)
    X = rng.randn(40, 12)
    D = rng.randn(8, 12)
    return X, D / np.linalg.norm(D, axis=1, keepdims=True)


@pytest.mark.parametrize("alg,pos", [("lasso_lars", False), ("lasso_lars", True),
                                     ("lasso_cd", False), ("lasso_cd", True), ("lars", False),
                                     ("omp", False), ("threshold", False), ("threshold", True)])
def test_sparse_encode_parity(data, alg, pos):
    X, D = data
    kw = (dict(algorithm=alg, n_nonzero_coefs=3) if alg in ("lars", "omp")
          else dict(algorithm=alg, alpha=0.5, positive=pos))
    np.testing.assert_allclose(S.sparse_encode(X, D, **kw), Q.sparse_encode(X, D, **kw),
                               atol=1e-10)


def test_positive_rejected(data):
    X, D = data
    with pytest.raises(ValueError):
        Q.sparse_encode(X, D, algorithm="omp", positive=True)


def test_sparse_coder_split_sign(data):
    X, D = data
    kw = dict(transform_algorithm="lasso_lars", transform_alpha=0.3, split_sign=True)
    np.testing.assert_allclose(S.SparseCoder(D, **kw).transform(X),
                               Q.SparseCoder(D, **kw).transform(X), atol=1e-10)


@pytest.mark.parametrize("alg", ["lars", "cd"])
@pytest.mark.parametrize("pd", [False, True])
def test_dictionary_learning_parity(data, alg, pd):
    X, _ = data
    kw = dict(alpha=0.5, max_iter=20, random_state=0, fit_algorithm=alg, positive_dict=pd)
    a = S.DictionaryLearning(6, **kw).fit(X)
    b = Q.DictionaryLearning(6, **kw).fit(X)
    np.testing.assert_allclose(a.components_, b.components_, atol=1e-10)
    np.testing.assert_allclose(a.error_, b.error_, rtol=1e-10)
    assert np.all(np.diff(b.error_) <= 1e-9)


def test_sparse_pca_parity(data):
    X, _ = data
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a = S.SparsePCA(4, random_state=0).fit(X)
    b = Q.SparsePCA(4, random_state=0).fit(X)
    np.testing.assert_allclose(np.abs(a.components_), np.abs(b.components_), atol=1e-10)
    assert a.n_iter_ == b.n_iter_
    np.testing.assert_allclose(np.abs(a.transform(X)), np.abs(b.transform(X)), atol=1e-8)


def test_online_learners(data):
    X, _ = data
    m = Q.MiniBatchDictionaryLearning(6, alpha=0.5, n_iter=60, random_state=0).fit(X)
    assert m.components_.shape == (6, 12)
    np.testing.assert_allclose(np.linalg.norm(m.components_, axis=1), 1.0, atol=1e-8)
    code = m.transform(X)
    assert code.shape == (40, 6)
    off = m.iter_offset_
    m.partial_fit(X[:10])
    assert m.iter_offset_ == off + 1
    m2 = Q.MiniBatchDictionaryLearning(6, alpha=0.5, n_iter=60, random_state=0).fit(X)
    np.testing.assert_array_equal(m2.components_, Q.MiniBatchDictionaryLearning(
        6, alpha=0.5, n_iter=60, random_state=0).fit(X).components_)
    p = Q.MiniBatchSparsePCA(4, random_state=0, n_iter=20).fit(X)
    assert p.components_.shape == (4, 12) and p.transform(X).shape == (40, 4)
    code, dic = Q.dict_learning_online(X, 5, alpha=0.1, n_iter=100, random_state=0)
    # the online dictionary explains the data better than the zero model
    assert np.linalg.norm(X - code @ dic) < np.linalg.norm(X)
