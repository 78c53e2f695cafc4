"""API substrate on the CPU path: model selection, preprocessing, pipeline,
MiniBatchKMeans, IncrementalPCA, pairwise/metrics parity with scikit-learn,
and an estimator-contract sweep over ``all_estimators()`` (the analogue of
the reference's ``test_common.py`` / ``estimator_checks.py``; SURVEY.md §4
item 4)."""
import inspect
import pickle
import warnings

import numpy as np
import pytest

sk = pytest.importorskip("sklearn")
import sklearn.decomposition as skd  # noqa: E402
import sklearn.metrics as skm  # noqa: E402
import sklearn.metrics.pairwise as skp  # noqa: E402
import sklearn.model_selection as skms  # noqa: E402
import sklearn.preprocessing as skpre  # noqa: E402
import sklearn.pipeline  # noqa: E402,F401
import sklearn.cluster  # noqa: E402,F401
import sklearn.neighbors  # noqa: E402,F401

from sq_learn_amd.base import clone  # noqa: E402
from sq_learn_amd.cluster import KMeans, MiniBatchKMeans, QMeans  # noqa: E402
from sq_learn_amd.decomposition import PCA, QPCA, IncrementalPCA  # noqa: E402
from sq_learn_amd.metrics import (accuracy_score, adjusted_rand_score, confusion_matrix,  # noqa: E402
                                  euclidean_distances, polynomial_kernel, r2_score, rbf_kernel,
                                  sigmoid_kernel, linear_kernel)
from sq_learn_amd.model_selection import (GridSearchCV, KFold, StratifiedKFold,  # noqa: E402
                                          cross_val_score, cross_validate, train_test_split)
from sq_learn_amd.neighbors import KNeighborsClassifier  # noqa: E402
from sq_learn_amd.pipeline import Pipeline, make_pipeline  # noqa: E402
from sq_learn_amd.preprocessing import MinMaxScaler, StandardScaler, normalize  # noqa: E402
from sq_learn_amd.utils import all_estimators  # noqa: E402
from sq_learn_amd.utils.datasets import make_blobs, make_classification  # noqa: E402


@pytest.fixture(scope="module")
def clf_data():
    return make_classification(n_samples=240, n_features=10, n_informative=6, n_classes=3,
                               random_state=0)


# ------------------------------------------------------------ model selection
@pytest.mark.parametrize("shuffle,rs", [(False, None), (True, 0), (True, 7)])
def test_kfold_matches_sklearn(shuffle, rs):
    X = np.zeros((23, 2))
    ours = list(KFold(4, shuffle=shuffle, random_state=rs).split(X))
    ref = list(skms.KFold(4, shuffle=shuffle, random_state=rs).split(X))
    for (a, b), (c, d) in zip(ours, ref):
        np.testing.assert_array_equal(a, c)
        np.testing.assert_array_equal(b, d)


@pytest.mark.parametrize("shuffle,rs", [(False, None), (True, 0), (True, 3)])
def test_stratified_kfold_matches_sklearn(shuffle, rs):
    y = np.array([0] * 11 + [1] * 7 + [2] * 5 + [1] * 4)
    X = np.zeros((len(y), 1))
    ours = list(StratifiedKFold(3, shuffle=shuffle, random_state=rs).split(X, y))
    ref = list(skms.StratifiedKFold(3, shuffle=shuffle, random_state=rs).split(X, y))
    for (a, b), (c, d) in zip(ours, ref):
        np.testing.assert_array_equal(np.sort(a), np.sort(c))
        np.testing.assert_array_equal(np.sort(b), np.sort(d))


def test_train_test_split_matches_sklearn(clf_data):
    X, y = clf_data
    ours = train_test_split(X, y, test_size=0.3, random_state=5)
    ref = skms.train_test_split(X, y, test_size=0.3, random_state=5)
    for a, b in zip(ours, ref):
        np.testing.assert_array_equal(a, b)
    Xtr, Xte, ytr, yte = train_test_split(X, y, test_size=0.25, random_state=1, stratify=y)
    assert len(Xte) == 60 and len(Xtr) == 180
    for c in np.unique(y):
        assert abs(np.mean(yte == c) - np.mean(y == c)) < 0.03


def test_cross_validate_knn(clf_data):
    X, y = clf_data
    r = cross_validate(KNeighborsClassifier(5), X, y, cv=5, return_train_score=True)
    ref = skms.cross_validate(sk.neighbors.KNeighborsClassifier(5), X, y, cv=5,
                              return_train_score=True)
    np.testing.assert_allclose(r["test_score"], ref["test_score"])
    np.testing.assert_allclose(r["train_score"], ref["train_score"])
    assert r["fit_time"].shape == (5,)
    s = cross_val_score(KNeighborsClassifier(3), X, y, cv=KFold(4), scoring="accuracy")
    assert s.shape == (4,) and np.all((0 <= s) & (s <= 1))


def test_grid_search(clf_data):
    X, y = clf_data
    gs = GridSearchCV(KNeighborsClassifier(), {"n_neighbors": [1, 5, 15]}, cv=3).fit(X, y)
    assert gs.best_params_["n_neighbors"] in (1, 5, 15)
    assert gs.cv_results_["rank_test_score"].min() == 1
    assert gs.score(X, y) >= gs.best_score_ - 0.2


# -------------------------------------------------------------- preprocessing
def test_standard_scaler_matches_sklearn(clf_data):
    X, _ = clf_data
    ours = StandardScaler().fit(X)
    ref = skpre.StandardScaler().fit(X)
    np.testing.assert_allclose(ours.mean_, ref.mean_)
    np.testing.assert_allclose(ours.scale_, ref.scale_)
    np.testing.assert_allclose(ours.transform(X), ref.transform(X), atol=1e-12)
    np.testing.assert_allclose(ours.inverse_transform(ours.transform(X)), X, atol=1e-12)
    # streaming partial_fit == one-shot fit
    p = StandardScaler()
    for s in range(0, len(X), 37):
        p.partial_fit(X[s:s + 37])
    np.testing.assert_allclose(p.mean_, ours.mean_, rtol=1e-12)
    np.testing.assert_allclose(p.var_, ours.var_, rtol=1e-10)
    assert p.n_samples_seen_ == len(X)


def test_minmax_and_normalize(clf_data):
    X, _ = clf_data
    np.testing.assert_allclose(MinMaxScaler((-1, 2)).fit_transform(X),
                               skpre.MinMaxScaler((-1, 2)).fit_transform(X), atol=1e-12)
    for nrm in ("l1", "l2", "max"):
        np.testing.assert_allclose(normalize(X, nrm), skpre.normalize(X, nrm), atol=1e-12)


# ---------------------------------------------------------------- pipeline
def test_pipeline_qpca_knn(clf_data):
    X, y = clf_data
    pipe = Pipeline([("sc", StandardScaler()), ("pca", QPCA(n_components=5, svd_solver="full")),
                     ("knn", KNeighborsClassifier(3))])
    pipe.fit(X, y)
    assert pipe.score(X, y) > 0.8
    assert pipe.get_params()["pca__n_components"] == 5
    pipe.set_params(knn__n_neighbors=7)
    assert pipe.named_steps["knn"].n_neighbors == 7
    c = clone(pipe)
    assert c.named_steps["knn"] is not pipe.named_steps["knn"]
    r = cross_val_score(pipe, X, y, cv=3)
    assert r.mean() > 0.6


def test_make_pipeline_cluster():
    X, y = make_blobs(n_samples=300, centers=4, random_state=0)
    p = make_pipeline(StandardScaler(), KMeans(4, n_init=3, random_state=0))
    lab = p.fit_predict(X)
    ref = sk.pipeline.make_pipeline(skpre.StandardScaler(),
                                    sk.cluster.KMeans(4, n_init=3, random_state=0)).fit_predict(X)
    assert adjusted_rand_score(y, lab) >= adjusted_rand_score(y, ref) - 0.05
    assert [n for n, _ in p.steps] == ["standardscaler", "kmeans"]


# ------------------------------------------------------- minibatch / ipca
def test_minibatch_kmeans_quality():
    X, y = make_blobs(n_samples=3000, centers=5, cluster_std=0.6, random_state=1)
    mb = MiniBatchKMeans(5, batch_size=256, random_state=0, n_init=3).fit(X)
    km = sk.cluster.KMeans(5, n_init=5, random_state=0).fit(X)
    assert mb.inertia_ <= 1.1 * km.inertia_
    assert adjusted_rand_score(y, mb.labels_) > 0.95
    np.testing.assert_array_equal(mb.predict(X), mb.labels_)
    p = MiniBatchKMeans(5, random_state=0)
    for s in range(0, 3000, 300):
        p.partial_fit(X[s:s + 300])
    assert p.cluster_centers_.shape == (5, 2)
    assert p.score(X) > -2 * km.inertia_


def test_incremental_pca_matches_sklearn():
    rng = np.random.RandomState(0)
    X = rng.randn(500, 12) @ rng.randn(12, 12)
    ours = IncrementalPCA(n_components=6, batch_size=100).fit(X)
    ref = skd.IncrementalPCA(n_components=6, batch_size=100).fit(X)
    np.testing.assert_allclose(ours.explained_variance_, ref.explained_variance_, rtol=1e-8)
    np.testing.assert_allclose(np.abs(ours.components_), np.abs(ref.components_), atol=1e-8)
    np.testing.assert_allclose(ours.mean_, ref.mean_)
    np.testing.assert_allclose(np.abs(ours.transform(X)), np.abs(ref.transform(X)), atol=1e-7)
    full = PCA(n_components=6).fit(X)
    np.testing.assert_allclose(ours.explained_variance_, full.explained_variance_, rtol=1e-2)


# ------------------------------------------------------ pairwise / metrics
def test_pairwise_matches_sklearn():
    rng = np.random.RandomState(0)
    A, B = rng.randn(40, 7), rng.randn(30, 7)
    np.testing.assert_allclose(euclidean_distances(A, B), skp.euclidean_distances(A, B), atol=1e-10)
    np.testing.assert_allclose(euclidean_distances(A), skp.euclidean_distances(A), atol=1e-7)
    np.testing.assert_allclose(rbf_kernel(A, B, gamma=0.3), skp.rbf_kernel(A, B, gamma=0.3),
                               atol=1e-12)
    np.testing.assert_allclose(polynomial_kernel(A, B), skp.polynomial_kernel(A, B), rtol=1e-10)
    np.testing.assert_allclose(sigmoid_kernel(A, B), skp.sigmoid_kernel(A, B), atol=1e-12)
    np.testing.assert_allclose(linear_kernel(A, B), skp.linear_kernel(A, B), atol=1e-12)


def test_metrics_match_sklearn():
    rng = np.random.RandomState(1)
    a, b = rng.randint(0, 4, 200), rng.randint(0, 4, 200)
    assert accuracy_score(a, b) == skm.accuracy_score(a, b)
    np.testing.assert_array_equal(confusion_matrix(a, b), skm.confusion_matrix(a, b))
    assert np.isclose(adjusted_rand_score(a, b), skm.adjusted_rand_score(a, b))
    u, v = rng.randn(50), rng.randn(50)
    assert np.isclose(r2_score(u, v), skm.r2_score(u, v))


# ------------------------------------------------------ estimator contract
_DATA = make_classification(n_samples=60, n_features=6, n_informative=4, n_classes=2,
                            random_state=0)


def _instance(cls):
    kw = {}
    name = cls.__name__
    if name in ("KMeans", "qMeans_", "QMeans", "MiniBatchKMeans"):
        kw = {"n_clusters": 3, "random_state": 0}
        if name != "MiniBatchKMeans":
            kw["n_init"] = 1
    elif name in ("PCA", "qPCA", "QPCA", "IncrementalPCA", "TruncatedSVD"):
        kw = {"n_components": 3}
    elif name == "Pipeline":
        return Pipeline([("sc", StandardScaler()), ("knn", KNeighborsClassifier(3))])
    elif name in ("GaussianRandomProjection", "SparseRandomProjection", "SelectKBest"):
        kw = {"n_components": 3} if name != "SelectKBest" else {"k": 3}
    elif name in ("SpectralBiclustering", "SpectralCoclustering"):
        kw = {"n_clusters": 2, "random_state": 0, "n_init": 2}
    elif name == "SparseCoder":
        return cls(np.eye(6)[:4], transform_algorithm="threshold", transform_alpha=0.1)
    elif name in ("DictionaryLearning", "MiniBatchDictionaryLearning", "SparsePCA",
                  "MiniBatchSparsePCA"):
        kw = {"n_components": 3, "random_state": 0}
        kw.update({"max_iter": 5} if name in ("DictionaryLearning", "SparsePCA")
                  else {"n_iter": 5})
    elif name == "ColumnTransformer":
        return cls([("sc", StandardScaler(), [0, 1, 2])], remainder="passthrough")
    elif name == "FeatureUnion":
        return cls([("sc", StandardScaler()), ("sc2", StandardScaler(with_mean=False))])
    elif name in ("VotingClassifier", "StackingClassifier"):
        from sq_learn_amd.naive_bayes import GaussianNB
        return cls([("a", GaussianNB()), ("b", KNeighborsClassifier(3))])
    elif name in ("VotingRegressor", "StackingRegressor"):
        from sq_learn_amd.linear_model import Ridge
        return cls([("a", Ridge()), ("b", Ridge(alpha=10.0))])
    elif name in ("GridSearchCV", "HalvingGridSearchCV"):
        return cls(KNeighborsClassifier(), {"n_neighbors": [1, 3]}, cv=3)
    elif name in ("RandomizedSearchCV", "HalvingRandomSearchCV"):
        return cls(KNeighborsClassifier(), {"n_neighbors": [1, 3, 5]}, cv=3, random_state=0)
    params = inspect.signature(cls.__init__).parameters
    for arg in ("estimator", "base_estimator"):
        if arg in params and params[arg].default is inspect.Parameter.empty:
            from sq_learn_amd.linear_model import LogisticRegression, Ridge
            kw[arg] = Ridge() if "Regressor" in name else LogisticRegression()
    return cls(**kw)


# estimators that only accept non-negative features
_NONNEG = ("CategoricalNB", "ComplementNB", "MultinomialNB", "AdditiveChi2Sampler",
           "SkewedChi2Sampler", "NMF", "LatentDirichletAllocation", "TfidfTransformer",
           "BernoulliRBM")


_MULTI_OUTPUT = ("MultiOutputClassifier", "MultiOutputRegressor", "ClassifierChain",
                 "RegressorChain", "CCA", "PLSCanonical", "PLSSVD", "MultiTaskElasticNet",
                 "MultiTaskLasso", "MultiTaskElasticNetCV", "MultiTaskLassoCV")


def _X(name):
    X = _DATA[0]
    return np.round(np.abs(X) * 2) if name in _NONNEG else X


_LABEL_TRANSFORMERS = ("LabelEncoder", "LabelBinarizer", "MultiLabelBinarizer")
_DOCS = ["the quick brown fox", "a lazy dog sleeps", "the fox and the dog", "quick quick fox"]
_SPECIAL_INPUT = {
    "CountVectorizer": _DOCS, "TfidfVectorizer": _DOCS, "HashingVectorizer": _DOCS,
    "DictVectorizer": [{"a": 1.0, "b": "x"}, {"a": 2.0, "c": 3.0}],
    "PatchExtractor": np.arange(2 * 20 * 20, dtype=float).reshape(2, 20, 20),
}


def _fit(est):
    X, y = _DATA
    name = type(est).__name__
    X = _X(name)
    if name in _LABEL_TRANSFORMERS:
        return est.fit([[v] for v in y] if name == "MultiLabelBinarizer" else y)
    if name == "IsotonicRegression":
        return est.fit(X[:, 0], X[:, 1])
    if name == "FeatureHasher":
        return est.fit()
    if name in _SPECIAL_INPUT:
        return est.fit(_SPECIAL_INPUT[name])
    if name in ("LSSVC", "QLSSVC"):
        return est.fit(X, np.where(y == 0, -1.0, 1.0))
    if name in _MULTI_OUTPUT:
        return est.fit(X, np.c_[y, 1 - y])
    if name in ("GammaRegressor", "PoissonRegressor", "TweedieRegressor"):
        return est.fit(X, y + 1.0)
    if name in ("KNeighborsClassifier", "KNeighborsRegressor", "Pipeline") or \
            "estimator" in est.get_params(deep=False) or \
            "regressor" in est.get_params(deep=False):
        return est.fit(X, y)
    sig = inspect.signature(est.fit).parameters
    yp = sig.get("y", sig.get("Y"))
    if yp is not None and yp.default is inspect.Parameter.empty:
        return est.fit(X, y.astype(float) if getattr(est, "_estimator_type", "") == "regressor"
                       else y)
    return est.fit(X)


@pytest.mark.parametrize("name,cls", all_estimators(), ids=[n for n, _ in all_estimators()])
def test_estimator_contract(name, cls):
    est = _instance(cls)
    # get_params / set_params round trip and clone
    params = est.get_params()
    est.set_params(**{k: v for k, v in est.get_params(deep=False).items()})
    assert est.get_params().keys() == params.keys()
    c = clone(est)
    assert type(c) is type(est)
    repr(est)
    # pickle unfitted
    pickle.loads(pickle.dumps(est))
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        _fit(est)
    # fitted attributes survive a pickle round trip (checkpoint compatibility)
    est2 = pickle.loads(pickle.dumps(est))
    X, y = _X(name), _DATA[1]
    if name in _LABEL_TRANSFORMERS:
        yy = [[v] for v in y] if name == "MultiLabelBinarizer" else y
        np.testing.assert_array_equal(est.transform(yy), est2.transform(yy))
        return
    if name == "IsotonicRegression":
        X = X[:, 0]
    elif name == "FeatureHasher":
        X = [{"a": 1.0, "b": 2.0}, {"c": 3.0}]
    elif name in _SPECIAL_INPUT:
        X = _SPECIAL_INPUT[name]
    for meth in ("predict", "transform"):
        if hasattr(est, meth) and name not in ("Pipeline",) or (name == "Pipeline" and meth == "predict"):
            try:
                a = getattr(est, meth)(X)
            except (AttributeError, NotImplementedError):
                continue
            b = getattr(est2, meth)(X)
            if isinstance(a, dict):
                continue
            if hasattr(a, "toarray"):
                a, b = a.toarray(), b.toarray()
            np.testing.assert_allclose(np.asarray(a, dtype=float), np.asarray(b, dtype=float),
                                       atol=1e-8)
    # n_features_in_ checking
    if hasattr(est, "n_features_in_") and hasattr(est, "transform") and name not in (
            "Normalizer", "Pipeline"):
        with pytest.raises(ValueError):
            est.transform(X[:, :3])


def test_reference_layout_imports():
    from sq_learn_amd.QuantumUtility import Utility
    from sq_learn_amd.cluster import qMeans_  # noqa: F401
    from sq_learn_amd.decomposition import qPCA  # noqa: F401
    from sq_learn_amd.svm import QLSSVC  # noqa: F401
    assert hasattr(Utility, "amplitude_estimation") and hasattr(Utility, "tomography")
    assert QMeans is qMeans_
