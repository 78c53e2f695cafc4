"""Text vectorisation (reference ``feature_extraction/text.py``):
preprocessing / tokenisation / n-gram analysers, CountVectorizer,
HashingVectorizer, TfidfTransformer and TfidfVectorizer.

Analysis is string work and stays on the host; the document-term matrices
are scipy CSR, and the hashing path goes through the native
``sqh_hash_features`` kernel (``FeatureHasher``).  Vocabulary ordering,
pruning (``max_df`` / ``min_df`` / ``max_features`` tie-breaks) and idf
smoothing follow the reference exactly so the matrices are identical.
"""

import numbers
import re
import unicodedata
import warnings
from collections import defaultdict
from collections.abc import Mapping
from functools import partial
from operator import itemgetter

import numpy as np
import scipy.sparse as sp

from ..base import BaseEstimator, TransformerMixin
from ..exceptions import NotFittedError
from ._hash import FeatureHasher
from ._stop_words import ENGLISH_STOP_WORDS

__all__ = ["HashingVectorizer", "CountVectorizer", "ENGLISH_STOP_WORDS", "TfidfTransformer",
           "TfidfVectorizer", "strip_accents_ascii", "strip_accents_unicode", "strip_tags"]

_FLOATS = (np.float64, np.float32, np.float16)
_DEFAULT_TOKEN = r"(?u)\b\w\w+\b"
_SPACES = re.compile(r"\s\s+")


def strip_accents_unicode(s):
    """Decompose to NFKD and drop the combining characters."""
    try:
        s.encode("ASCII", errors="strict")
        return s
    except UnicodeEncodeError:
        return "".join(c for c in unicodedata.normalize("NFKD", s)
                       if not unicodedata.combining(c))


def strip_accents_ascii(s):
    """Transliterate to ASCII, dropping what has no ASCII form."""
    return unicodedata.normalize("NFKD", s).encode("ASCII", "ignore").decode("ASCII")


def strip_tags(s):
    """Replace ``<...>`` markup with a space."""
    return re.compile(r"<([^>]+)>", flags=re.UNICODE).sub(" ", s)


def _check_stop_list(stop):
    if stop == "english":
        return ENGLISH_STOP_WORDS
    if isinstance(stop, str):
        raise ValueError("not a built-in stop list: %s" % stop)
    return None if stop is None else frozenset(stop)


def _preprocess(doc, accent_function=None, lower=False):
    if lower:
        doc = doc.lower()
    if accent_function is not None:
        doc = accent_function(doc)
    return doc


def _analyze(doc, analyzer=None, tokenizer=None, ngrams=None, preprocessor=None, decoder=None,
             stop_words=None):
    if decoder is not None:
        doc = decoder(doc)
    if analyzer is not None:
        return analyzer(doc)
    if preprocessor is not None:
        doc = preprocessor(doc)
    if tokenizer is not None:
        doc = tokenizer(doc)
    if ngrams is not None:
        doc = ngrams(doc, stop_words) if stop_words is not None else ngrams(doc)
    return doc


def _normalize_rows(X, norm):
    """In-place row normalisation of a CSR matrix."""
    X = X.tocsr()
    counts = np.diff(X.indptr)
    rows = np.repeat(np.arange(X.shape[0]), counts)
    if norm == "l1":
        r = np.bincount(rows, np.abs(X.data), minlength=X.shape[0])
    elif norm == "l2":
        r = np.sqrt(np.bincount(rows, X.data * X.data, minlength=X.shape[0]))
    elif norm == "max":
        r = np.zeros(X.shape[0])
        np.maximum.at(r, rows, np.abs(X.data))
    else:
        raise ValueError("'%s' is not a supported norm" % norm)
    r[r == 0] = 1.0
    X.data /= r[rows]
    return X


def _document_frequency(X):
    if sp.isspmatrix_csr(X) or isinstance(X, sp.csr_array):
        return np.bincount(X.indices, minlength=X.shape[1])
    return np.diff(sp.csc_matrix(X).indptr)


class _VectorizerMixin:
    """Shared analysis machinery of the vectorisers."""

    _white_spaces = _SPACES

    def decode(self, doc):
        if self.input == "filename":
            with open(doc, "rb") as fh:
                doc = fh.read()
        elif self.input == "file":
            doc = doc.read()
        if isinstance(doc, bytes):
            doc = doc.decode(self.encoding, self.decode_error)
        if doc is np.nan:
            raise ValueError("np.nan is an invalid document, expected byte or unicode string.")
        return doc

    def _word_ngrams(self, tokens, stop_words=None):
        if stop_words is not None:
            tokens = [w for w in tokens if w not in stop_words]
        lo, hi = self.ngram_range
        if hi == 1:
            return tokens
        orig = tokens
        if lo == 1:
            tokens = list(orig)
            lo += 1
        else:
            tokens = []
        m = len(orig)
        for n in range(lo, min(hi + 1, m + 1)):
            tokens.extend(" ".join(orig[i:i + n]) for i in range(m - n + 1))
        return tokens

    def _char_ngrams(self, text):
        text = _SPACES.sub(" ", text)
        m = len(text)
        lo, hi = self.ngram_range
        if lo == 1:
            grams = list(text)
            lo += 1
        else:
            grams = []
        for n in range(lo, min(hi + 1, m + 1)):
            grams.extend(text[i:i + n] for i in range(m - n + 1))
        return grams

    def _char_wb_ngrams(self, text):
        text = _SPACES.sub(" ", text)
        lo, hi = self.ngram_range
        grams = []
        for w in text.split():
            w = " " + w + " "
            wl = len(w)
            for n in range(lo, hi + 1):
                off = 0
                grams.append(w[off:off + n])
                while off + n < wl:
                    off += 1
                    grams.append(w[off:off + n])
                if off == 0:  # short word: counted once
                    break
        return grams

    def build_preprocessor(self):
        if self.preprocessor is not None:
            return self.preprocessor
        if not self.strip_accents:
            acc = None
        elif callable(self.strip_accents):
            acc = self.strip_accents
        elif self.strip_accents == "ascii":
            acc = strip_accents_ascii
        elif self.strip_accents == "unicode":
            acc = strip_accents_unicode
        else:
            raise ValueError('Invalid value for "strip_accents": %s' % self.strip_accents)
        return partial(_preprocess, accent_function=acc, lower=self.lowercase)

    def build_tokenizer(self):
        if self.tokenizer is not None:
            return self.tokenizer
        pat = re.compile(self.token_pattern)
        if pat.groups > 1:
            raise ValueError("More than 1 capturing group in token pattern. Only a single group "
                             "should be captured.")
        return pat.findall

    def get_stop_words(self):
        return _check_stop_list(self.stop_words)

    def _check_stop_words_consistency(self, stop_words, preprocess, tokenize):
        if id(stop_words) == getattr(self, "_stop_words_id", None):
            return None
        try:
            bad = set()
            for w in stop_words or ():
                for tok in tokenize(preprocess(w)):
                    if tok not in stop_words:
                        bad.add(tok)
            self._stop_words_id = id(stop_words)
            if bad:
                warnings.warn("Your stop_words may be inconsistent with your preprocessing. "
                              "Tokenizing the stop words generated tokens %r not in stop_words."
                              % sorted(bad))
            return not bad
        except Exception:
            self._stop_words_id = id(stop_words)
            return "error"

    def build_analyzer(self):
        if callable(self.analyzer):
            return partial(_analyze, analyzer=self.analyzer, decoder=self.decode)
        pre = self.build_preprocessor()
        if self.analyzer == "char":
            return partial(_analyze, ngrams=self._char_ngrams, preprocessor=pre,
                           decoder=self.decode)
        if self.analyzer == "char_wb":
            return partial(_analyze, ngrams=self._char_wb_ngrams, preprocessor=pre,
                           decoder=self.decode)
        if self.analyzer == "word":
            stop = self.get_stop_words()
            tok = self.build_tokenizer()
            self._check_stop_words_consistency(stop, pre, tok)
            return partial(_analyze, ngrams=self._word_ngrams, tokenizer=tok, preprocessor=pre,
                           decoder=self.decode, stop_words=stop)
        raise ValueError("%s is not a valid tokenization scheme/analyzer" % self.analyzer)

    def _validate_vocabulary(self):
        vocab = self.vocabulary
        if vocab is None:
            self.fixed_vocabulary_ = False
            return
        if isinstance(vocab, set):
            vocab = sorted(vocab)
        if not isinstance(vocab, Mapping):
            v = {}
            for i, t in enumerate(vocab):
                if v.setdefault(t, i) != i:
                    raise ValueError("Duplicate term in vocabulary: %r" % t)
            vocab = v
        else:
            idx = set(vocab.values())
            if len(idx) != len(vocab):
                raise ValueError("Vocabulary contains repeated indices.")
            for i in range(len(vocab)):
                if i not in idx:
                    raise ValueError("Vocabulary of size %d doesn't contain index %d."
                                     % (len(vocab), i))
        if not vocab:
            raise ValueError("empty vocabulary passed to fit")
        self.fixed_vocabulary_ = True
        self.vocabulary_ = dict(vocab)

    def _check_vocabulary(self):
        if not hasattr(self, "vocabulary_"):
            self._validate_vocabulary()
            if not self.fixed_vocabulary_:
                raise NotFittedError("Vocabulary not fitted or provided")
        if len(self.vocabulary_) == 0:
            raise ValueError("Vocabulary is empty")

    def _validate_params(self):
        lo, hi = self.ngram_range
        if lo > hi:
            raise ValueError("Invalid value for ngram_range=%s lower boundary larger than the "
                             "upper boundary." % str(self.ngram_range))

    def _warn_for_unused_params(self):
        if self.tokenizer is not None and self.token_pattern is not None:
            warnings.warn("The parameter 'token_pattern' will not be used since 'tokenizer' is "
                          "not None'")
        if self.preprocessor is not None and callable(self.analyzer):
            warnings.warn("The parameter 'preprocessor' will not be used since 'analyzer' is "
                          "callable'")
        if self.ngram_range not in ((1, 1), None) and callable(self.analyzer):
            warnings.warn("The parameter 'ngram_range' will not be used since 'analyzer' is "
                          "callable'")
        if self.analyzer != "word" or callable(self.analyzer):
            if self.stop_words is not None:
                warnings.warn("The parameter 'stop_words' will not be used since 'analyzer' != "
                              "'word'")
            if self.token_pattern is not None and self.token_pattern != _DEFAULT_TOKEN:
                warnings.warn("The parameter 'token_pattern' will not be used since 'analyzer' "
                              "!= 'word'")
            if self.tokenizer is not None:
                warnings.warn("The parameter 'tokenizer' will not be used since 'analyzer' != "
                              "'word'")


class HashingVectorizer(TransformerMixin, _VectorizerMixin, BaseEstimator):
    """Stateless token-count hashing into ``n_features`` columns."""

    def __init__(self, *, input="content", encoding="utf-8", decode_error="strict",
                 strip_accents=None, lowercase=True, preprocessor=None, tokenizer=None,
                 stop_words=None, token_pattern=_DEFAULT_TOKEN, ngram_range=(1, 1),
                 analyzer="word", n_features=(2 ** 20), binary=False, norm="l2",
                 alternate_sign=True, dtype=np.float64):
        self.input = input
        self.encoding = encoding
        self.decode_error = decode_error
        self.strip_accents = strip_accents
        self.preprocessor = preprocessor
        self.tokenizer = tokenizer
        self.analyzer = analyzer
        self.lowercase = lowercase
        self.token_pattern = token_pattern
        self.stop_words = stop_words
        self.n_features = n_features
        self.ngram_range = ngram_range
        self.binary = binary
        self.norm = norm
        self.alternate_sign = alternate_sign
        self.dtype = dtype

    def partial_fit(self, X, y=None):
        return self

    def fit(self, X, y=None):
        if isinstance(X, str):
            raise ValueError("Iterable over raw text documents expected, string object "
                             "received.")
        self._warn_for_unused_params()
        self._validate_params()
        self._get_hasher().fit(X, y=y)
        return self

    def transform(self, X):
        if isinstance(X, str):
            raise ValueError("Iterable over raw text documents expected, string object "
                             "received.")
        self._validate_params()
        an = self.build_analyzer()
        M = self._get_hasher().transform(an(doc) for doc in X)
        if self.binary:
            M.data.fill(1)
        if self.norm is not None:
            M = _normalize_rows(M, self.norm)
        return M

    def fit_transform(self, X, y=None):
        return self.fit(X, y).transform(X)

    def _get_hasher(self):
        return FeatureHasher(n_features=self.n_features, input_type="string", dtype=self.dtype,
                             alternate_sign=self.alternate_sign)

    def _more_tags(self):
        return {"X_types": ["string"], "stateless": True}


class CountVectorizer(_VectorizerMixin, BaseEstimator):
    """Document-term count matrix over a learned (or given) vocabulary."""

    def __init__(self, *, input="content", encoding="utf-8", decode_error="strict",
                 strip_accents=None, lowercase=True, preprocessor=None, tokenizer=None,
                 stop_words=None, token_pattern=_DEFAULT_TOKEN, ngram_range=(1, 1),
                 analyzer="word", max_df=1.0, min_df=1, max_features=None, vocabulary=None,
                 binary=False, dtype=np.int64):
        self.input = input
        self.encoding = encoding
        self.decode_error = decode_error
        self.strip_accents = strip_accents
        self.preprocessor = preprocessor
        self.tokenizer = tokenizer
        self.analyzer = analyzer
        self.lowercase = lowercase
        self.token_pattern = token_pattern
        self.stop_words = stop_words
        self.max_df = max_df
        self.min_df = min_df
        self.max_features = max_features
        self.ngram_range = ngram_range
        self.vocabulary = vocabulary
        self.binary = binary
        self.dtype = dtype

    def _sort_features(self, X, vocab):
        order = sorted(vocab.items())
        remap = np.empty(len(order), dtype=X.indices.dtype)
        for new, (term, old) in enumerate(order):
            vocab[term] = new
            remap[old] = new
        X.indices = remap.take(X.indices, mode="clip")
        return X

    def _limit_features(self, X, vocab, high=None, low=None, limit=None):
        if high is None and low is None and limit is None:
            return X, set()
        dfs = _document_frequency(X)
        mask = np.ones(len(dfs), dtype=bool)
        if high is not None:
            mask &= dfs <= high
        if low is not None:
            mask &= dfs >= low
        if limit is not None and mask.sum() > limit:
            tfs = np.asarray(X.sum(axis=0)).ravel()
            keep = (-tfs[mask]).argsort()[:limit]
            m2 = np.zeros(len(dfs), dtype=bool)
            m2[np.where(mask)[0][keep]] = True
            mask = m2
        newidx = np.cumsum(mask) - 1
        removed = set()
        for term, old in list(vocab.items()):
            if mask[old]:
                vocab[term] = newidx[old]
            else:
                del vocab[term]
                removed.add(term)
        kept = np.where(mask)[0]
        if len(kept) == 0:
            raise ValueError("After pruning, no terms remain. Try a lower min_df or a higher "
                             "max_df.")
        return X[:, kept], removed

    def _count_vocab(self, docs, fixed_vocab):
        if fixed_vocab:
            vocab = self.vocabulary_
        else:
            vocab = defaultdict()
            vocab.default_factory = vocab.__len__
        analyze = self.build_analyzer()
        cols, vals, indptr = [], [], [0]
        for doc in docs:
            cnt = {}
            for feat in analyze(doc):
                try:
                    j = vocab[feat]
                except KeyError:
                    continue
                cnt[j] = cnt.get(j, 0) + 1
            cols.extend(cnt.keys())
            vals.extend(cnt.values())
            indptr.append(len(cols))
        if not fixed_vocab:
            vocab = dict(vocab)
            if not vocab:
                raise ValueError("empty vocabulary; perhaps the documents only contain stop "
                                 "words")
        itype = np.int32 if indptr[-1] <= np.iinfo(np.int32).max else np.int64
        X = sp.csr_matrix((np.asarray(vals, dtype=np.intc),
                           np.asarray(cols, dtype=itype), np.asarray(indptr, dtype=itype)),
                          shape=(len(indptr) - 1, len(vocab)), dtype=self.dtype)
        X.sort_indices()
        return vocab, X

    def fit(self, raw_documents, y=None):
        self._warn_for_unused_params()
        self.fit_transform(raw_documents)
        return self

    def fit_transform(self, raw_documents, y=None):
        if isinstance(raw_documents, str):
            raise ValueError("Iterable over raw text documents expected, string object "
                             "received.")
        self._validate_params()
        self._validate_vocabulary()
        hi, lo, mf = self.max_df, self.min_df, self.max_features
        if mf is not None and (not isinstance(mf, numbers.Integral) or mf <= 0):
            raise ValueError("max_features=%r, neither a positive integer nor None" % mf)
        vocab, X = self._count_vocab(raw_documents, self.fixed_vocabulary_)
        if self.binary:
            X.data.fill(1)
        if not self.fixed_vocabulary_:
            n = X.shape[0]
            hi_c = hi if isinstance(hi, numbers.Integral) else hi * n
            lo_c = lo if isinstance(lo, numbers.Integral) else lo * n
            if hi_c < lo_c:
                raise ValueError("max_df corresponds to < documents than min_df")
            if mf is not None:
                X = self._sort_features(X, vocab)
            X, self.stop_words_ = self._limit_features(X, vocab, hi_c, lo_c, mf)
            if mf is None:
                X = self._sort_features(X, vocab)
            self.vocabulary_ = vocab
        return X

    def transform(self, raw_documents):
        if isinstance(raw_documents, str):
            raise ValueError("Iterable over raw text documents expected, string object "
                             "received.")
        self._check_vocabulary()
        _, X = self._count_vocab(raw_documents, fixed_vocab=True)
        if self.binary:
            X.data.fill(1)
        return X

    def inverse_transform(self, X):
        self._check_vocabulary()
        terms = np.array(list(self.vocabulary_.keys()))
        inv = terms[np.argsort(np.array(list(self.vocabulary_.values())))]
        if sp.issparse(X):
            X = sp.csr_matrix(X)
            return [inv[X[i, :].nonzero()[1]].ravel() for i in range(X.shape[0])]
        X = np.asarray(X)
        if X.ndim != 2:
            raise ValueError("Expected 2D array, got %dD array instead" % X.ndim)
        return [inv[np.flatnonzero(X[i, :])].ravel() for i in range(X.shape[0])]

    def get_feature_names_out(self, input_features=None):
        self._check_vocabulary()
        return np.asarray([t for t, _ in sorted(self.vocabulary_.items(), key=itemgetter(1))],
                          dtype=object)

    def get_feature_names(self):
        """Deprecated alias of ``get_feature_names_out`` returning a list."""
        return list(self.get_feature_names_out())

    def _more_tags(self):
        return {"X_types": ["string"]}


class TfidfTransformer(TransformerMixin, BaseEstimator):
    """Count matrix -> (sublinear) tf times smoothed idf, row-normalised."""

    def __init__(self, *, norm="l2", use_idf=True, smooth_idf=True, sublinear_tf=False):
        self.norm = norm
        self.use_idf = use_idf
        self.smooth_idf = smooth_idf
        self.sublinear_tf = sublinear_tf

    def fit(self, X, y=None):
        X = X if sp.issparse(X) else sp.csr_matrix(np.asarray(X))
        dtype = X.dtype if X.dtype in _FLOATS else np.float64
        self.n_features_in_ = X.shape[1]
        if self.use_idf:
            n, d = X.shape
            df = _document_frequency(X).astype(dtype)
            df += int(self.smooth_idf)
            n += int(self.smooth_idf)
            self._idf = (np.log(n / df) + 1).astype(dtype)
        return self

    def transform(self, X, copy=True):
        if sp.issparse(X):
            X = sp.csr_matrix(X, dtype=X.dtype if X.dtype in _FLOATS else np.float64, copy=copy)
        else:
            X = sp.csr_matrix(np.asarray(X, dtype=np.float64))
        if self.sublinear_tf:
            np.log(X.data, X.data)
            X.data += 1
        if self.use_idf:
            if not hasattr(self, "_idf"):
                raise NotFittedError("idf vector is not fitted")
            if X.shape[1] != self._idf.shape[0]:
                raise ValueError("Input has n_features=%d while the model has been trained "
                                 "with n_features=%d" % (X.shape[1], self._idf.shape[0]))
            X = X @ sp.diags(self._idf, 0, shape=(X.shape[1],) * 2, format="csr")
        if self.norm:
            X = _normalize_rows(X, self.norm)
        return X

    @property
    def idf_(self):
        if not hasattr(self, "_idf"):
            raise AttributeError("idf_")
        return self._idf

    @idf_.setter
    def idf_(self, value):
        self._idf = np.asarray(value, dtype=np.float64)

    def _more_tags(self):
        return {"X_types": ["2darray", "sparse"]}


class TfidfVectorizer(CountVectorizer):
    """CountVectorizer followed by TfidfTransformer."""

    def __init__(self, *, input="content", encoding="utf-8", decode_error="strict",
                 strip_accents=None, lowercase=True, preprocessor=None, tokenizer=None,
                 analyzer="word", stop_words=None, token_pattern=_DEFAULT_TOKEN,
                 ngram_range=(1, 1), max_df=1.0, min_df=1, max_features=None, vocabulary=None,
                 binary=False, dtype=np.float64, norm="l2", use_idf=True, smooth_idf=True,
                 sublinear_tf=False):
        super().__init__(input=input, encoding=encoding, decode_error=decode_error,
                         strip_accents=strip_accents, lowercase=lowercase,
                         preprocessor=preprocessor, tokenizer=tokenizer, analyzer=analyzer,
                         stop_words=stop_words, token_pattern=token_pattern,
                         ngram_range=ngram_range, max_df=max_df, min_df=min_df,
                         max_features=max_features, vocabulary=vocabulary, binary=binary,
                         dtype=dtype)
        self.norm = norm
        self.use_idf = use_idf
        self.smooth_idf = smooth_idf
        self.sublinear_tf = sublinear_tf

    @property
    def idf_(self):
        return self._tfidf.idf_

    @idf_.setter
    def idf_(self, value):
        self._validate_vocabulary()
        if hasattr(self, "vocabulary_") and len(self.vocabulary_) != len(value):
            raise ValueError("idf length = %d must be equal to vocabulary size = %d"
                             % (len(value), len(self.vocabulary)))
        self._tfidf = TfidfTransformer(norm=self.norm, use_idf=self.use_idf,
                                       smooth_idf=self.smooth_idf,
                                       sublinear_tf=self.sublinear_tf)
        self._tfidf.idf_ = value

    def _check_params(self):
        if self.dtype not in _FLOATS:
            warnings.warn("Only {} 'dtype' should be used. {} 'dtype' will be converted to "
                          "np.float64.".format(_FLOATS, self.dtype), UserWarning)

    def _new_tfidf(self):
        self._tfidf = TfidfTransformer(norm=self.norm, use_idf=self.use_idf,
                                       smooth_idf=self.smooth_idf,
                                       sublinear_tf=self.sublinear_tf)

    def fit(self, raw_documents, y=None):
        self._check_params()
        self._warn_for_unused_params()
        self._new_tfidf()
        self._tfidf.fit(super().fit_transform(raw_documents))
        return self

    def fit_transform(self, raw_documents, y=None):
        self._check_params()
        self._new_tfidf()
        X = super().fit_transform(raw_documents)
        self._tfidf.fit(X)
        return self._tfidf.transform(X, copy=False)

    def transform(self, raw_documents):
        if not hasattr(self, "_tfidf"):
            raise NotFittedError("The TF-IDF vectorizer is not fitted")
        return self._tfidf.transform(super().transform(raw_documents), copy=False)

    def _more_tags(self):
        return {"X_types": ["string"], "_skip_test": True}
