"""Helpers for meta-estimators (reference ``utils/metaestimators.py``):
``_BaseComposition`` - parameter get/set for estimators that hold a list of
``(name, estimator)`` pairs - and ``available_if``, a descriptor that makes
a delegated method exist only when a check passes (so ``hasattr`` works
the way duck-typing callers expect)."""

from functools import update_wrapper

from ..base import BaseEstimator


class _BaseComposition(BaseEstimator):
    def _get_params(self, attr, deep=True):
        out = super().get_params(deep=False)
        if not deep:
            return out
        estimators = getattr(self, attr)
        try:
            out.update(estimators)
        except (TypeError, ValueError):
            return out
        for name, est in estimators:
            if hasattr(est, "get_params"):
                for k, v in est.get_params(deep=True).items():
                    out["%s__%s" % (name, k)] = v
        return out

    def _set_params(self, attr, **params):
        if attr in params:
            setattr(self, attr, params.pop(attr))
        items = getattr(self, attr)
        if isinstance(items, list) and items:
            try:
                names, _ = zip(*items)
            except (TypeError, ValueError):
                names = ()
            for name in list(params):
                if "__" not in name and name in names:
                    self._replace_estimator(attr, name, params.pop(name))
        own = super().get_params(deep=False)
        direct = {k: v for k, v in params.items() if "__" not in k and k in own}
        for k, v in direct.items():
            setattr(self, k, v)
            params.pop(k)
        nested = {}
        named = dict(getattr(self, attr))
        for key, value in params.items():
            name, delim, sub = key.partition("__")
            if not delim or name not in named:
                raise ValueError("Invalid parameter %r for estimator %s. Check the list of "
                                 "available parameters with `estimator.get_params().keys()`."
                                 % (key, type(self).__name__))
            nested.setdefault(name, {})[sub] = value
        for name, sub in nested.items():
            named[name].set_params(**sub)
        return self

    def _replace_estimator(self, attr, name, new_val):
        new = []
        for item in getattr(self, attr):
            if item[0] == name:
                new.append((name, new_val) + tuple(item[2:]))
            else:
                new.append(item)
        setattr(self, attr, new)

    def _validate_names(self, names):
        if len(set(names)) != len(names):
            raise ValueError("Names provided are not unique: {0!r}".format(list(names)))
        own = set(super().get_params(deep=False))
        clash = own.intersection(names)
        if clash:
            raise ValueError("Estimator names conflict with constructor arguments: {0!r}"
                             .format(sorted(clash)))
        bad = [n for n in names if "__" in n]
        if bad:
            raise ValueError("Estimator names must not contain __: got {0!r}".format(bad))


class _AvailableIf:
    def __init__(self, fn, check, name):
        self.fn, self.check, self.name = fn, check, name
        update_wrapper(self, fn)

    def __get__(self, obj, owner=None):
        if obj is None:
            return self.fn
        if not self.check(obj):
            raise AttributeError("This %r has no attribute %r" % (type(obj).__name__, self.name))
        fn = self.fn

        def bound(*args, **kwargs):
            return fn(obj, *args, **kwargs)
        update_wrapper(bound, fn)
        return bound


def available_if(check):
    return lambda fn: _AvailableIf(fn, check, fn.__name__)


def _delegate_has(attr, *names):
    """check: the delegate (``self.<attr>`` fitted or unfitted) has ``name``."""
    def check(self):
        for n in names:
            obj = getattr(self, n, None)
            if obj is not None:
                inner = obj[0] if isinstance(obj, list) and obj else obj
                return hasattr(inner, attr)
        return False
    return check


def if_delegate_has_method(delegate):
    """Method decorator of meta-estimators (reference
    ``utils/metaestimators.py:158``): the decorated method exists only when
    the sub-estimator stored under ``delegate`` (an attribute name, or a
    tuple of them tried in order - e.g. the fitted ``estimator_`` before the
    unfitted ``estimator``) has a method of the same name; otherwise
    accessing it raises AttributeError, so ``hasattr`` reflects the
    delegate's capabilities."""
    if isinstance(delegate, list):
        delegate = tuple(delegate)
    names = delegate if isinstance(delegate, tuple) else (delegate,)

    def wrap(fn):
        attr = fn.__name__

        def check(self):
            for n in names:
                obj = getattr(self, n, None)
                if obj is not None:
                    return hasattr(obj, attr)
            # none of the delegates is set: raise like the reference (the
            # last name's AttributeError)
            getattr(self, names[-1])
            return False
        return _AvailableIf(fn, check, attr)
    return wrap
