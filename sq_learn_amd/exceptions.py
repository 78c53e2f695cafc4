"""Exceptions and warnings (reference: ``sklearn/exceptions.py:21-146``)."""


class NotFittedError(ValueError, AttributeError):
    """Raised when an estimator is used before ``fit``."""


class ConvergenceWarning(UserWarning):
    """Raised by iterative estimators that did not converge."""


class DataConversionWarning(UserWarning):
    """Raised on implicit data conversion."""


class DataDimensionalityWarning(UserWarning):
    """Raised on dimensionality problems of the input."""


class EfficiencyWarning(UserWarning):
    """Raised when a computational path is known to be slow."""


class FitFailedWarning(RuntimeWarning):
    """Raised when fitting failed inside a meta-estimator."""


class ClassicalPathWarning(UserWarning):
    """Emitted where the reference warns that a path is 'purely classic'
    (e.g. ``_qPCA.py:551``, ``_dmeans.py:1329``)."""


class InconsistentVersionWarning(UserWarning):
    """Unpickling an estimator saved by another framework version
    (reference ``base.py:296-320``)."""

    def __init__(self, *, estimator_name, current_version, original_version):
        self.estimator_name = estimator_name
        self.current_version = current_version
        self.original_version = original_version

    def __str__(self):
        return (f"Trying to unpickle estimator {self.estimator_name} from version "
                f"{self.original_version} when using version {self.current_version}.")


class DistributedError(RuntimeError):
    """A collective failed, timed out or saw inconsistent state across ranks."""


class NumericalGuardError(FloatingPointError):
    """The per-iteration NaN/inf guard tripped."""


class UndefinedMetricWarning(UserWarning):
    """A metric is ill-defined (e.g. no positive predictions for precision)."""


class ChangedBehaviorWarning(UserWarning):
    """A class or function changed behaviour since an earlier release."""


class NonBLASDotWarning(EfficiencyWarning):
    """A dot product could not use BLAS (kept for API parity: every product
    here goes to a library GEMM or a hand-written MFMA kernel)."""


class SkipTestWarning(UserWarning):
    """A test was skipped (estimator_checks)."""


class PositiveSpectrumWarning(UserWarning):
    """Tiny negative eigenvalues of a PSD matrix were set to zero."""
