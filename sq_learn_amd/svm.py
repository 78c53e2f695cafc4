"""Reference-layout import path (``sklearn.svm``): LS-SVM and quantum LS-SVM."""
from .models.svm import LSSVC, QLSSVC  # noqa: F401
