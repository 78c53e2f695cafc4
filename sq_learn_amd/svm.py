"""Reference-layout import path (``sklearn.svm``): libsvm / liblinear SVMs, LS-SVM and
quantum LS-SVM."""
from .models.svm import *  # noqa: F401,F403
from .models.svm import __all__  # noqa: F401
