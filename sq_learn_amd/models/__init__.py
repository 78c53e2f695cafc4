"""Estimators (sklearn API): cluster, decomposition, svm, neighbors."""
