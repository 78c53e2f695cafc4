"""Partial dependence plots (reference ``inspection/_plot/partial_dependence.py``:
``plot_partial_dependence`` ``:21`` and ``PartialDependenceDisplay`` ``:409``).

The display keeps the computed results (one Bunch per requested feature or
feature pair, as returned by ``partial_dependence(kind=...)``) and the
deciles of the plotted features; ``plot`` lays them out on an
``n_cols``-wide grid of axes: one-way results as lines (the average and/or up
to ``subsample`` ICE curves), two-way results as filled contours, decile
ticks along the feature axes.  matplotlib is imported only when drawing."""

import numbers
from math import ceil

import numpy as np
from scipy.stats.mstats import mquantiles

from .base import is_classifier, is_regressor
from .utils.validation import check_random_state


def _to_np(a):
    return a.detach().cpu().numpy() if hasattr(a, "detach") else np.asarray(a)


def _normalise_features(features, feature_names, n_features):
    """Feature specs (int index, name, or pairs of them) -> tuples of
    column indices; every index checked against the data width."""
    def one(fx):
        if isinstance(fx, str):
            if feature_names is None:
                raise ValueError("When the features are given by name, feature_names must be "
                                 "provided (or X must be a DataFrame).")
            try:
                return feature_names.index(fx)
            except ValueError:
                raise ValueError(f"Feature {fx} not in feature_names")
        fx = int(fx)
        if not 0 <= fx < n_features:
            raise ValueError(f"All entries of features must be in [0, {n_features - 1}].")
        return fx

    out = []
    for f in features:
        if isinstance(f, (numbers.Integral, str)):
            f = (f,)
        f = tuple(f)
        if not 1 <= len(f) <= 2:
            raise ValueError("Each entry in features must be either an int, a string, or an "
                             "iterable of size at most 2.")
        out.append(tuple(one(x) for x in f))
    return out


class PartialDependenceDisplay:
    """Partial dependence (PD) and individual conditional expectation (ICE)
    plots.

    Parameters mirror the reference: ``pd_results`` (list of Bunch with
    ``average`` / ``individual`` and ``values``), ``features`` (tuples of
    column indices), ``feature_names``, ``target_idx`` (output / class
    plotted), ``pdp_lim`` ({1 or 2: (min, max)} shared y / colour range),
    ``deciles`` ({column: deciles}), ``kind`` ('average', 'individual' or
    'both'), ``subsample`` (ICE curves drawn: int count or float fraction)
    and ``random_state`` (which ICE curves)."""

    def __init__(self, pd_results, *, features, feature_names, target_idx, pdp_lim, deciles,
                 kind="average", subsample=1000, random_state=None):
        self.pd_results = pd_results
        self.features = features
        self.feature_names = feature_names
        self.target_idx = target_idx
        self.pdp_lim = pdp_lim
        self.deciles = deciles
        self.kind = kind
        self.subsample = subsample
        self.random_state = random_state

    # ------------------------------------------------------------ helpers
    def _n_ice(self, n_samples):
        s = self.subsample
        if s is None:
            return n_samples
        if isinstance(s, numbers.Integral):
            return min(int(s), n_samples)
        return ceil(float(s) * n_samples)

    def _ice_rows(self, n_samples):
        m = self._n_ice(n_samples)
        if m >= n_samples:
            return np.arange(n_samples)
        rs = check_random_state(self.random_state)
        return np.sort(rs.choice(n_samples, m, replace=False))

    def _one_way(self, ax, res, fx, line_kw, lines_row):
        values = res["values"][0]
        lines = []
        if self.kind in ("individual", "both"):
            ind = res["individual"][self.target_idx]
            rows = self._ice_rows(ind.shape[0])
            kw = {"color": "tab:blue", "alpha": 0.3 if self.kind == "individual" else 0.15,
                  "linewidth": 0.5}
            kw.update(line_kw)
            kw.pop("label", None)
            for r in rows:
                lines.append(ax.plot(values, ind[r], **kw)[0])
        if self.kind in ("average", "both"):
            kw = dict(line_kw)
            if self.kind == "both":
                kw.setdefault("color", "tab:orange")
                kw.setdefault("linestyle", "--")
                kw.setdefault("label", "average")
            lines.append(ax.plot(values, res["average"][self.target_idx], **kw)[0])
        lines_row.append(lines)
        ymin, ymax = self.pdp_lim[1]
        pad = 0.05 * (ymax - ymin)
        ax.set_ylim(ymin - pad, ymax + pad)
        ax.set_xlabel(self.feature_names[fx[0]])
        if self.kind == "both":
            ax.legend()
        return ax

    def _two_way(self, ax, res, fx, contour_kw):
        import matplotlib.pyplot as plt
        v0, v1 = res["values"][0], res["values"][1]
        Z = res["average"][self.target_idx].T
        XX, YY = np.meshgrid(v0, v1)
        zmin, zmax = self.pdp_lim[2]
        kw = {"alpha": 0.75}
        kw.update(contour_kw)
        levels = np.linspace(zmin, zmax, num=8)
        cs = ax.contour(XX, YY, Z, levels=levels, linewidths=0.5, colors="k")
        cf = ax.contourf(XX, YY, Z, levels=levels, vmax=zmax, vmin=zmin, **kw)
        ax.clabel(cs, fmt="%2.2f", colors="k", fontsize=10, inline=True)
        ax.set_xlabel(self.feature_names[fx[0]])
        ax.set_ylabel(self.feature_names[fx[1]])
        plt.colorbar(cf, ax=ax)
        return cf

    def _decile_ticks(self, ax, fx, i):
        import matplotlib.transforms as mtransforms
        trans = mtransforms.blended_transform_factory(ax.transData, ax.transAxes)
        self.deciles_vlines_.flat[i] = ax.vlines(self.deciles[fx[0]], 0, 0.05, transform=trans,
                                                 color="k")
        if len(fx) == 2:
            trans2 = mtransforms.blended_transform_factory(ax.transAxes, ax.transData)
            self.deciles_hlines_.flat[i] = ax.hlines(self.deciles[fx[1]], 0, 0.05,
                                                     transform=trans2, color="k")

    # --------------------------------------------------------------- plot
    def plot(self, *, ax=None, n_cols=3, line_kw=None, contour_kw=None):
        """Draw on ``ax`` (None: a new figure; one Axes: split into an
        ``n_cols`` grid; an array of Axes: one per feature, same shape)."""
        import matplotlib.pyplot as plt
        from matplotlib.gridspec import GridSpecFromSubplotSpec
        line_kw = {} if line_kw is None else dict(line_kw)
        contour_kw = {} if contour_kw is None else dict(contour_kw)
        nf = len(self.features)
        if ax is None:
            _, ax = plt.subplots()
        if isinstance(ax, plt.Axes):
            if not ax.axison:
                raise ValueError("The ax was already used in another plot function, please set "
                                 "ax=display.axes_ instead")
            ax.set_axis_off()
            self.bounding_ax_ = ax
            self.figure_ = ax.figure
            n_cols = min(n_cols, nf)
            n_rows = int(ceil(nf / float(n_cols)))
            self.axes_ = np.empty((n_rows, n_cols), dtype=object)
            self.lines_ = np.empty((n_rows, n_cols), dtype=object)
            self.contours_ = np.empty((n_rows, n_cols), dtype=object)
            gs = GridSpecFromSubplotSpec(n_rows, n_cols, subplot_spec=ax.get_subplotspec())
            for i in range(nf):
                self.axes_.flat[i] = self.figure_.add_subplot(gs[i // n_cols, i % n_cols])
        else:
            ax = np.asarray(ax, dtype=object)
            if ax.size != nf:
                raise ValueError(f"Expected ax to have {nf} axes, got {ax.size}")
            self.bounding_ax_ = None
            self.figure_ = ax.ravel()[0].figure
            self.axes_ = ax
            self.lines_ = np.empty(ax.shape, dtype=object)
            self.contours_ = np.empty(ax.shape, dtype=object)
        self.deciles_vlines_ = np.empty(self.axes_.shape, dtype=object)
        self.deciles_hlines_ = np.empty(self.axes_.shape, dtype=object)
        first_one_way = True
        for i, (a, fx, res) in enumerate(zip(self.axes_.flat, self.features, self.pd_results)):
            if len(fx) == 1:
                row = []
                self._one_way(a, res, fx, line_kw, row)
                lines = row[0]
                self.lines_.flat[i] = lines[0] if len(lines) == 1 else np.asarray(lines,
                                                                                  dtype=object)
                if first_one_way:
                    a.set_ylabel("Partial dependence")
                    first_one_way = False
                else:
                    a.set_yticklabels([])
            else:
                self.contours_.flat[i] = self._two_way(a, res, fx, contour_kw)
            self._decile_ticks(a, fx, i)
        return self

    # -------------------------------------------------------- constructor
    @classmethod
    def from_estimator(cls, estimator, X, features, *, feature_names=None, target=None,
                       response_method="auto", n_cols=3, grid_resolution=100,
                       percentiles=(0.05, 0.95), method="auto", n_jobs=None, verbose=0,
                       line_kw=None, contour_kw=None, ax=None, kind="average",
                       subsample=1000, random_state=None):
        """Compute the partial dependences of ``features`` and plot them
        (the reference's ``plot_partial_dependence``)."""
        from .inspection import partial_dependence
        if not (is_classifier(estimator) or is_regressor(estimator)):
            raise ValueError("'estimator' must be a fitted regressor or classifier.")
        if kind not in ("average", "individual", "both"):
            raise ValueError("kind must be one of 'average', 'individual', 'both'")
        if hasattr(X, "columns") and feature_names is None:
            feature_names = [str(c) for c in X.columns]
        Xn = np.asarray(X.values if hasattr(X, "values") else X)
        n_features = Xn.shape[1]
        if feature_names is None:
            feature_names = [str(i) for i in range(n_features)]
        feature_names = list(feature_names)
        if len(set(feature_names)) != len(feature_names):
            raise ValueError("feature_names should not contain duplicates.")
        if isinstance(features, (numbers.Integral, str)):
            features = [features]
        feats = _normalise_features(features, feature_names, n_features)
        if kind != "average" and any(len(f) > 1 for f in feats):
            raise ValueError("It is not possible to display individual effects for more than "
                             "one feature at a time.")
        # output plotted: the class for a multiclass classifier, the target
        # column for a multi-output regressor, else the only output
        target_idx = 0
        classes = getattr(estimator, "classes_", None)
        if is_classifier(estimator) and classes is not None and len(_to_np(classes)) > 2:
            if target is None:
                raise ValueError("target must be specified for multi-class")
            cl = _to_np(classes).tolist()
            if target not in cl:
                raise ValueError(f"target not in est.classes_, got {target}")
            target_idx = cl.index(target)
        elif target is not None:
            target_idx = int(target)
        pkind = "both" if kind in ("individual", "both") else "average"
        results = [partial_dependence(estimator, Xn, list(f), response_method=response_method,
                                      percentiles=percentiles, grid_resolution=grid_resolution,
                                      method=method, kind=pkind) for f in feats]
        n_out = results[0]["average"].shape[0]
        if not 0 <= target_idx < n_out:
            raise ValueError(f"target must be in [0, {n_out - 1}]")
        # shared y range for one-way plots, colour range for two-way plots
        lim = {}
        for f, r in zip(feats, results):
            src = r["average"][target_idx] if kind == "average" or len(f) == 2 else \
                np.concatenate([r["average"][target_idx].ravel(),
                                r["individual"][target_idx].ravel()])
            lo, hi = float(np.min(src)), float(np.max(src))
            old = lim.get(len(f), (lo, hi))
            lim[len(f)] = (min(lo, old[0]), max(hi, old[1]))
        deciles = {}
        for f in feats:
            for c in f:
                if c not in deciles:
                    deciles[c] = mquantiles(Xn[:, c], prob=np.arange(0.1, 1.0, 0.1))
        disp = cls(results, features=feats, feature_names=feature_names, target_idx=target_idx,
                   pdp_lim=lim, deciles=deciles, kind=kind, subsample=subsample,
                   random_state=random_state)
        return disp.plot(ax=ax, n_cols=n_cols, line_kw=line_kw, contour_kw=contour_kw)


def plot_partial_dependence(estimator, X, features, *, feature_names=None, target=None,
                            response_method="auto", n_cols=3, grid_resolution=100,
                            percentiles=(0.05, 0.95), method="auto", n_jobs=None, verbose=0,
                            line_kw=None, contour_kw=None, ax=None, kind="average",
                            subsample=1000, random_state=None):
    """Partial dependence plots of ``features`` (see
    :meth:`PartialDependenceDisplay.from_estimator`)."""
    return PartialDependenceDisplay.from_estimator(
        estimator, X, features, feature_names=feature_names, target=target,
        response_method=response_method, n_cols=n_cols, grid_resolution=grid_resolution,
        percentiles=percentiles, method=method, n_jobs=n_jobs, verbose=verbose, line_kw=line_kw,
        contour_kw=contour_kw, ax=ax, kind=kind, subsample=subsample, random_state=random_state)
