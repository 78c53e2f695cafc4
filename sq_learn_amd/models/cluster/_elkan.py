"""Elkan iteration engine for the classical ``KMeans(algorithm='elkan')``.

Reference: ``cluster/_kmeans.py:_kmeans_single_elkan`` (:404-530 of the
fork's sklearn base) driving ``_k_means_elkan.pyx``.  Same step contract
as :class:`LloydEngine` (``step() -> (labels, [inertia, shift, 0])``,
``estep()``, ``centers()``), so ``KMeans._single`` runs either engine.

The E-step is the bounded assignment of ``ops/elkan.py``; the M-step is
the engine's generic path (deterministic fixed-point segmented reduce on
the GPU, one packed all-reduce across ranks).  Distances are exact
Euclidean distances in the data dtype (fp32 on the GPU, fp64 on the CPU),
not the bf16 MFMA distances of the Lloyd fast path.  Bounds are per-rank
state (rows are sharded); the centre geometry is computed redundantly on
every rank from the replicated centres.
"""

import torch

from ...ops import elkan as E
from ._lloyd import LloydEngine


class ElkanEngine(LloydEngine):
    def __init__(self, X, k, **kw):
        kw = dict(kw)
        kw["delta"] = 0.0
        kw["gemm_precision"] = "fp32"
        kw["generic"] = True     # the bounded Elkan E-step replaces the fused one
        super().__init__(X, k, **kw)
        dt = self.Xf.dtype
        self.Xe = self.Xf.contiguous()
        self.upper = torch.zeros(self.n, dtype=dt, device=self.device)
        self.lower = torch.zeros((self.n, self.k), dtype=dt, device=self.device)
        self.elabels = torch.zeros(self.n, dtype=torch.int32, device=self.device)
        self.cshift = torch.zeros(self.k, dtype=dt, device=self.device)
        self._fresh = True

    def set_centers(self, C, reset_hints=True):
        super().set_centers(C, reset_hints=reset_hints)
        self._fresh = True

    def estep(self, C=None):
        if C is not None:
            self.set_centers(C)
        Cw = self.C.to(self.Xe.dtype).contiguous()
        hcc, snext = E.centre_geometry(Cw)
        E.elkan_step(self.Xe, Cw, hcc, snext, self.cshift, self.elabels, self.upper, self.lower,
                     init=self._fresh)
        self._fresh = False
        self.cshift.zero_()
        inertia = (self.upper.double() ** 2).sum().reshape(1)
        return self.elabels, self.upper, inertia

    def step(self):
        labels, _, inertia = self.estep()
        old = self.C.clone()
        sc = self.mstep(labels, inertia)
        self.cshift.copy_(E.centre_shift(old, self.C).to(self.cshift.dtype))
        self.it += 1
        return labels, sc
