"""Device-resident Lloyd / q-means iteration engine.

One :class:`LloydEngine` owns every buffer of a fit on this rank's device
and runs iterations with at most one small device->host read each
(``[inertia, shift, overflow]`` for the convergence test).  It implements
the reference's quantum Lloyd loop (``_dmeans.py:534-671``):

    E-step   labels_estimation (``_dmeans.py:732-777``)
               delta == 0                 : exact argmin, random tie-break
               delta > 0, not true_dist   : uniform label in the delta-band
               delta > 0, true_dist (IPE) : argmin of IPE-noised distances
    M-step   _centers_update (``_dmeans.py:780-830``): cluster means, then
               (intermediate_error) tomography with error delta/2
    loop     best-inertia iterate, Frobenius shift <= tol, final E-step

GPU fast path (d_pad <= 1024, k_pad <= 16384, no IPE): per iteration
    E-step   gemm_precision 'fp32' (default): the certified filter
               (csrc/estep_f32.hip estep_x64: one fp16 MFMA pass with a
               rigorous error bound, Hamerly pruning, fp32 screen + fp64
               re-check of multi-candidate rows; dense rows through the
               fp32-faithful 3-pass kernel (d_pad <= 256) or the exact fp64
               rows kernel (csrc/rows_f64.hip), which also takes the 3-pass
               overflow rows) - the fp64 delta-band labels, device-driven;
             gemm_precision 'bf16' (d_pad <= 256): estep_bf16 (bf16
               operands, faster, the band edge is only bf16-accurate)
    -> centroid_accumulate (segmented reduce) -> pack_stats (one fp64 bucket)
    -> all_reduce over RCCL (C1: the only collective of the iteration)
    -> centroid_finalize (mean + fused truncated-normal tomography noise +
       shift + bf16 centroids and norms for the next E-step).
CPU tensors run the torch twins; GPU shapes outside the filter run the exact
fp64 rows kernel on every row (csrc/rows_f64.hip); IPE distances run the
fused IPE kernel (csrc/ipe.hip).
"""

import math
import os

import torch

from ...runtime.rng import RngKey
from ...ops import kmeans as K
from ...ops import linalg as L
from ...ops.random import trunc_normal_add_
from ...ops.failure import failure_inject_
from ...ops import _native as nat
from ...parallel.comm import Comm
from ...utils import tracing


class _HostScalars:
    """The iteration's scalars in pinned host memory, valid once ``event``
    has completed (pipelined steps: the read must not wait for the next
    iteration's E-step, already enqueued behind the copy)."""

    __slots__ = ("host", "event", "sink")

    def __init__(self, host, event, sink=None):
        self.host, self.event, self.sink = host, event, sink

    def tolist(self):
        self.event.synchronize()
        vals = self.host.tolist()
        if self.sink is not None:
            # one measurement per iteration, however often the caller reads
            sink, self.sink = self.sink, None
            sink(vals)
        return vals


class LloydEngine:
    def __init__(self, X, k, *, delta=0.0, true_distance_estimate=False, intermediate_error=False,
                 true_tomography=False, tomography_kw=None, sample_weight=None, seed=0,
                 comm=None, row_offset=0, gemm_precision="fp32", ipe_Q=13, empty_policy=0,
                 Xb=None, xn=None, failure_prob=0.0, failure_attempts=1, generic=False,
                 relocate_empty=False):
        self.X = X
        self.device = X.device
        self.n, self.d = X.shape
        self.k = int(k)
        self.delta = float(delta or 0.0)
        self.ipe = bool(true_distance_estimate) and self.delta > 0
        self.intermediate_error = bool(intermediate_error)
        self.true_tomography = bool(true_tomography)
        self.tomography_kw = dict(tomography_kw or {})
        self.sample_weight = sample_weight
        self.seed = seed
        self.comm = comm if comm is not None else Comm(None)
        self.row_offset = int(row_offset)
        self.ipe_Q = int(ipe_Q)
        self.empty_policy = int(empty_policy)
        self.k_pad = K.pad_clusters(self.k)
        self.d_pad = K.pad_features(self.d)
        self.restart = 0
        self.it = 0
        # pipeline: step() enqueues the NEXT iteration's E-step right after
        # its M-step (same key, same order of device work), so the GPU has
        # work while the host reads the iteration's scalars and re-enters the
        # loop (no per-iteration bubble); opt-in by the loop owner
        self.pipeline = False
        self._pending = None
        self._label_snap = None
        self._sc_ring = None
        self.relocate_empty = bool(relocate_empty)
        self.n_relocated = 0
        self.failure_prob = float(failure_prob or 0.0)
        self.failure_attempts = max(1, int(failure_attempts))
        # [estimations made, corrupted rows] over the engine's lifetime (device)
        self.failure_counters = torch.zeros(2, dtype=torch.int64, device=X.device)
        gpu = self.device.type == "cuda"
        if gemm_precision not in ("bf16", "fp32"):
            raise ValueError("gemm_precision must be 'bf16' or 'fp32', got %r" % (gemm_precision,))
        # the bf16 kernel is an option up to d_pad = 256; wider rows take the
        # certified path (a precision upgrade, never an uncertified fallback)
        if gemm_precision == "bf16" and self.d_pad > 256:
            gemm_precision = "fp32"
        self.precision = gemm_precision
        # generic=True: engines that replace the E-step (e.g. ElkanEngine);
        # GPU shapes outside the certified filter (d_pad > 1024, k_pad >
        # 16384) run the exact fp64 rows kernel on every row (_estep_generic)
        self.fast = (gpu and not generic and not self.ipe and self.d_pad in K.X64_D
                     and self.k_pad <= K.X64_MAX_K)
        self.alpha = 1.0
        self.acc_dtype = torch.float64 if not gpu else torch.float32
        if gpu:
            nat.native()  # fail loudly if the HIP layer is unavailable on a GPU box
        if self.fast:
            self._prepare_fast(Xb, xn)
        else:
            self._prepare_generic(xn)

    # ------------------------------------------------------------ prep
    def _prepare_fast(self, Xb, xn):
        dev = self.device
        if self.precision == "fp32":
            return self._prepare_fast_f32(xn)
        if Xb is None:
            if self.X.dtype == torch.bfloat16 and self.d == self.d_pad and self.X.is_contiguous():
                Xb = self.X
            else:
                Xb = torch.zeros((self.n, self.d_pad), dtype=torch.bfloat16, device=dev)
                Xb[:, :self.d] = self.X.to(torch.bfloat16)
        self.Xb = Xb
        self.xn = xn if xn is not None else L.row_norms_sq(Xb)
        # M-step source: the original data when it is fp32 (means keep fp32
        # precision), the padded bf16 copy otherwise
        if self.X.dtype == torch.float32 and self.d % 4 == 0:
            self.Xm = self.X.contiguous()
        else:
            self.Xm = Xb
        self.C_bf16 = torch.zeros(K.operand_shape(self.k_pad, self.d_pad), dtype=torch.bfloat16,
                                  device=dev)
        self.C_op = None
        self._prepare_reduce()

    def _prepare_fast_f32(self, xn):
        """fp32-faithful path: fp32 rows (zero-padded to d_pad only when
        needed) feed both the E-step (split to fp16 hi/lo in registers) and
        the M-step; alpha from the largest row norm over all ranks."""
        dev = self.device
        X = self.X
        if X.dtype == torch.float32 and self.d == self.d_pad and X.is_contiguous():
            Xf = X
        else:
            Xf = torch.zeros((self.n, self.d_pad), dtype=torch.float32, device=dev)
            Xf[:, :self.d] = X.to(torch.float32)
        self.Xf32 = Xf
        self.xn = (xn.float().contiguous() if xn is not None else L.row_norms_sq(Xf))
        mx = (self.xn.max() if self.n else torch.zeros((), device=dev)).double().reshape(1)
        self.comm.all_reduce_(mx, op="max")
        # a centroid is a mean of rows plus at most delta/2 of tomography error
        margin = self.delta + self._noise_bound() * math.sqrt(self.k * self.d)
        self.alpha = K.choose_alpha(float(mx.item()), margin)
        self.Xm = Xf
        self.C_bf16 = None
        self.C_op = torch.zeros(K.operand_f16_shape(self.k_pad, self.d_pad), dtype=torch.float16,
                                device=dev)
        # largest alpha^2 |c|^2 (the certified E-step's error bound; refreshed
        # by every centroid_finalize)
        self.cmax2 = torch.zeros(1, dtype=torch.float32, device=dev)
        # certified filter + fp64 re-check (default); SQ_ESTEP_FILTER=0 runs
        # the fp32-faithful 3-pass kernel on every row instead (A/B, tests)
        import os
        self.certified = os.environ.get("SQ_ESTEP_FILTER", "1") != "0"
        # the filter's A operand: fp16(alpha x), rounded once (2 B per value,
        # the bf16 kernel's HBM stream); exact fp32 rows stay for the re-check
        # and the M-step
        self.Xh16 = (Xf * self.alpha).to(torch.float16) if self.certified else None
        self._prepare_reduce()
        # 512 block partials of the min-distance sums + (incremental M-step)
        # the k per-cluster inertia parts, reduced together in one launch
        self.mind_part = torch.zeros(512 + self.k, dtype=torch.float64, device=dev)
        # incremental M-step (certified path, unweighted): only the rows
        # whose label moved are re-read; the inertia comes from the
        # per-cluster statistics + the E-step's min-vs-label corrections
        # (failure injection moves a corrupted row's correction with its
        # label).  SQ_MSTEP_INCREMENTAL=0 disables it.
        self.incremental = (self.certified and self.sample_weight is None
                            and os.environ.get("SQ_MSTEP_INCREMENTAL", "1") != "0")
        if self.incremental:
            self.prev_labels = torch.full((self.n,), -1, dtype=torch.int32, device=dev)
            self.qsum = torch.zeros(self.k, dtype=torch.float64, device=dev)
            self.perm2 = torch.empty(max(4 * self.n, 1), dtype=torch.int32, device=dev)
            self.buf.corr = torch.zeros(max(self.n, 1), dtype=torch.float32, device=dev)
            nr = int(self._nrows_global)
            self.qexp = K.fixed_point_exp(self._max_abs ** 2 * self.dm, nr)
        self.inc_valid = False
        # Hamerly pruning of the certified E-step (exact: pruned rows keep a
        # one-member band; a row corrupted by failure injection gets lb = 0,
        # so the next E-step re-evaluates it); SQ_ESTEP_BOUNDS=0 disables it
        self.bounds = (self.certified
                       and os.environ.get("SQ_ESTEP_BOUNDS", "1") != "0")
        # adaptive pruning: when the filter kept more than keep_max of the
        # rows in the last TWO measured E-steps (one high measurement is the
        # normal start of a fit: the centres still move a lot, and converge
        # within a step or two), the next E-steps sweep every row directly
        # (bounds still maintained) and the filter is re-probed every
        # probe_every steps.  keep_max = 0.8: the measured break-even of the
        # filter pass + list-mode sweep against the full sweep (list mode at
        # 100 % kept costs ~1.2x the full sweep at 10M x 256).
        self.keep_max = float(os.environ.get("SQ_ESTEP_KEEP_MAX", "0.8"))
        self.probe_every = 2
        self._kept_frac = None
        self._kept_prev = None
        self._skips = 0
        self._probing = False
        self._filter_ran = False
        self._minus1 = torch.full((1,), -1, dtype=torch.int32, device=dev)
        if self.bounds:
            self.ub = torch.zeros(max(self.n, 1), dtype=torch.float32, device=dev)
            self.lb = torch.zeros(max(self.n, 1), dtype=torch.float32, device=dev)
            self.rlist = torch.empty(max(self.n, 1), dtype=torch.int64, device=dev)
            self.rcount = torch.zeros(1, dtype=torch.int32, device=dev)
            self.shift_s = torch.zeros(self.k, dtype=torch.float64, device=dev)
            self.smax = torch.zeros(1, dtype=torch.float64, device=dev)
            # the fastest centroids are bounded through the label (Elkan)
            # instead of widening every row's lower bound by their shift
            self.n_fast = min(int(os.environ.get("SQ_ESTEP_FAST", "16")), self.k - 1)
            self.fast_idx = torch.zeros(max(self.n_fast, 1), dtype=torch.int32, device=dev)
            self.fast_cc = torch.zeros(max(self.k * (self.n_fast + 1), 1), dtype=torch.float32,
                                       device=dev)
        # gap records of the multi-candidate rows (csrc/estep_f32.hip): the
        # fp32 screen records a row's certain {argmin} band as distance gaps
        # with an error bound, based on that iteration's centres; while the
        # row's candidate set is unchanged, later iterations move the gaps by
        # the centroid shifts since the base (fp16 row x fp16 shift operand,
        # gap_screen_kernel: 512 B per row at d = 256 instead of the fp32 row
        # and two fp32 centroid rows; nothing stored while the label stands).
        # A ring of SQ_GAP_RING base iterations (snapshots + operands).
        # SQ_MULTI_RECORDS: 1 on, 0 off, default: on for shards of >= 4M rows
        # (measured: 10M rows 0.995-0.999 vs 0.981-1.017 ms per step; at
        # 1.25M rows - the 8-GPU share - the short list B leaves the gap
        # screen latency-bound, 0.32 vs 0.25 ms)
        self.mrec = None
        mr = os.environ.get("SQ_MULTI_RECORDS", "auto")
        if (self.bounds and self.incremental and self.d_pad % 128 == 0 and self.k <= 16384
                and (mr == "1" or (mr == "auto" and self.n >= 4_000_000))):
            R = min(max(int(os.environ.get("SQ_GAP_RING", "8")), 2), 16)
            self.mrec = torch.zeros((max(self.n, 1), 8), dtype=torch.float32, device=dev)
            self.rows_b = torch.empty(max(self.n, 1), dtype=torch.int64, device=dev)
            self.gsnap = torch.zeros((R, self.k, self.d_pad), dtype=torch.float32, device=dev)
            self.dsh = torch.zeros((R, self.k, self.d_pad), dtype=torch.float16, device=dev)
            self.dq = torch.zeros((R, self.k, 8), dtype=torch.float32, device=dev)
            # >= 2: the multi flag stores 2 + a record's base, 1 = no record
            self._rit = 2
            self._rlo = 2
        self.bounds_valid = False

    def _prepare_reduce(self):
        dev = self.device
        self.dm = self.Xm.shape[1]
        self.buf = K.EStepBuffers(self.n, dev)
        # deterministic fixed-point reduction: one global quantum for all ranks
        mx = torch.stack([self.Xm.abs().max().float() if self.n else torch.zeros((), device=dev),
                          (self.sample_weight.abs().max().float() if self.sample_weight is not None
                           and self.n else torch.zeros((), device=dev))]).double()
        nrows = torch.full((1,), float(self.n), dtype=torch.float64, device=dev)
        self.comm.all_reduce_(mx, op="max")
        self.comm.all_reduce_(nrows)
        mxl = mx.tolist()
        self._max_abs, self._nrows_global = mxl[0], nrows.item()
        self.rws = K.ReduceWorkspace(self.n, self.k, dev).set_scale(
            mxl[0], int(nrows.item()), mxl[1] if self.sample_weight is not None else None)
        self.sums = torch.zeros((self.k, self.dm), dtype=torch.float64, device=dev)
        self.counts = torch.zeros(self.k, dtype=torch.float64, device=dev)
        self.packed = torch.zeros(self.k * self.d + self.k + 1, dtype=torch.float64, device=dev)
        self.shift = torch.zeros(1, dtype=torch.float64, device=dev)
        self.shift_part = torch.zeros(self.k, dtype=torch.float64, device=dev)
        self.C = torch.zeros((self.k, self.d), dtype=torch.float32, device=dev)
        self.C_new = torch.zeros_like(self.C)
        self.cn = torch.full((self.k_pad,), K.BIG, dtype=torch.float32, device=dev)
        # [inertia, shift, overflow rows, rows kept by the Hamerly filter
        # (-1: no filter ran)] - one D2H read per iteration
        self.scalars = torch.zeros(4, dtype=torch.float64, device=dev)
        self.scalars[3] = -1.0
        self.weights = (self.sample_weight.to(torch.float32).contiguous()
                        if self.sample_weight is not None else None)

    def _prepare_generic(self, xn):
        self.Xf = self.X if self.X.dtype in (torch.float32, torch.float64) else self.X.float()
        self.xn = xn if xn is not None else (self.Xf * self.Xf).sum(1)
        wd = torch.float64 if self.device.type == "cpu" else torch.float32
        self.C = torch.zeros((self.k, self.d), dtype=wd, device=self.device)
        self.labels = torch.empty(self.n, dtype=torch.int64, device=self.device)
        self.mind = torch.empty(self.n, dtype=self.Xf.dtype, device=self.device)

    # ---------------------------------------------------------- keys
    def _key(self, purpose, it=None):
        it = self.it if it is None else it
        return RngKey(self.seed, purpose, (self.restart << 24) | (it & 0xFFFFFF))

    # ---------------------------------------------------------- state
    def drop_pending(self):
        """Forget a speculative next-iteration E-step (its device work has
        run; re-running that E-step is exact: bounds moved twice stay valid
        bounds, every processed row gets the same label)."""
        self._pending = None

    def set_centers(self, C, reset_hints=True):
        self._pending = None
        C = C.to(self.device)
        if reset_hints and getattr(self, "_ipe_lab", None) is not None:
            # new centres (a restart, the final E-step): the IPE label hints
            # of the previous trajectory must not seed this one, so every
            # restart and a resumed fit see the same (empty) hints
            for h in self._ipe_lab:
                h.fill_(-1)
            self._ipe_hint_valid = False
        self.inc_valid = False   # the incremental M-step restarts from scratch
        self.bounds_valid = False
        self._records_epoch()
        self._kept_frac = self._kept_prev = None   # new centres: re-measure the filter
        self._skips = 0
        self._probing = False
        self._probe_gap = getattr(self, "probe_every", 2)
        self._sc_dev = None
        if self.fast:
            self.C.copy_(C.to(torch.float32))
            if self.C_op is not None:
                K.centers_to_f16_native(self.C, self.C_op, self.k, self.d, self.d_pad, self.k_pad,
                                        self.alpha)
                self.cmax2.copy_(((self.C.double() * self.alpha) ** 2).sum(1).max().float()
                                 .reshape(1) if self.k else torch.zeros(1, device=self.device))
                return
            Cb, cn = K.centers_to_bf16(self.C, self.k_pad, self.d_pad)
            self.C_bf16.copy_(Cb)
            self.cn.copy_(cn)
        else:
            self.C = C.to(self.C.dtype).clone()

    def centers(self):
        return self.C

    def checkpoint_tensors(self):
        """Derived device state that must round-trip bit-exactly on resume
        (the E-step operand written by ``centroid_finalize``)."""
        if not self.fast:
            return {}
        if self.C_op is not None:
            return {"C_op": self.C_op}
        return {"C_bf16": self.C_bf16, "cn": self.cn}

    def checkpoint_local(self):
        """Per-rank state that must round-trip on resume: the IPE label
        hints (the previous E-step's labels seed the next one's thresholds,
        so they pick the realisation - ``ipe.hip`` hazard screen)."""
        if getattr(self, "_ipe_lab", None) is None:
            return {}
        return {"ipe_hint": self._ipe_lab[self._ipe_cur]}

    def restore_local(self, d):
        t = d.get("ipe_hint") if d else None
        if t is None or not self.ipe:
            return
        self._ipe_buffers()
        self._ipe_lab[self._ipe_cur].copy_(t.to(self.device).to(torch.int32))
        self._ipe_hint_valid = bool((t >= 0).all())
        if getattr(self, "_ipe16", None) is not None:
            self._ipe16.invalidate_bounds()   # restored hints: no skip until a full sweep

    def _ipe_buffers(self):
        if getattr(self, "_ipe_lab", None) is None:
            self._ipe_lab = [torch.full((self.n,), -1, dtype=torch.int32, device=self.device)
                             for _ in range(2)]
            self._ipe_cur = 0
            self._ipe_xn = self.xn.float().contiguous()

    def _list_rs(self):
        """Row sets per wave of the list-mode sweep: the full sweep's tiling
        (2) while the filter is expected to keep most rows (no measurement
        yet after new centres, or the last one above 30 %), one row set (the
        short-list default) once it prunes."""
        force = os.environ.get("SQ_LIST_RS")
        if force is not None:
            return int(force)
        kf = self._kept_frac
        return 2 if (kf is None or kf > 0.3) else 0

    def _records_epoch(self):
        """New centres not reached by the shift operands: every gap record
        written so far is void (current records have a base >= _rlo)."""
        if getattr(self, "mrec", None) is not None:
            self._rit += 2
            self._rlo = self._rit

    def restore_tensors(self, d):
        self._pending = None
        self.inc_valid = False
        self.bounds_valid = False
        self._records_epoch()
        if self.fast and self.C_op is not None and "C_op" in d:
            self.C_op.copy_(d["C_op"].to(self.device))
        elif self.fast and self.C_op is None and "C_bf16" in d:
            self.C_bf16.copy_(d["C_bf16"].to(self.device))
            self.cn.copy_(d["cn"].to(self.device))

    # ---------------------------------------------------------- E-step
    def estep(self, C=None):
        """Labels and min distances for the current (or given) centres;
        returns (labels, mind, local_inertia_tensor)."""
        self._pending = None
        if C is not None:
            self.set_centers(C)
        lab, mind, inertia = self._estep(self._key("band_select"), full=True)
        if self.fast and self.C_op is not None and self.certified:
            # single-candidate rows: their min distance is |x - c_label|^2
            K.fill_mind_native(self.Xf32, self.C, lab, mind)
            K.sum_f32_native(mind, self.n, self.mind_part, self.buf.inertia)
        return lab, mind, inertia

    def _estep(self, key, full=False):
        # the row lists of a filtered E-step (the only rows whose label can
        # change): the incremental M-step walks just those
        self._dlists = None
        if self.fast and self.C_op is not None and self.certified:
            with tracing.range("estep_x64"):
                Cp = self.C if self.d == self.d_pad else self._padded_centers()
                rows = None
                self._filter_ran = False
                if self.bounds and not full:
                    mode = self._filter_mode()
                    if mode == "filter" and not self.bounds_valid:
                        mode = "bounds"    # no valid bounds to filter with: maintain them now
                else:
                    mode = "bounds" if self.bounds else "none"
                # dormant bounds are not maintained by this sweep: invalid
                # until a bounds-maintaining sweep (the step before a probe)
                self._bounds_kept = mode != "none"
                screen = (self.incremental and not full
                          and os.environ.get("SQ_SCREEN", "1") != "0")
                if self.mrec is not None and screen:
                    # the record iteration lives in the multi flag (2 + it)
                    K.ensure_multi_buffers(self.buf, self.n, self.device, True)
                    R = self.dsh.shape[0]
                    K.multi_records(self.mrec, self.buf.mflag, self._rit,
                                    max(self._rlo, self._rit - R + 1), self.dsh, self.dq,
                                    self.rows_b, self.buf.counts[5:6], self.buf.counts[4:5])
                else:
                    # thread-local: a previous engine's records never leak in
                    K.multi_records(None)
                try:
                    # a probe (the filter kept > keep_max of the rows twice and was
                    # skipped since) only MEASURES: the filter pass counts the rows
                    # it would keep (the M-step records the fraction), the sweep
                    # stays full and maintains the bounds - a probe costs one
                    # filter pass, not a near-full list sweep
                    probe = mode == "filter" and self._probing
                    zero = True
                    if mode == "filter":
                        self._filter_ran = True
                        K.ensure_multi_buffers(self.buf, self.n, self.device, True)
                        # one fill clears the E-step counters and the kept count
                        self.rcount = self.buf.counts[3:4]
                        self.buf.counts.zero_()
                        K.bounds_filter_native(self.buf.labels[:self.n], self.ub, self.lb,
                                               self.shift_s, self.smax, self.delta, self.rlist,
                                               self.rcount, self.buf, cc=self.fast_cc,
                                               nf=self.n_fast, fidx=self.fast_idx)
                        if probe:
                            # the full sweep lists from scratch (list B too)
                            self.buf.counts[:3].zero_()
                            self.buf.counts[5:6].zero_()
                        else:
                            rows = (self.rlist, self.rcount)
                            # disjoint: unpruned rows, the filter's multi rows
                            # (the multi list's head), list B
                            self._dlists = ((self.rlist, self.rcount),
                                            (self.buf.multi_rows, self.buf.counts[7:8]),
                                            (self.rows_b, self.buf.counts[5:6])
                                            if self.mrec is not None and screen else None)
                        zero = False
                    lab, mind = K.estep_x64_native(self.Xh16, self.Xf32, self.C_op, Cp, self.xn,
                                                   self.cmax2, self.k, self.delta, self.alpha, key,
                                                   self.row_offset, self.buf,
                                                   bounds=(self.ub, self.lb)
                                                   if self.bounds and self._bounds_kept else None,
                                                   rows=rows, zero_counts=zero, screen=screen,
                                                   list_rs=self._list_rs())
                finally:
                    if self.mrec is not None:
                        # thread-local: never leak into another engine, even
                        # when the native E-step raised
                        K.multi_records(None)
                if self.mrec is not None and not screen:
                    # the sweep rewrote candidate lists the screen did not
                    # re-record: every record so far is void
                    self._records_epoch()
            return lab, mind, self.buf.inertia
        if self.fast and self.C_op is not None:
            with tracing.range("estep_f32"):
                lab, mind = K.estep_f32_native(self.Xf32, self.C_op, self.xn, self.C, self.k,
                                               self.delta, self.alpha, key, self.row_offset,
                                               self.buf)
            return lab, mind, self.buf.inertia
        if self.fast:
            with tracing.range("estep_bf16"):
                lab, mind = K.estep_native(self.Xb, self.C_bf16, self.cn, self.xn, self.k,
                                           self.delta, key, self.row_offset, self.buf)
            return lab, mind, self.buf.inertia
        if self.ipe:
            return self._estep_ipe(key)
        return self._estep_generic(key)

    def _filter_mode(self):
        """Adaptive Hamerly pruning: 'filter' (bounds filter + list-mode
        sweep), 'bounds' (full sweep that maintains the bounds, so the next
        E-step can filter) or 'none' (full sweep, bounds dormant).  The filter
        runs unless the last two measured iterations both kept more than
        ``keep_max`` of the rows (then its pass and the row-list indirection
        cost more than they save); it is re-probed after 2, 4, 8, 16 skipped
        steps while probes keep finding it useless, the step before a probe
        re-validating the bounds."""
        sd = getattr(self, "_sc_dev", None)
        if sd is not None:
            self._sc_dev = None
            self._on_scalars(sd.tolist())
        kf, kp = self._kept_frac, self._kept_prev
        was_probe = self._probing
        self._probing = False
        if kf is None or kp is None or kf <= self.keep_max or kp <= self.keep_max:
            self._skips = 0
            self._probe_gap = self.probe_every
            return "filter"
        if was_probe and kf >= 0.98 and kp >= 0.98:
            # the probe found (almost) nothing to prune: the rows are crowded
            # by the centres, not moving - probe rarely (a probe and the
            # bound-maintaining sweep before it cost more than the full sweep)
            self._probe_gap = 64
        self._skips += 1
        gap = getattr(self, "_probe_gap", self.probe_every)
        if self._skips >= gap:
            # a probe of a filter that kept > keep_max twice: back off (the
            # probe measures the kept fraction over a full sweep, see _estep)
            self._skips = 0
            self._probe_gap = min(2 * gap, 16) if gap < 16 else gap
            self._probing = True
            return "filter"
        return "bounds" if self._skips == gap - 1 else "none"

    def _on_scalars(self, vals):
        """Host values of an iteration's scalars (called by the pipelined
        read): records the filter's kept fraction."""
        if len(vals) > 3 and vals[3] >= 0 and self.n:
            self._kept_prev = self._kept_frac
            self._kept_frac = vals[3] / self.n

    def _chunk_rows(self):
        wm = 1 << 28  # 256 MiB of distances per chunk
        return max(1024, wm // (4 * max(self.k, 1)))

    def _estep_generic(self, key):
        n = self.n
        if self.device.type == "cuda":
            # exact fp64 E-step on every row (csrc/rows_f64.hip: fp64-MFMA
            # candidates + direct-form re-check): the reference's fp64 band
            # rule at any shape, no uncertified library-GEMM fallback
            labels32 = torch.empty(n, dtype=torch.int32, device=self.device)
            mind = torch.empty(n, dtype=torch.float32, device=self.device)
            Xg = self.Xf if (self.Xf.dtype == torch.float32 and self.Xf.stride(1) == 1) \
                else self.Xf.float().contiguous()
            K.rows_f64_native(Xg, self.C.float().contiguous(), labels32, mind, self.delta, key,
                              self.row_offset)
            return labels32, mind, mind.double().sum().reshape(1)
        Cw = self.C.to(self.Xf.dtype)
        lab, mind = K.estep_torch(self.Xf, Cw, self.delta, key, self.row_offset, self.k_pad,
                                  chunk_rows=self._chunk_rows(), xn=self.xn)
        return lab, mind, mind.double().sum().reshape(1)

    def _ipe16_ok(self):
        """The certified fp16 IPE screen (csrc/ipe16.hip) covers d <= 1024
        (above d_pad 256 through its values pass), k <= 16384, odd Q <= 31,
        fp32 rows; SQ_IPE16=0 disables it."""
        return (self.device.type == "cuda" and self.Xf.dtype == torch.float32
                and self.Xf.stride(1) == 1 and self.ipe_Q % 2 == 1 and self.ipe_Q <= 31
                and K.pad_features(self.d) in K.IPE16_D and self.k <= K.IPE16_MAX_K
                and os.environ.get("SQ_IPE16", "1") != "0")

    def _estep_ipe16(self, ipe_key):
        """IPE E-step by the certified fp16 screen: hint pair in full, fp16
        MFMA band classification of every other pair, canonical fp32 inner
        products and samplers only for the near / fired pairs (the law of
        ``_estep_ipe``'s fused kernel, see csrc/ipe16.hip)."""
        eps = self.delta / 2.0
        n = self.n
        self._ipe_buffers()
        d_pad = K.pad_features(self.d)
        k_pad = K.pad_clusters(self.k)
        if getattr(self, "_ipe16", None) is None:
            mx = (self._ipe_xn.max() if n else torch.zeros((), device=self.device)).double()
            mx = mx.reshape(1)
            self.comm.all_reduce_(mx, op="max")
            margin = self.delta + self._noise_bound() * math.sqrt(self.k * self.d)
            alpha = K.choose_alpha(float(mx.item()), margin)
            self._ipe16 = K.Ipe16(self.Xf, self.k, d_pad, k_pad, alpha, self.device)
        st = self._ipe16
        hint = self._ipe_lab[self._ipe_cur]
        self._ipe_cur ^= 1
        labels32 = self._ipe_lab[self._ipe_cur]
        first = not getattr(self, "_ipe_hint_valid", False)
        mind = torch.empty(n, dtype=torch.float32, device=self.device)
        C32 = self.C.float().contiguous()
        cn = (C32 * C32).sum(1).contiguous()
        st.set_centers(C32, cn)
        tie = self._key("band_select")
        xn = self._ipe_xn
        stats = getattr(self, "ipe16_stats", None)

        def fallback(rl, rc, ln, thr, hj, s, e):
            dp = 32
            while dp < self.d:
                dp *= 2
            kp = -(-self.k // 16) * 16
            K.ipe_fused_native(self.Xf[s:e], K.ipe_center_fragments(C32, kp, dp), xn[s:e], cn,
                               self.k, kp, dp, eps, self.ipe_Q, ipe_key, tie,
                               self.row_offset + s, labels32[s:e], mind[s:e], C=C32,
                               skip_key=self._key("ipe_skip"), rows=(rl, rc, ln), ext=(thr, hj),
                               stats=getattr(self, "ipe_stats", None))

        with tracing.range("ipe16"):
            st.estep(self.Xf, C32, hint, xn, cn, labels32, mind, eps, self.ipe_Q, ipe_key, tie,
                     self._key("ipe16_skip"), self._key("ipe16_row"), self.row_offset, first,
                     stats=stats, fallback=fallback)
        self._ipe_hint_valid = True
        return labels32, mind, mind.double().sum().reshape(1)

    def _estep_ipe(self, key):
        eps = self.delta / 2.0
        ipe_key = self._key("ipe")
        if self._ipe16_ok():
            return self._estep_ipe16(ipe_key)
        if self.device.type == "cuda" and self.d <= 2048 and self.Xf.dtype == torch.float32 \
                and self.Xf.stride(1) == 1 and self.ipe_Q <= 31:
            # fused kernel: fp32 MFMA inner products + per-pair median-of-Q AE.
            # The previous E-step's labels are the hint pairs (their estimates
            # seed the pruned screen; any hint gives the same law): two label
            # buffers alternate, so the labels returned by the last step stay
            # valid through the next one
            n = self.n
            self._ipe_buffers()
            hint = self._ipe_lab[self._ipe_cur]
            self._ipe_cur ^= 1
            labels32 = self._ipe_lab[self._ipe_cur]
            mind = torch.empty(n, dtype=torch.float32, device=self.device)
            dp = 32
            while dp < self.d:
                dp *= 2
            kp = -(-self.k // 16) * 16
            C32 = self.C.float().contiguous()
            cn = (C32 * C32).sum(1).contiguous()
            with tracing.range("ipe_fused"):
                K.ipe_fused_native(self.Xf, K.ipe_center_fragments(C32, kp, dp), self._ipe_xn, cn,
                                   self.k, kp, dp, eps, self.ipe_Q, ipe_key,
                                   self._key("band_select"), self.row_offset, labels32, mind,
                                   C=C32, hint_labels=hint, skip_key=self._key("ipe_skip"),
                                   stats=getattr(self, "ipe_stats", None))
            return labels32, mind, mind.double().sum().reshape(1)
        if self.device.type == "cuda":
            n = self.n
            labels32 = torch.empty(n, dtype=torch.int32, device=self.device)
            mind = torch.empty(n, dtype=torch.float32, device=self.device)
            C32 = self.C.float()
            cn = (C32 * C32).sum(1).contiguous()
            step = max(256, min(self._chunk_rows(), 1 << 16))
            for s in range(0, n, step):
                e = min(n, s + step)
                G = self.Xf[s:e].float() @ C32.T
                K.ipe_estep_native(G, self.xn[s:e].float().contiguous(), cn, eps, self.ipe_Q,
                                   ipe_key, self.row_offset + s, labels32[s:e], mind[s:e])
            return labels32, mind, mind.double().sum().reshape(1)
        lab, mind = K.ipe_estep_torch(self.Xf, self.C, eps, ipe_key, self.row_offset, self.k_pad,
                                      Q=self.ipe_Q)
        return lab, mind, mind.double().sum().reshape(1)

    # ---------------------------------------------------------- M-step
    def _noise_bound(self):
        if not self.intermediate_error or self.delta <= 0 or self.true_tomography:
            return 0.0
        # make_gaussian_est on the flattened k x d centre matrix (Utility.py:97)
        return (self.delta / 2.0) / math.sqrt(self.k * self.d)

    def mstep(self, labels, inertia, events=None):
        """Centroid update from labels; returns the device scalar tensor
        [inertia, shift, overflow_count] (one D2H read by the caller).
        ``events`` (two CUDA events, optional) are recorded after the
        segmented reduce and after the all-reduce (phase timing)."""
        noise_key = self._key("trunc_normal")
        if self.fast and getattr(self, "incremental", False) and self.buf.corr is not None:
            return self._mstep_incremental(labels, inertia, noise_key, events)
        if self.fast:
            with tracing.range("mstep"):
                exact = self.C_op is not None and self.certified
                Cold = None
                if exact:
                    Cold = self.C if self.dm == self.d else self._padded_centers()
                # the row pass fills the single-candidate rows' min distances
                # when a row is one column pass (d <= 256); wider rows: a
                # separate wave-per-row pass
                in_pass = exact and self.dm <= 256
                K.centroid_reduce_native(self.Xm, labels, self.weights, self.sums,
                                         self.counts, self.k, self.rws,
                                         mind=self.buf.mind if in_pass else None,
                                         C_old=Cold if in_pass else None)
                if exact and not in_pass:
                    K.fill_mind_native(self.Xf32, self.C, labels, self.buf.mind)
                if exact:
                    # inertia = sum of the (now complete) min distances, fixed order
                    K.sum_f32_native(self.buf.mind, self.n, self.mind_part, inertia)
                sums = self.sums if self.dm == self.d else self.sums[:, :self.d].contiguous()
                K.pack_stats_native(sums, self.counts, inertia, self.packed, self.k, self.d,
                                    self.rws, weighted=self.weights is not None)
            if events is not None:
                events[0].record()
            with tracing.range("allreduce"):
                self.comm.all_reduce_(self.packed)
            if events is not None:
                events[1].record()
            self._last_counts = self.packed[self.k * self.d:self.k * self.d + self.k]
            with tracing.range("finalize"):
                K.centroid_finalize_native(self.packed, self.C, self.C_new, self.C_bf16, self.cn,
                                           self.shift, self.k, self.d, self._noise_bound(),
                                           noise_key, self.empty_policy,
                                           shift_part=self.shift_part, scalars=self.scalars,
                                           buf=self.buf, C_f16=self.C_op, alpha=self.alpha,
                                           k_pad=self.k_pad,
                                           cmax2=self.cmax2 if self.C_op is not None else None,
                                           kept=(self.rcount if getattr(self, "_filter_ran", False)
                                                 else getattr(self, "_minus1", None)))
                self.C, self.C_new = self.C_new, self.C
                if self.intermediate_error and self.true_tomography and self.delta > 0:
                    self._true_tomography_centers()
                    self.scalars[1:2].copy_(((self.C.double() - self.C_new.double()) ** 2).sum())
            return self.scalars
        # generic / CPU
        w = self.sample_weight
        if self.device.type == "cuda" and self.Xf.dtype == torch.float32 and self.d % 4 == 0:
            # deterministic fixed-point segmented reduce (same kernel as the fast path)
            if not hasattr(self, "_g_rws"):
                mx = torch.stack([self.Xf.abs().max(), w.abs().max().float() if w is not None
                                  else torch.zeros((), device=self.device)]).double()
                nr = torch.full((1,), float(self.n), dtype=torch.float64, device=self.device)
                self.comm.all_reduce_(mx, op="max")
                self.comm.all_reduce_(nr)
                mxl = mx.tolist()
                self._g_rws = K.ReduceWorkspace(self.n, self.k, self.device).set_scale(
                    mxl[0], int(nr.item()), mxl[1] if w is not None else None)
                self._g_sums = torch.zeros((self.k, self.d), dtype=torch.float64,
                                           device=self.device)
                self._g_counts = torch.zeros(self.k, dtype=torch.float64, device=self.device)
                self._g_w = w.to(torch.float32).contiguous() if w is not None else None
                # incremental statistics (unweighted, contiguous rows of <= 1024
                # features - the IPE path): only the rows whose label moved are
                # re-read (csrc/kmeans.hip delta_segment_kernel; exact fixed
                # point, bit-identical to the full reduce below)
                self._g_inc = (w is None and self.Xf.is_contiguous() and self.d <= 1024
                               and os.environ.get("SQ_MSTEP_INCREMENTAL", "1") != "0")
                if self._g_inc:
                    self._g_prev = torch.full((max(self.n, 1),), -1, dtype=torch.int32,
                                              device=self.device)
                    self._g_qsum = torch.zeros(self.k, dtype=torch.float64, device=self.device)
                    self._g_perm2 = torch.empty(max(4 * self.n, 1), dtype=torch.int32,
                                                device=self.device)
                    self._g_qexp = K.fixed_point_exp(mxl[0] ** 2 * self.d, int(nr.item()))
            if self._g_inc:
                K.centroid_delta_native(self.Xf, labels.to(torch.int32).contiguous(),
                                        self._g_prev[:self.n], self._g_sums, self._g_counts,
                                        self._g_qsum, self.k, self._g_rws, self._g_perm2,
                                        self._g_qexp)
            else:
                K.centroid_reduce_native(self.Xf, labels.to(torch.int32), self._g_w, self._g_sums,
                                         self._g_counts, self.k, self._g_rws)
            packed = torch.empty(self.k * self.d + self.k + 1, dtype=torch.float64,
                                 device=self.device)
            K.pack_stats_native(self._g_sums, self._g_counts, inertia.double().reshape(1), packed,
                                self.k, self.d, self._g_rws, weighted=w is not None)
        else:
            sums, counts = K.centroid_sums_torch(self.Xf, labels, self.k, w,
                                                 acc_dtype=torch.float64)
            packed = torch.cat([sums.reshape(-1).double(), counts.double(),
                                inertia.double().reshape(1)])
        self.comm.all_reduce_(packed)
        kd = self.k * self.d
        sums = packed[:kd].reshape(self.k, self.d)
        counts = packed[kd:kd + self.k]
        self._last_counts = counts
        self._C_prev = self.C
        tot_inertia = packed[-1]
        old = self.C
        # (no clamp of the counts: where() discards the empty clusters' 0/0, and
        # every distinct torch kernel costs 30-130 ms of lazy loading at its
        # first use in a process - the first IPE step paid for clamp and pow)
        new = torch.where(counts[:, None] > 0, sums / counts[:, None],
                          old.double() if self.empty_policy == 0 else torch.zeros_like(sums))
        new = new.to(old.dtype).contiguous()
        b = self._noise_bound()
        if b > 0:
            flat = new.view(-1)
            trunc_normal_add_(flat, b, noise_key, offset=0)
        self.C = new
        if self.intermediate_error and self.true_tomography and self.delta > 0:
            self._true_tomography_centers()
        dd = self.C.double() - old.double()
        shift = (dd * dd).sum()
        return torch.stack([tot_inertia, shift, torch.zeros((), dtype=torch.float64,
                                                            device=self.device)])

    def _mstep_incremental(self, labels, inertia, noise_key, events):
        """Incremental fixed-point M-step (``centroid_delta_native``): the
        cluster sums / counts / squared-norm sums are updated by the rows
        whose label moved; the iteration's inertia is
        sum_c (Q_c - 2 c.S_c + n_c |c|^2) at the E-step's centroids plus the
        E-step's per-row (min - label distance) corrections - the reference's
        sum of minimum distances (``_dmeans.py:774-777``)."""
        with tracing.range("mstep_incremental"):
            if not self.inc_valid:
                self.sums.zero_()
                self.counts.zero_()
                self.qsum.zero_()
                self.prev_labels.fill_(-1)
            # (prev_labels <- labels inside the same pass); after a filtered
            # E-step only its row lists (labels changed nowhere else: no
            # failure injection, statistics valid)
            # (measured: the list walk gathers, the full walk streams - a win
            # on a 1.25M-row shard, 18.8 -> 11.5 us; even at 10M rows with
            # ~14 % of the rows listed: SQ_DELTA_LISTS=1 forces it, 0 never)
            dl = os.environ.get("SQ_DELTA_LISTS")
            use = (self.n <= 4_000_000) if dl is None else dl != "0"
            lists = getattr(self, "_dlists", None) if (use and self.inc_valid
                                                       and not self.failure_prob > 0) else None
            self._dlists = None
            if lists is not None:
                self.delta_list_steps = getattr(self, "delta_list_steps", 0) + 1
            K.centroid_delta_native(self.Xm, labels, self.prev_labels, self.sums, self.counts,
                                    self.qsum, self.k, self.rws, self.perm2, self.qexp,
                                    lists=lists)
            self.inc_valid = True
            Cold = self.C if self.dm == self.d else self._padded_centers()
            if self.dm == self.d:
                # cluster parts + correction sums, then pack + total: 2 launches
                K.mstep_stats_native(self.sums, self.counts, self.qsum, Cold, self.k, self.dm,
                                     self.rws, self.qexp, self.buf.corr, self.n, self.mind_part,
                                     inertia, self.packed)
            else:
                K.cluster_inertia_native(self.sums, self.counts, self.qsum, Cold, self.k, self.dm,
                                         self.rws, self.qexp, self.mind_part[512:512 + self.k])
                K.sum_f32_native(self.buf.corr, self.n, self.mind_part, inertia, extra=self.k)
                K.pack_stats_native(self.sums[:, :self.d].contiguous(), self.counts, inertia,
                                    self.packed, self.k, self.d, self.rws, weighted=False)
        if events is not None:
            events[0].record()
        with tracing.range("allreduce"):
            self.comm.all_reduce_(self.packed)
        if events is not None:
            events[1].record()
        self._last_counts = self.packed[self.k * self.d:self.k * self.d + self.k]
        with tracing.range("finalize"):
            K.centroid_finalize_native(self.packed, self.C, self.C_new, self.C_bf16, self.cn,
                                       self.shift, self.k, self.d, self._noise_bound(),
                                       noise_key, self.empty_policy,
                                       shift_part=self.shift_part, scalars=self.scalars,
                                       buf=self.buf, C_f16=self.C_op, alpha=self.alpha,
                                       k_pad=self.k_pad, cmax2=self.cmax2,
                                       kept=self.rcount if self._filter_ran else self._minus1)
            self.C, self.C_new = self.C_new, self.C
            if self.intermediate_error and self.true_tomography and self.delta > 0:
                self._true_tomography_centers()
                self.scalars[1:2].copy_(((self.C.double() - self.C_new.double()) ** 2).sum())
                if self.bounds:
                    self.shift_part[:self.k].copy_(
                        ((self.C.double() - self.C_new.double()) ** 2).sum(1))
            if self.bounds and getattr(self, "_bounds_kept", True):
                # per-centroid shifts of this update (fp64, rounded up) for the
                # next E-step's Hamerly bound update (after a sweep that left the
                # bounds dormant nothing reads them: the next E-step rebuilds)
                if self.n_fast > 0 and self.device.type == "cuda":
                    # sqrt + margin fused into the top-shift select
                    K.fast_centroids_native(self.shift_s, self.C, self.n_fast, self.fast_idx,
                                            self.smax, self.fast_cc,
                                            shift_sq=self.shift_part[:self.k])
                else:
                    torch.sqrt(self.shift_part[:self.k], out=self.shift_s)
                    self.shift_s.mul_(1.0 + 1e-12)
                    torch.amax(self.shift_s, dim=0, keepdim=True, out=self.smax)
            if self.mrec is not None:
                # the gap screen's operands of this update: the E-step centres
                # (base t, snapshotted) and every older base still current at
                # the next E-step -> the new centres (after a tomography reset
                # the records are void anyway)
                R = self.dsh.shape[0]
                t = self._rit
                valid = 0
                for b in range(max(self._rlo, t + 2 - R), t + 1):
                    valid |= 1 << (b % R)
                K.shift_operand_native(self.C_new, self.C, self.alpha, self.gsnap, self.dsh,
                                       self.dq, t % R, valid)
                self._rit += 1
            if self.bounds:
                self.bounds_valid = getattr(self, "_bounds_kept", True)
        return self.scalars

    def _padded_centers(self):
        if getattr(self, "_Cpad", None) is None:
            self._Cpad = torch.zeros((self.k, self.d_pad), dtype=torch.float32, device=self.device)
        self._Cpad[:, :self.d].copy_(self.C)
        return self._Cpad

    def _true_tomography_centers(self):
        """Real (shot-based) tomography of the k centre rows with error delta/2,
        replicated on every rank (Philox-keyed: identical everywhere); on the
        GPU one batched HIP launch pair (csrc/tomography.hip), no host trip."""
        from ...quantum.device import tomography_rows_torch
        key = self._key("tomography")
        C = self.C.double()
        est = tomography_rows_torch(C, self.delta / 2.0, key, **self.tomography_kw)
        # a centroid update, not a restart: the incremental statistics stay
        # valid (label based) and the bounds move by the recomputed shifts
        flags = (self.inc_valid, self.bounds_valid)
        self.set_centers(est.to(self.C.dtype), reset_hints=False)
        self.inc_valid, self.bounds_valid = flags

    # ---------------------------------------------------------- iteration
    def step_phases(self):
        """One Lloyd iteration (GPU fast path) timed per phase with CUDA
        events: E-step, segmented reduce (+ min distances, inertia, packing),
        all-reduce, finalize; plus the host wall of the whole step including
        the scalar read-back.  Returns {phase: ms}."""
        import time
        self._pending = None
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
        t0 = time.perf_counter()
        ev[0].record()
        labels, mind, inertia = self._estep(self._key("band_select"))
        ev[1].record()
        sc = self.mstep(labels, inertia, events=(ev[2], ev[3]))
        ev[4].record()
        sc.tolist()
        wall = (time.perf_counter() - t0) * 1e3
        self.it += 1
        return {"estep": ev[0].elapsed_time(ev[1]), "reduce": ev[1].elapsed_time(ev[2]),
                "allreduce": ev[2].elapsed_time(ev[3]), "finalize": ev[3].elapsed_time(ev[4]),
                "step_wall": wall}

    def _undo_update(self):
        """Back to the centres the last M-step started from (the relocation
        re-runs that M-step; the finalize recomputes every derived operand)."""
        if self.fast:
            self.C, self.C_new = self.C_new, self.C
        else:
            self.C = self._C_prev

    def _relocate(self, labels, counts):
        """Empty-cluster relocation of the classical Lloyd step (reference
        ``cluster/_k_means_fast.pyx:162-200``): each cluster the M-step left
        without weight takes one of the rows farthest from their own centre
        (the row moves: old cluster loses it, the empty one gets it - the
        reference's sums / weights update, expressed as a relabel before the
        M-step is re-run).  Row sharded: per-shard top-e distances, one
        all-gather, the same device-side global order on every
        rank (descending distance, ascending global row), the owner relabels
        its rows.  Only runs when the M-step's global counts (already
        all-reduced) show an empty cluster."""
        dev = self.device
        empty = torch.nonzero(counts == 0)[:, 0]
        e = int(empty.numel())
        if e == 0:
            return labels
        lab = labels[:self.n].long()
        valid = lab >= 0
        C = self.C.double()
        d = torch.empty(self.n, dtype=torch.float64, device=dev)
        X = self.X
        step = 1 << 19
        for s0 in range(0, self.n, step):
            xs = X[s0:s0 + step].double()
            d[s0:s0 + step] = ((xs - C[lab[s0:s0 + step].clamp(min=0)]) ** 2).sum(1)
        d = torch.where(valid, d, torch.full_like(d, -1.0))
        m = min(e, self.n)
        vals, idx = torch.topk(d, m) if m > 0 else (d[:0], lab[:0])
        rows = idx + self.row_offset
        if m < e:   # pad so every rank sends e entries
            vals = torch.cat([vals, torch.full((e - m,), -2.0, dtype=vals.dtype, device=dev)])
            rows = torch.cat([rows, torch.full((e - m,), -1, dtype=rows.dtype, device=dev)])
        allv = torch.cat(self.comm.all_gather(vals))
        allr = torch.cat(self.comm.all_gather(rows))
        # global order on the device: ascending row, then (stable) descending
        # distance - identical on every rank
        o1 = torch.argsort(allr, stable=True)
        o2 = torch.argsort(-allv[o1], stable=True)
        order = o1[o2][:e]
        g = allr[order]
        loc = g - self.row_offset
        mine = (g >= 0) & (loc >= 0) & (loc < self.n)
        li = loc[mine]
        newlab = empty[mine]
        if li.numel():
            if getattr(self, "incremental", False) and self.buf.corr is not None:
                # the per-cluster inertia counts a row at its label's centre
                # plus its correction (min - label distance, non-zero when
                # delta > 0 picked a band member other than the argmin): the
                # row moves to the empty cluster's centre, so its correction
                # grows by d(old label) - d(new label) and it still adds its
                # minimum distance
                xr = X[li].double()
                dnew = ((xr - C[newlab]) ** 2).sum(1)
                self.buf.corr[li] += (d[li] - dnew).to(self.buf.corr.dtype)
            labels[li] = newlab.to(labels.dtype)
            if getattr(self, "bounds", False):
                self.lb[li] = 0.0   # label moved: re-evaluate next E-step
            if getattr(self, "_ipe16", None) is not None:
                self._ipe16.lb[li] = 0.0   # the IPE row skip's bound too
        self.n_relocated += e
        return labels

    def step(self):
        """One Lloyd iteration; returns (labels, scalars_tensor).

        With empty-cluster relocation the scalars come back as a host tensor:
        the iteration's single device->host read carries the number of
        empty clusters of the M-step's (global) counts as well, and only when
        it is non-zero is the M-step re-run after the relocation."""
        if self._pending is not None:
            labels, mind, inertia = self._pending
            self._pending = None
        else:
            labels, mind, inertia = self._estep(self._key("band_select"))
        if self.failure_prob > 0:
            # Bernoulli estimation failures (+ resampling);
            # the pruned / incremental step's per-row state follows the label
            extra = {}
            if self.fast and getattr(self, "bounds", False):
                extra["lb"] = self.lb
            if self.fast and self.C_op is not None and self.certified:
                Cm = self.C if self.dm == self.d else self._padded_centers()
                extra.update(X=self.Xm, C=Cm, mind=self.buf.mind)
                if getattr(self, "incremental", False) and self.buf.corr is not None:
                    extra["corr"] = self.buf.corr
            failure_inject_(labels, self.k, self.failure_prob, self.failure_attempts,
                            self._key("failure"), self.row_offset, self.failure_counters, **extra)
        sc = self.mstep(labels, inertia)
        if self.relocate_empty:
            counts = self._last_counts
            ne = (counts == 0).sum().to(torch.float64).reshape(1)
            vals = torch.cat([sc.reshape(-1)[:3].to(torch.float64), ne]).cpu()
            if vals[3] > 0:
                self._undo_update()
                labels = self._relocate(labels, counts.clone())
                sc = self.mstep(labels, inertia)
                vals = torch.cat([sc.reshape(-1)[:3].to(torch.float64),
                                  torch.zeros(1, dtype=torch.float64, device=sc.device)]).cpu()
            sc = vals
        self.it += 1
        if self.pipeline and self.fast and not self.relocate_empty:
            # the iteration's scalars go to pinned host memory BEFORE the next
            # E-step is enqueued (a plain .tolist() would wait for that E-step
            # too); the caller's .tolist() waits on this event only
            if self._sc_ring is None:
                self._sc_ring = [(torch.empty(sc.numel(), dtype=sc.dtype, pin_memory=True),
                                  torch.cuda.Event()) for _ in range(2)]
            host, ev = self._sc_ring[self.it & 1]
            host.copy_(sc.reshape(-1), non_blocking=True)
            ev.record()
            # the caller keeps this iteration's labels: a device snapshot
            # before the next E-step rewrites the buffer
            if self._label_snap is None or self._label_snap.shape != labels.shape:
                self._label_snap = torch.empty_like(labels)
            self._label_snap.copy_(labels)
            labels = self._label_snap
            self._pending = self._estep(self._key("band_select"))
            sc = _HostScalars(host, ev, self._on_scalars)
        elif getattr(self, "bounds", False) and torch.is_tensor(sc) and sc.numel() > 3:
            # unpipelined: the next E-step reads this iteration's kept count
            # (the caller has usually synchronised on it already)
            self._sc_dev = sc
        return labels, sc
