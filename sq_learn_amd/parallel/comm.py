"""Collectives for row-sharded data parallelism (SURVEY.md §2.5 P5/P7, §2.6
C1-C8).

One process per GPU, ``torch.distributed`` with the ``nccl`` backend (= RCCL
on ROCm, over xGMI inside an MI355X node) for device tensors and ``gloo`` for
CPU tensors (tests).  The framework's per-iteration traffic is tiny and
latency-bound (one packed k*d+k+1 fp64 bucket per Lloyd iteration, a d*d
Gram, d*l power-iteration products), so the design rule is *one collective
per logical reduction*: statistics are packed into a single contiguous
buffer before the call, never reduced field by field (the reference has no
collectives at all; this layer is new).
"""

import datetime
import os

import torch
import torch.distributed as dist

from ..exceptions import DistributedError

_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}


def env_world():
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_distributed(backend=None, timeout_s=600, device=None):
    """Initialise the default process group from env (idempotent).

    backend None -> 'nccl' (RCCL) when a GPU is visible, else 'gloo'.
    Returns a :class:`Comm` for the default group.
    """
    rank, world, local = env_world()
    if world <= 1:
        return Comm(None)
    if not dist.is_initialized():
        if backend is None:
            # SQ_DIST_BACKEND=gloo rehearses multi-rank GPU runs on one device
            backend = os.environ.get("SQ_DIST_BACKEND") or (
                "nccl" if torch.cuda.is_available() else "gloo")
        kw = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            torch.cuda.set_device(local % torch.cuda.device_count())
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group(**kw)
    return Comm(dist.group.WORLD)


class Comm:
    """Thin collective wrapper bound to one process group (``None`` = single
    process: every collective is the identity)."""

    def __init__(self, group=None):
        self.group = group
        if group is not None and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.world_size = dist.get_world_size(group)
            self.backend = dist.get_backend(group)
        else:
            self.group = None
            self.rank = 0
            self.world_size = 1
            self.backend = None
        self.bytes_reduced = 0
        self.calls = 0

    @classmethod
    def default(cls):
        if dist.is_available() and dist.is_initialized():
            return cls(dist.group.WORLD)
        return cls(None)

    @property
    def distributed(self):
        return self.world_size > 1

    def _staged(self, t):
        """Tensor on a device the backend can reduce (nccl: GPU, gloo: CPU)."""
        if self.backend == "nccl" and not t.is_cuda:
            return t.to(torch.device("cuda", torch.cuda.current_device())), True
        if self.backend == "gloo" and t.is_cuda:
            return t.cpu(), True
        return t, False

    def all_reduce_(self, t, op="sum"):
        if not self.distributed:
            return t
        s, moved = self._staged(t)
        try:
            dist.all_reduce(s, op=_OPS[op], group=self.group)
        except Exception as e:  # pragma: no cover - surfaced to the estimator
            raise DistributedError(f"all_reduce failed on rank {self.rank}: {e}") from e
        self.calls += 1
        self.bytes_reduced += s.numel() * s.element_size()
        if moved:
            t.copy_(s)
        return t

    def broadcast_(self, t, src=0):
        if not self.distributed:
            return t
        s, moved = self._staged(t)
        dist.broadcast(s, src=src, group=self.group)
        if moved:
            t.copy_(s)
        return t

    def all_gather(self, t):
        """List of every rank's tensor (same shape on all ranks)."""
        if not self.distributed:
            return [t]
        s, moved = self._staged(t.contiguous())
        out = [torch.empty_like(s) for _ in range(self.world_size)]
        dist.all_gather(out, s, group=self.group)
        if moved:
            out = [o.to(t.device) for o in out]
        return out

    def all_gather_varlen(self, t):
        """Gather tensors whose first dimension differs between ranks."""
        if not self.distributed:
            return [t]
        n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
        sizes = [int(x.item()) for x in self.all_gather(n)]
        mx = max(sizes)
        pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        got = self.all_gather(pad)
        return [g[:s] for g, s in zip(got, sizes)]

    def allreduce_scalars(self, values, op="sum", device=None, dtype=torch.float64):
        """Reduce a list of python scalars in ONE collective; returns a list."""
        t = torch.tensor(values, dtype=dtype, device=device or "cpu")
        self.all_reduce_(t, op=op)
        return t.tolist()

    def barrier(self):
        if self.distributed:
            if self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
            else:
                dist.barrier(group=self.group)


def shard_bounds(n, rank, world):
    """Contiguous row range [start, stop) of ``rank`` in an n-row dataset."""
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    stop = start + base + (1 if rank < rem else 0)
    return start, stop
