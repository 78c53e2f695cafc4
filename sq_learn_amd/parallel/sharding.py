"""Row-sharded datasets.

A :class:`ShardedArray` is the local slice ``X[start:stop]`` of a global
``n x d`` matrix that lives on this rank's device, plus the global geometry.
Estimators accept it anywhere they accept an array; statistics that span the
full dataset (means, Gram matrices, centroid sums, mu(A) power sums) are then
reduced across ranks by :class:`~sq_learn_amd.parallel.comm.Comm`.

Because the stochastic layer is keyed by *global* row index, a sharded fit
draws the same random numbers as a single-GPU fit of the same data
(SURVEY.md §7.4 shard invariance).
"""

import torch

from .comm import Comm, shard_bounds


class ShardedArray:
    def __init__(self, local, n_global, row_offset, comm=None):
        if not isinstance(local, torch.Tensor):
            local = torch.as_tensor(local)
        self.local = local
        self.n_global = int(n_global)
        self.row_offset = int(row_offset)
        self.comm = comm if comm is not None else Comm.default()

    @property
    def shape(self):
        return (self.n_global,) + tuple(self.local.shape[1:])

    @property
    def ndim(self):
        return self.local.ndim

    @property
    def dtype(self):
        return self.local.dtype

    @property
    def device(self):
        return self.local.device

    def __len__(self):
        return self.n_global

    def __repr__(self):
        return (f"ShardedArray(global_shape={self.shape}, local_rows={self.local.shape[0]}, "
                f"row_offset={self.row_offset}, rank={self.comm.rank}/{self.comm.world_size})")

    def gather(self):
        """Full matrix on every rank (small data / tests only)."""
        parts = self.comm.all_gather_varlen(self.local)
        return torch.cat(parts, 0)


def shard_rows(X, comm=None, device=None):
    """Split a full (host) matrix into this rank's ShardedArray."""
    comm = comm if comm is not None else Comm.default()
    X = torch.as_tensor(X)
    start, stop = shard_bounds(X.shape[0], comm.rank, comm.world_size)
    local = X[start:stop]
    if device is not None:
        local = local.to(device)
    return ShardedArray(local.contiguous(), X.shape[0], start, comm)
