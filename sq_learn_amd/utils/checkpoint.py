"""Iteration-level checkpoint / resume for multi-GPU fits.

The reference only pickles fitted estimators (``base.py:296-320``) and has
no mid-fit resume.  A q-means iteration here is a pure function of
(centres, restart, iteration, seed): every random draw is Philox-keyed by
those, so storing the centres, the loop counters, the best-so-far iterate
and the host RandomState (used only by the initialisations) is enough to
continue a fit bit-identically after a crash or preemption.

Layout: ``<dir>/<tag>.state.pt`` (replicated state, written by rank 0) and
``<dir>/<tag>.rank<r>.pt`` (this rank's rows: best labels).  Writes go to a
temporary file and are renamed (atomic on POSIX), then all ranks meet at a
barrier, so a checkpoint is either complete or absent.  Files hold only
tensors and plain scalars and are read back with
``torch.load(weights_only=True)`` - nothing in them is executed.
"""

import os

import numpy as np
import torch


def rs_state_to_tensors(rs):
    name, keys, pos, has_gauss, cached = rs.get_state()
    return {"rs_keys": torch.as_tensor(np.asarray(keys, dtype=np.int64)), "rs_pos": int(pos),
            "rs_has_gauss": int(has_gauss), "rs_cached": float(cached)}


def rs_state_from_tensors(rs, st):
    keys = st["rs_keys"].numpy().astype(np.uint32)
    rs.set_state(("MT19937", keys, int(st["rs_pos"]), int(st["rs_has_gauss"]),
                  float(st["rs_cached"])))


class Checkpointer:
    def __init__(self, directory, comm, tag="fit", every=10):
        self.directory = directory
        self.comm = comm
        self.tag = tag
        self.every = int(every)
        if directory is not None and comm.rank == 0:
            os.makedirs(directory, exist_ok=True)

    @property
    def enabled(self):
        return self.directory is not None and self.every > 0

    def _state_path(self):
        return os.path.join(self.directory, f"{self.tag}.state.pt")

    def _rank_path(self, rank=None):
        r = self.comm.rank if rank is None else rank
        return os.path.join(self.directory, f"{self.tag}.rank{r}.pt")

    @staticmethod
    def _atomic_save(obj, path):
        tmp = path + ".tmp"
        torch.save(obj, tmp)
        os.replace(tmp, path)

    def due(self, iteration):
        return self.enabled and (iteration + 1) % self.every == 0

    def save(self, state, local):
        """``state``: replicated (identical on all ranks) dict; ``local``:
        this rank's tensors.  Host copies are made here."""
        if not self.enabled:
            return
        self.comm.barrier()
        # a generation tag ties the rank files to the state file: a crash
        # between the two writes leaves new rank files beside an old state,
        # which load() then rejects instead of mixing iterations
        self._generation = getattr(self, "_generation", 0) + 1
        gen = (int(state.get("restart", 0)) << 32) | (int(state.get("it", 0)) & 0xFFFFFFFF)
        tag = float(gen) * 1024.0 + float(self._generation % 1024)
        cpu_local = {k: (v.detach().cpu() if isinstance(v, torch.Tensor) else v)
                     for k, v in local.items()}
        cpu_local["_generation"] = torch.tensor([tag], dtype=torch.float64)
        # rank files first, then the state file that makes the set valid
        self._atomic_save(cpu_local, self._rank_path())
        self.comm.barrier()
        if self.comm.rank == 0:
            cpu_state = {k: (v.detach().cpu() if isinstance(v, torch.Tensor) else v)
                         for k, v in state.items()}
            cpu_state["world_size"] = self.comm.world_size
            cpu_state["_generation"] = torch.tensor([tag], dtype=torch.float64)
            self._atomic_save(cpu_state, self._state_path())
        self.comm.barrier()

    def load(self):
        """(state, local) or None when no complete, compatible checkpoint."""
        if self.directory is None:
            return None
        ok = torch.tensor([1.0 if os.path.exists(self._state_path())
                           and os.path.exists(self._rank_path()) else 0.0])
        self.comm.all_reduce_(ok, op="min")   # every rank must hold its part
        if float(ok.item()) < 1.0:
            return None
        state = torch.load(self._state_path(), weights_only=True)
        if int(state.get("world_size", 1)) != self.comm.world_size:
            return None
        local = torch.load(self._rank_path(), weights_only=True)
        # every rank's file must belong to the state's generation (all ranks)
        sg = state.get("_generation")
        lg = local.get("_generation")
        same = torch.tensor([1.0 if (sg is None and lg is None) or
                             (sg is not None and lg is not None and torch.equal(sg, lg)) else 0.0])
        self.comm.all_reduce_(same, op="min")
        if float(same.item()) < 1.0:
            return None
        state.pop("_generation", None)
        local.pop("_generation", None)
        return state, local

    def clear(self):
        if self.directory is None:
            return
        self.comm.barrier()
        for p in (self._rank_path(),) + ((self._state_path(),) if self.comm.rank == 0 else ()):
            try:
                os.remove(p)
            except FileNotFoundError:
                pass
        self.comm.barrier()
