"""Branch sharding over GPUs (one process per GPU) through the library's C ABI.

Branches share no weights, so a packed leapfrog step needs no
communication: each rank owns a contiguous range of branches (balanced by
marker count, bann_shard_branches) and their genotype columns.  The exchanges
live in the library (bann_dist.hip), on the context's communicator:
  * RCCL over xGMI (bann_ctx_comm_init; the 128-byte unique id travels over
    torch.distributed here), or
  * a caller all-reduce (bann_ctx_comm_callback), e.g. gloo on the CPU --
    TorchAllreduce below wraps torch.distributed.all_reduce as that callback.
bann_exchange_residual sums each rank's residual change after a leapfrog
session (the sweep bookkeeping of net.rs:292-300, over ranks); network-joint HMC
(bann_network_hmc_step) all-reduces the summed branch outputs every step.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence, Tuple

import numpy as np

from ._lib import ALLREDUCE_FN, BannError, load_library


def shard_ranges(marker_counts: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous branch ranges per rank with ~equal total markers (bann_shard_branches)."""
    counts = np.ascontiguousarray(marker_counts, dtype=np.int32)
    if world < 1 or world > counts.size:
        raise ValueError(f"cannot shard {counts.size} branches over {world} ranks (every rank needs a branch)")
    starts = np.zeros(world + 1, np.int32)
    rc = load_library().bann_shard_branches(counts.ctypes.data_as(C.POINTER(C.c_int32)), counts.size, world,
                                            starts.ctypes.data_as(C.POINTER(C.c_int32)))
    if rc != 0:
        raise BannError(rc, "bann_shard_branches")
    return [(int(starts[r]), int(starts[r + 1])) for r in range(world)]


class TorchAllreduce:
    """bann_allreduce_fn over torch.distributed (gloo on CPU tensors): the
    in-place host-buffer sum the library calls for a callback communicator."""

    def __init__(self, dist):
        self.dist = dist
        self.fn = ALLREDUCE_FN(self._call)   # keep a reference: the library holds the pointer

    def _call(self, user, buf, count, dtype):
        try:
            import torch
            ct, tt = (C.c_float, torch.float32) if dtype == 0 else (C.c_double, torch.float64)
            arr = np.ctypeslib.as_array(C.cast(buf, C.POINTER(ct)), shape=(count,))
            t = torch.from_numpy(arr)   # shares memory with the library's buffer
            if self.dist is not None and self.dist.is_initialized() and self.dist.get_world_size() > 1:
                self.dist.all_reduce(t)
            return 0
        except Exception:   # a Python exception must not cross the C boundary
            return 1


def residual_update(residual: np.ndarray, local_delta: np.ndarray, allreduce: TorchAllreduce | None):
    """residual -= sum over ranks of local_delta (bann_residual_update_host, in place)."""
    res = np.ascontiguousarray(residual, dtype=np.float32)
    dl = np.ascontiguousarray(local_delta, dtype=np.float32).copy()
    fn = allreduce.fn if allreduce is not None else ALLREDUCE_FN()
    rc = load_library().bann_residual_update_host(fn, None, dl.ctypes.data_as(C.POINTER(C.c_float)),
                                                  res.ctypes.data_as(C.POINTER(C.c_float)), res.size)
    if rc != 0:
        raise BannError(rc, "bann_residual_update_host")
    return res


def comm_unique_id() -> bytes:
    """128-byte RCCL unique id (rank 0), to be sent to the other ranks."""
    buf = (C.c_uint8 * 128)()
    rc = load_library().bann_comm_unique_id(buf)
    if rc != 0:
        raise BannError(rc, "bann_comm_unique_id")
    return bytes(buf)
