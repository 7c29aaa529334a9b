"""Branch sharding over GPUs (one process per GPU, torch.distributed / RCCL).

Branches share no weights, so a packed leapfrog step needs no
communication: each rank owns a contiguous range of branches (balanced by
marker count) and their genotype columns.  The only exchange is per trajectory
/ Gibbs sweep: the n-vector change of the summed branch predictions (the
network output, net.rs:545-559), all-reduced so that every rank holds the same
residual (net.rs:279-300), plus a few scalars (output-weight sum of squares,
architectures.rs:175-185).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


def shard_ranges(marker_counts: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous branch ranges per rank with ~equal total markers."""
    counts = np.asarray(marker_counts, dtype=np.int64)
    B = counts.size
    if world <= 1:
        return [(0, B)]
    csum = np.concatenate([[0], np.cumsum(counts)])
    total = csum[-1]
    cuts = [0]
    for r in range(1, world):
        target = total * r / world
        cuts.append(int(np.clip(np.searchsorted(csum, target, side="left"), cuts[-1], B)))
    cuts.append(B)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def allreduce_sum_(tensor, dist=None):
    """In-place sum over ranks (RCCL for CUDA tensors, gloo on CPU)."""
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(tensor)
    return tensor


def update_residual(residual, local_delta, dist=None):
    """residual -= all_reduce(local_delta)   (net.rs:292-300 for every rank's branches)."""
    allreduce_sum_(local_delta, dist)
    residual -= local_delta
    return residual
