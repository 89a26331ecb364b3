"""Packet sharding across the GPUs of one node.

Frames are independent on this path (no cross-packet state; the socket table is a read-only replica per GPU), so a
batch shards by contiguous frame ranges balanced by bytes (sum of frame lengths), not by frame count — that matters
for IMIX. The only exchange is the per-flow (and per-verdict) packet counters, reduced with one all-reduce over RCCL
(torch.distributed "nccl" backend on ROCm) — or gloo on CPU for tests.
"""
from __future__ import annotations

import numpy as np


def byte_balanced_shards(lens: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Contiguous [begin, end) frame ranges, one per rank, splitting sum(lens) as evenly as frame boundaries allow."""
    n = len(lens)
    if world <= 0:
        raise ValueError("world must be >= 1")
    csum = np.cumsum(lens, dtype=np.int64)
    total = int(csum[-1]) if n else 0
    bounds = [0]
    for r in range(1, world):
        target = total * r // world
        # first frame index whose prefix sum reaches the target
        bounds.append(int(np.searchsorted(csum, target, side="left")) + (1 if n else 0))
    bounds.append(n)
    bounds = [min(max(b, 0), n) for b in bounds]
    for k in range(1, len(bounds)):  # keep monotone
        bounds[k] = max(bounds[k], bounds[k - 1])
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def allreduce_counts(counts, group=None) -> None:
    """Sum a rank's counter tensor (int64 flow or verdict counts) over all ranks, in place."""
    import torch.distributed as dist

    dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
