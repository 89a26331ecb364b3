"""Packet sharding across the GPUs of one node.

Frames are independent on this path (no cross-packet state; the socket table is a read-only replica per GPU), so a
batch shards by contiguous frame ranges balanced by bytes (sum of frame lengths), not by frame count — that matters
for IMIX. The only exchange is the per-flow (and per-verdict) packet counters: one grouped all-reduce per batch over
RCCL / xGMI through the C ABI (dk_rx_flow_counts_allreduce on a dk_comm.h communicator). Per-frame results stay on
their GPU; frame bytes never cross xGMI.

`ShardedReceiver` is the per-rank driver bench.py --gpus N runs (one process per GPU under torchrun): it bootstraps
the RCCL communicator (rank 0's id handed out over the launcher's process group), receives the rank's shard and
all-reduces the counters on a side stream so the reduction of batch k overlaps the kernel of batch k + 1. The CPU
rehearsal (tests/test_multiproc.py, gloo, world size 2) drives the same sharding and bootstrap code with torch's
all_reduce standing in for the RCCL call, which is covered on the GPU by a 1-rank communicator test.
"""
from __future__ import annotations

from typing import Callable, Optional

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


def broadcast_comm_id(dist, make_id: Callable[[], bytes]) -> bytes:
    """Rank 0 makes the RCCL bootstrap id (dk_comm_unique_id); every rank gets it over the launcher's process group."""
    obj = [make_id() if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def allreduce_counts(counts, group=None) -> None:
    """CPU rehearsal stand-in for dk_rx_flow_counts_allreduce: sum a rank's counter tensor over all ranks, in place."""
    import torch.distributed as dist

    dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)


class TorchCountsAllreduce:
    """Fallback when the receive path's own RCCL communicator (dk_comm.h) cannot be created on a node: the same
    all-reduce of the counter arrays through torch.distributed's RCCL (backend "nccl") process group."""

    def __init__(self, group):
        self.group = group

    def __call__(self, results, stream) -> None:
        import torch
        import torch.distributed as dist

        with torch.cuda.stream(stream):
            dist.all_reduce(results.t["flow_counts"], op=dist.ReduceOp.SUM, group=self.group)
            dist.all_reduce(results.t["verdict_counts"], op=dist.ReduceOp.SUM, group=self.group)


class ShardedReceiver:
    """One rank of a packet-sharded receive: its engine, its RCCL communicator, and double-buffered counters whose
    all-reduce runs on a side stream (the collective of batch k overlaps the kernel of batch k + 1)."""

    def __init__(self, engine, results, comm, stream, nbuf: int = 2):
        import torch

        from .rx import RxResults

        self.eng, self.comm, self.stream = engine, comm, stream
        self.side = torch.cuda.Stream(device=stream.device)
        self.res = [results]
        for _ in range(nbuf - 1):  # same per-frame arrays, own counters
            r = RxResults.__new__(RxResults)
            r.n, r.t = results.n, dict(results.t)
            r.t["flow_counts"] = torch.zeros_like(results.t["flow_counts"])
            r.t["verdict_counts"] = torch.zeros_like(results.t["verdict_counts"])
            self.res.append(r)
        self.done = [None] * nbuf
        self.k = 0

    def step(self, batch) -> None:
        import torch

        slot = self.k % len(self.res)
        r = self.res[slot]
        if self.comm is not None:  # per-step counters, all-reduced (N = 1: they accumulate over steps, no reset)
            if self.done[slot] is not None:  # this slot's previous all-reduce has finished before the reset
                self.stream.wait_event(self.done[slot])
            r.t["flow_counts"].zero_()
            r.t["verdict_counts"].zero_()
        self.eng.receive_batch(batch, r, stream=self.stream)
        if self.comm is not None:
            ev = torch.cuda.Event()
            ev.record(self.stream)
            self.side.wait_event(ev)
            if isinstance(self.comm, TorchCountsAllreduce):
                self.comm(r, self.side)
            else:
                self.eng.counts_allreduce(r, self.comm.handle, stream=self.side)
            done = torch.cuda.Event()
            done.record(self.side)
            self.done[slot] = done
        self.k += 1

    def drain(self) -> None:
        self.side.synchronize()
        self.stream.synchronize()

    def counts(self, slot: Optional[int] = None):
        """The counters of the last step (or of `slot`)."""
        s = (self.k - 1) % len(self.res) if slot is None else slot
        return self.res[s].t["flow_counts"], self.res[s].t["verdict_counts"]
