"""Packet sharding across the GPUs of one node.

Frames are independent on this path (no cross-packet state; the socket table is a read-only replica per GPU), so a
batch shards by contiguous frame ranges balanced by bytes (sum of frame lengths), not by frame count — that matters
for IMIX. The only exchange is the per-flow (and per-verdict) packet counters: one grouped all-reduce per batch over
RCCL / xGMI through the C ABI (dk_rx_flow_counts_allreduce on a dk_comm.h communicator). Per-frame results stay on
their GPU; frame bytes never cross xGMI.

`ShardedReceiver` is the per-rank driver bench.py --gpus N runs (one process per GPU under torchrun): it bootstraps
the RCCL communicator (rank 0's id handed out over the launcher's process group), receives the rank's shard into
accumulating counters (each batch's counter rows completed inside the next batch's kernel) and all-reduces them out of
place every K batches (bench.py: K = 8, on the launch stream, since RCCL's kernel does not run beside the persistent
receive kernels); no step zeroes anything. The CPU rehearsal (tests/test_multiproc.py, gloo, world size 2)
drives the same sharding and bootstrap code with torch's all_reduce standing in for the RCCL call; on the GPU the
RCCL call runs through a 1-rank communicator test, and bench.py --gpus 2 runs as two child ranks on one GPU
(tests/test_gpu_multiproc.py, gloo counts: RCCL refuses two ranks on one device).
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
    """TEST-ONLY stand-in for the product collective (dk_rx_flow_counts_allreduce_to over a dk_comm.h RCCL
    communicator) when RCCL cannot run: the CPU gloo rehearsal, and 2-rank GPU tests on ONE GPU (RCCL refuses two
    ranks on one device, rccl.h). The same out-of-place sum of the counter arrays through torch.distributed. bench.py
    uses it only under --counts-via-torch-gloo-test and says so in its JSON line; a failed RCCL init otherwise ends the
    run with an error."""

    def __init__(self, group):
        self.group = group

    def to(self, results, flow_out, verdict_out, stream) -> None:
        import torch
        import torch.distributed as dist

        with torch.cuda.stream(stream):
            flow_out.copy_(results.t["flow_counts"])
            verdict_out.copy_(results.t["verdict_counts"])
            dist.all_reduce(flow_out, op=dist.ReduceOp.SUM, group=self.group)
            dist.all_reduce(verdict_out, op=dist.ReduceOp.SUM, group=self.group)


class ShardedReceiver:
    """One rank of a packet-sharded receive: its engine, its RCCL communicator, and `nbuf` sets of accumulating
    counters. Steps are grouped in gather periods of `gather_every` steps; the steps of period j add their counts to
    the set of slot j % nbuf (never zeroed: no memset kernels on the launch stream). With `defer` (the default) each
    kernel leaves its counter rows pending (DK_RX_BATCH_DEFER_COUNTS) and the next step's kernel adds them inside its
    own launch, so no step pays a dependent second launch for its counters. Once a period's counts are complete (after
    the first kernel of the next period), dk_rx_flow_counts_allreduce_to sums that set over the ranks into the slot's
    node-wide totals, on a side stream (side_stream=True) or between two kernels on the launch stream. A set is changed again only after its
    previous all-reduce has read it (one event wait). flush() completes the last step and gathers it. The node-wide
    counts of every step so far are the sum of the slots' totals (`counts()`), exact at every gather.

    gather_every = 1 gathers after every batch; tools/overlap_collective.py measured that RCCL's kernel does not run
    beside the receive kernels (they hold every CU), so each gather costs the step ~its own time (~10 us); gathering
    every K batches keeps the totals exact at each gather and divides that cost by K.
    With comm=None (one GPU) there is one set and no collective."""

    def __init__(self, engine, results, comm, stream, nbuf: int = 2, defer: bool = True, gather_every: int = 1,
                 side_stream: bool = True):
        """side_stream=False issues the all-reduce on the launch stream itself (serialised between two kernels)."""
        import torch

        from .rx import RxResults

        self.eng, self.comm, self.stream, self.defer = engine, comm, stream, defer
        self.every = max(int(gather_every), 1)
        if comm is None:
            nbuf = 1
        self.side = (torch.cuda.Stream(device=stream.device) if side_stream else stream) if comm is not None else None
        results.zero_counts()
        self.res = [results]
        for _ in range(nbuf - 1):  # same per-frame arrays, own counters
            r = RxResults.__new__(RxResults)
            r.n, r.t = results.n, dict(results.t)
            r.t["flow_counts"] = torch.zeros_like(results.t["flow_counts"])
            r.t["verdict_counts"] = torch.zeros_like(results.t["verdict_counts"])
            self.res.append(r)
        self.tot = [(torch.zeros_like(r.t["flow_counts"]), torch.zeros_like(r.t["verdict_counts"])) for r in self.res] \
            if comm is not None else None
        self.done = [None] * nbuf     # the event after each set's latest all-reduce
        self.waited = [True] * nbuf   # the launch stream already waits for that event
        self.k = 0
        self.pending = None  # the set whose counts wait for the next launch (deferred rows)

    def reduce(self, slot: int, stream) -> None:
        """The slot's node-wide totals from every rank's accumulated set (on `stream`)."""
        r, (fo, vo) = self.res[slot], self.tot[slot]
        if isinstance(self.comm, TorchCountsAllreduce):
            self.comm.to(r, fo, vo, stream)
        else:
            self.eng.counts_allreduce_to(r, fo, vo, self.comm.handle, stream=stream)

    def _allreduce_after(self, slot: int) -> None:
        """All-reduce `slot`'s set on the side stream once the launch stream has completed its counts."""
        import torch

        ev = torch.cuda.Event()
        ev.record(self.stream)
        self.side.wait_event(ev)
        self.reduce(slot, self.side)
        done = torch.cuda.Event()
        done.record(self.side)
        self.done[slot] = done
        self.waited[slot] = False

    def _before_change(self, slot) -> None:
        """The launch stream is about to add to set `slot`: its previous all-reduce must have read it."""
        if slot is not None and not self.waited[slot]:
            self.stream.wait_event(self.done[slot])
            self.waited[slot] = True

    def step(self, batch) -> None:
        slot = (self.k // self.every) % len(self.res)
        prev, prev_k = self.pending, self.k - 1
        # the sets this launch changes: deferred, the pending one it completes (its own rows stay pending) — and its
        # own too when the engine counts flows inside the launch (tables above DK_RX_MAX_DEFERRED_FLOWS, dk_rx.h);
        # otherwise its own
        self._before_change(prev if self.defer else slot)
        if self.defer and not getattr(self.eng, "flow_counts_deferred", True):
            self._before_change(slot)
        self.eng.receive_batch(batch, self.res[slot], stream=self.stream, defer_counts=self.defer)
        if self.comm is not None:
            if self.defer:
                if prev is not None and (prev_k + 1) % self.every == 0:  # step prev_k ended a gather period
                    self._allreduce_after(prev)
            elif (self.k + 1) % self.every == 0:
                self._allreduce_after(slot)
        self.pending = slot if self.defer else None
        self.k += 1

    def flush(self) -> None:
        """Complete the last deferred step's counters and gather whatever has not been gathered yet."""
        if self.pending is not None:
            s = self.pending
            self._before_change(s)
            self.eng.flush_counts(self.stream)
            self.pending = None
            if self.comm is not None:  # the last step's set, whether or not it ended a period
                self._allreduce_after(s)
        elif self.comm is not None and not self.defer and self.k % self.every != 0:
            self._allreduce_after(((self.k - 1) // self.every) % len(self.res))

    def drain(self) -> None:
        self.flush()
        if self.side is not None:
            self.side.synchronize()
        self.stream.synchronize()

    def counts(self):
        """Node-wide (comm) or this GPU's (no comm) flow and verdict counts of every step so far. Call after drain()."""
        if self.comm is None:
            return self.res[0].t["flow_counts"], self.res[0].t["verdict_counts"]
        used = [s for s in range(len(self.res)) if self.done[s] is not None]
        fo = sum(self.tot[s][0] for s in used) if used else self.tot[0][0]
        vo = sum(self.tot[s][1] for s in used) if used else self.tot[0][1]
        return fo, vo
