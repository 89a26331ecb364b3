"""ShardedReceiver's bookkeeping on the CPU (no GPU, no RCCL): which counter set each batch adds to, when a deferred
batch's counts are completed (by the next launch on the stream, or flush), and when each set is gathered — replayed in
program order by a stand-in engine that applies DK_RX_BATCH_DEFER_COUNTS exactly as dk_rx.h specifies (a deferred
launch's increments land in ITS counters when the next launch on the stream, or dk_rx_counts_flush, runs) and a
stand-in collective that sums the set over `world` identical ranks. For every gather period, deferral on/off and step
count, the node-wide counts after drain() equal steps x world x one batch's counts, and every all-reduce reads a set
after the last completion of its counts that precede it."""
import numpy as np
import pytest
import torch

from demikernel_amd import shard


class FakeStream:
    device = "cpu"

    def wait_event(self, ev):
        pass

    def synchronize(self):
        pass


class FakeEvent:
    def record(self, stream=None):
        pass


class Res:
    def __init__(self, nflows):
        self.n = 1
        self.t = {"flow_counts": torch.zeros(nflows, dtype=torch.int64),
                  "verdict_counts": torch.zeros(4, dtype=torch.int64)}

    def zero_counts(self):
        for v in self.t.values():
            v.zero_()


class FakeEngine:
    """dk_rx_process semantics for the counters only: one batch adds `inc` to its results' counters, at once or,
    deferred, when the stream's next launch or a flush runs."""

    def __init__(self, inc_f, inc_v, world):
        self.inc_f, self.inc_v, self.world = inc_f, inc_v, world
        self.pending = None
        self.log = []

    def _complete(self):
        if self.pending is not None:
            r = self.pending
            r.t["flow_counts"] += self.inc_f
            r.t["verdict_counts"] += self.inc_v
            self.log.append(("complete", id(r)))
            self.pending = None

    def receive_batch(self, batch, res, stream=None, defer_counts=False):
        self._complete()
        if defer_counts:
            self.pending = res
        else:
            res.t["flow_counts"] += self.inc_f
            res.t["verdict_counts"] += self.inc_v
            self.log.append(("complete", id(res)))

    def flush_counts(self, stream=None):
        self._complete()

    def counts_allreduce_to(self, res, fo, vo, comm, stream=None):
        fo.copy_(res.t["flow_counts"] * self.world)  # world identical ranks
        vo.copy_(res.t["verdict_counts"] * self.world)
        self.log.append(("gather", id(res)))


class Comm:
    handle = 1


@pytest.mark.parametrize("every", [1, 2, 3, 8])
@pytest.mark.parametrize("defer", [True, False])
@pytest.mark.parametrize("steps", [1, 2, 5, 8, 17])
def test_gathered_counts_exact(monkeypatch, every, defer, steps):
    monkeypatch.setattr(torch.cuda, "Stream", lambda device=None: FakeStream())
    monkeypatch.setattr(torch.cuda, "Event", lambda *a, **k: FakeEvent())
    monkeypatch.setattr(shard, "TorchCountsAllreduce", type("T", (), {}))  # not the stand-in's path
    world = 4
    inc_f = torch.arange(1, 6, dtype=torch.int64)
    inc_v = torch.tensor([3, 0, 1, 2], dtype=torch.int64)
    eng = FakeEngine(inc_f, inc_v, world)
    import demikernel_amd.rx as rx

    monkeypatch.setattr(rx, "RxResults", Res)
    sr = shard.ShardedReceiver(eng, Res(5), Comm(), FakeStream(), defer=defer, gather_every=every)
    for _ in range(steps):
        sr.step(None)
    sr.drain()
    fo, vo = sr.counts()
    assert torch.equal(fo, steps * world * inc_f), (fo, every, defer, steps)
    assert torch.equal(vo, steps * world * inc_v)
    # every gather of a set comes after that set's completions logged before it, and the last event of each set
    # is a gather (nothing completed after its final gather)
    last = {}
    for kind, sid in eng.log:
        last[sid] = kind
    assert all(k == "gather" for k in last.values()), eng.log
    n_gathers = sum(1 for k, _ in eng.log if k == "gather")
    assert n_gathers <= -(-steps // every) + 2, (n_gathers, steps, every)


class LoggedStream:
    device = "cpu"

    def __init__(self, name, log):
        self.name, self.log = name, log

    def wait_event(self, ev):
        self.log.append(("wait", self.name, ev.id))

    def synchronize(self):
        pass


class LoggedEvent:
    count = 0

    def __init__(self, log):
        LoggedEvent.count += 1
        self.id, self.log = LoggedEvent.count, log

    def record(self, stream=None):
        self.log.append(("record", self.id, stream.name))


class ImmediateFlowEngine(FakeEngine):
    """A flow table above DK_RX_MAX_DEFERRED_FLOWS (dk_rx.h): with DK_RX_BATCH_DEFER_COUNTS only the verdict counts
    wait for the next launch; flow counts land in the launch's own set at once."""

    flow_counts_deferred = False

    def __init__(self, inc_f, inc_v, world, log):
        super().__init__(inc_f, inc_v, world)
        self.glog = log
        self.pend_v = None

    def _complete(self):
        if self.pend_v is not None:
            self.pend_v.t["verdict_counts"] += self.inc_v
            self.glog.append(("mutate", id(self.pend_v)))
            self.pend_v = None

    def receive_batch(self, batch, res, stream=None, defer_counts=False):
        self._complete()
        res.t["flow_counts"] += self.inc_f
        self.glog.append(("mutate", id(res)))
        if defer_counts:
            self.pend_v = res
        else:
            res.t["verdict_counts"] += self.inc_v

    def counts_allreduce_to(self, res, fo, vo, comm, stream=None):
        super().counts_allreduce_to(res, fo, vo, comm, stream)
        self.glog.append(("gather", id(res), stream.name))


@pytest.mark.parametrize("every", [1, 2, 3])
@pytest.mark.parametrize("steps", [2, 5, 9])
def test_immediate_flow_counts_wait_for_their_sets_gather(monkeypatch, every, steps):
    """a launch that adds flow counts to its set immediately (large tables) must first wait for that set's
    previous all-reduce on the side stream: every mutation of a set after its gather is preceded, on the launch stream,
    by a wait on the event recorded after that gather."""
    log = []
    monkeypatch.setattr(torch.cuda, "Stream", lambda device=None: LoggedStream("side", log))
    monkeypatch.setattr(torch.cuda, "Event", lambda *a, **k: LoggedEvent(log))
    monkeypatch.setattr(shard, "TorchCountsAllreduce", type("T", (), {}))
    import demikernel_amd.rx as rx

    monkeypatch.setattr(rx, "RxResults", Res)
    world = 2
    inc_f = torch.arange(1, 6, dtype=torch.int64)
    inc_v = torch.tensor([3, 0, 1, 2], dtype=torch.int64)
    eng = ImmediateFlowEngine(inc_f, inc_v, world, log)
    sr = shard.ShardedReceiver(eng, Res(5), Comm(), LoggedStream("main", log), defer=True, gather_every=every)
    for _ in range(steps):
        sr.step(None)
    sr.drain()
    fo, vo = sr.counts()
    assert torch.equal(fo, steps * world * inc_f) and torch.equal(vo, steps * world * inc_v)
    for p, e in enumerate(log):
        if e[0] != "mutate":
            continue
        gathers = [q for q in range(p) if log[q][0] == "gather" and log[q][1] == e[1]]
        if not gathers:
            continue
        q = gathers[-1]
        done = next(x[1] for x in log[q:] if x[0] == "record" and x[2] == "side")
        assert ("wait", "main", done) in log[q:p], (p, log)


def test_one_gpu_no_collective(monkeypatch):
    monkeypatch.setattr(torch.cuda, "Stream", lambda device=None: FakeStream())
    monkeypatch.setattr(torch.cuda, "Event", lambda *a, **k: FakeEvent())
    inc_f = torch.arange(1, 6, dtype=torch.int64)
    inc_v = torch.tensor([3, 0, 1, 2], dtype=torch.int64)
    eng = FakeEngine(inc_f, inc_v, 1)
    sr = shard.ShardedReceiver(eng, Res(5), None, FakeStream())
    for _ in range(7):
        sr.step(None)
    sr.drain()
    fo, vo = sr.counts()
    assert torch.equal(fo, 7 * inc_f) and torch.equal(vo, 7 * inc_v)
    assert not any(k == "gather" for k, _ in eng.log)
    assert np.array_equal(fo.numpy(), (7 * inc_f).numpy())
