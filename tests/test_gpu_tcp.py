"""GPU parity of established-state TCP receive processing (dk_tcp_rx_process) with the CPU
restatement (oracle/dk_tcp_oracle.cpp): every per-frame action and view, every delivered buffer and the whole
connection table (RCV.NXT, state, FIN, the out-of-order store) bit for bit — on the hand-built branch scenarios of
tests/test_tcp_oracle.py and on synthetic streams that go through dk_rx first (frames -> verdicts/flow ids ->
TCP), over several batches so state carries across calls."""
import numpy as np
import pytest

import test_tcp_oracle as S
from demikernel_amd import Config, FrameBatch, RxEngine, RxResults, synth
from demikernel_amd import _native as N
from demikernel_amd.rx import Fail
from demikernel_amd.tcp import TcpOut, TcpReceiver
from oracle import oracle as O
from oracle.oracle import OraclePeer

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["lane", "wave", "relay", "scan"])
def tcp(request):
    """Every test runs through every walk: lanes = connections, one wave per connection with the parallel in-order
    check, 8 waves per connection relaying its state window to window, and the scan walk (windows precomputed across
    the chip, 64 windows per wave scan, the undecided ones through the state machine) (DK_TCP_WALK forces the choice
    the engine otherwise makes from the batch; dk_diag_tcp_set_walk forces one)."""
    import torch

    assert torch.cuda.is_available()
    r = TcpReceiver(0, walk=request.param)
    yield r
    r.close()


def rx_device(rx: dict):
    import torch

    n = len(rx["meta"])
    r = RxResults(n, 1, device=torch.device("cuda", 0), tcp_fields=True, counts=False)
    for k in ("meta", "flow_id", "tcp_seq", "tcp_ack", "payload"):
        r.t[k].copy_(torch.from_numpy(np.ascontiguousarray(rx[k], np.uint32).view(np.int32)))
    return r


def gpu_process(tcp, table: np.ndarray, r: RxResults) -> tuple[np.ndarray, dict]:
    import torch

    conns = tcp.conns_to_device(table)
    out = TcpOut(r.n, len(table))
    tcp.process(r, conns, out)
    torch.cuda.synchronize()
    return tcp.conns_to_host(conns), out.to_numpy()


def assert_same(got_t, got, exp_t, exp, ctx=""):
    for k in ("action", "view", "deliv_start", "deliv_count"):
        if not np.array_equal(got[k], exp[k]):
            bad = np.nonzero(got[k] != exp[k])[0][:8]
            raise AssertionError(f"{ctx}: {k} differs at {bad}: got {got[k][bad]} exp {exp[k][bad]}")
    for c in range(len(exp_t)):  # only the used delivery slots are defined
        s, m = int(exp["deliv_start"][c]), int(exp["deliv_count"][c])
        assert np.array_equal(got["deliv"][s:s + m], exp["deliv"][s:s + m]), f"{ctx}: deliv of conn {c}"
    if not np.array_equal(got_t.view(np.uint8), exp_t.view(np.uint8)):
        bad = np.nonzero((got_t.view(np.uint8).reshape(len(got_t), -1) !=
                          exp_t.view(np.uint8).reshape(len(exp_t), -1)).any(1))[0][:8]
        raise AssertionError(f"{ctx}: connection table differs at {bad}: got {got_t[bad]} exp {exp_t[bad]}")


SCENARIOS = {
    "fin_in_order": (S.conns(rn=1), [(0, 1, 1, S.FIN | S.ACK, 0)]),
    "ooo_fin": (S.conns(rn=1, snd=1001), [(0, 1001, 1001, S.FIN | S.ACK, 0), (0, 1, 1001, S.PSH | S.ACK, 1000)]),
    "dup_partial": (S.conns(rn=1001), [(0, 1, 1, S.ACK, 1000), (0, 501, 1, S.ACK, 1000)]),
    "window": (S.conns(rn=1), [(0, 65536, 1, S.ACK, 10), (0, 65535, 1, S.ACK, 10)]),
    "fin_trim": (S.conns(rn=1, bufsz=100), [(0, 1, 1, S.FIN | S.ACK, 100)]),
    "zero_window": (S.conns(rn=1001, reader=1, bufsz=1000), [(0, 1001, 1, S.ACK, 10)]),
    "syn": (S.conns(rn=100), [(0, 99, 1, S.SYN | S.ACK, 100), (0, 200, 1, S.SYN | S.ACK, 0)]),
    "wrap": (S.conns(rn=0xFFFFFF00), [(0, 0xFFFFFF00, 1, S.ACK, 1000), (0, 0xFFFFFF00, 1, S.ACK, 1000),
                                      (0, 0x2E8, 1, S.ACK, 8)]),
    "rst": (S.conns(rn=1), [(0, 0, 1, S.RST | S.ACK, 0), (0, 1, 1, S.RST, 0), (0, 1, 1, S.ACK, 10)]),
    "ack": (S.conns(rn=1, snd=5), [(0, 1, 0xFFFFFFF0, S.ACK, 0), (0, 1, 10, S.ACK, 0), (0, 1, 5, S.PSH, 10)]),
    "recovery": (S.conns(rn=1), [(0, 1001, 1, S.ACK, 1000), (0, 2001, 1, S.ACK, 1000), (0, 1, 1, S.ACK, 1000)]),
    "encompass": (S.conns(rn=1), [(0, 1501, 1, S.ACK, 100), (0, 1521, 1, S.ACK, 50), (0, 1001, 1, S.ACK, 1000)]),
    "end_overlap": (S.conns(rn=1), [(0, 1001, 1, S.ACK, 1000), (0, 1501, 1, S.ACK, 1000), (0, 1, 1, S.ACK, 1000)]),
    "front_overlap": (S.conns(rn=1), [(0, 2001, 1, S.ACK, 1000), (0, 1501, 1, S.ACK, 1000), (0, 1, 1, S.ACK, 1500)]),
    "sixteen": (S.conns(rn=1), [(0, 1001 + 200 * k, 1, S.ACK, 100) for k in range(17)] + [(0, 801, 1, S.ACK, 100)]),
    "ooo_fin_data": (S.conns(rn=1), [(0, 1001, 1, S.FIN | S.ACK, 100), (0, 1, 1, S.ACK, 1000),
                                     (0, 1102, 1, S.ACK, 5)]),
    "skip_layout": (S.conns(4, rn=1), [(0, 1, 1, S.ACK, 10), (1, 1, 1, S.ACK, 10), (2, 1, 1, S.ACK, 10),
                                       (1, 11, 1, S.ACK, 10), (N.DK_FLOW_NONE, 1, 1, S.ACK, 10),
                                       (3, 1, 1, S.ACK, 10, 25), (7, 1, 1, S.ACK, 10), (3, 1, 1, S.FIN | S.ACK, 0)]),
    "closed": (S.conns(2, rn=1, state=N.DK_TCP_CLOSED), [(0, 1, 1, S.ACK, 10), (1, 1, 1, S.ACK, 0)]),
    "empty_batch": (S.conns(3, rn=1), []),
    # store full, then segments after every entry (inserted and popped: STORED with no change), one without ACK, one
    # trimmed at the window end, a retransmission inside the store, and the hole filled (the store drains)
    "full_store_beyond": (S.conns(rn=1, bufsz=6000), [(0, 1001 + 200 * k, 1, S.ACK, 100) for k in range(16)] +
                          [(0, 5001, 1, S.ACK, 100), (0, 5201, 1, S.PSH, 100), (0, 5950, 1, S.ACK, 100),
                           (0, 5600, 9, S.ACK, 10), (0, 1201, 1, S.ACK, 50), (0, 1, 1, S.ACK, 1000),
                           (0, 5401, 1, S.ACK, 100)]),
    # long in-order runs (64-segment windows of the wave walk) with drops between and a stored segment whose front
    # an in-order push does not reach exactly
    "long_runs": (S.conns(rn=1), [(0, 1 + 10 * k, 1, S.ACK, 10) for k in range(150)] +
                  [(0, 3001, 1, S.ACK, 10), (0, 1, 1, S.ACK, 10)] +
                  [(0, 1501 + 10 * k, 1, S.ACK, 10) for k in range(149)] + [(0, 2991, 1, S.ACK, 20)]),
    # partial retransmissions inside in-order runs (the wave walk's parallel check trims and delivers them): plain,
    # one re-trimming the next in-order segment, one without ACK, one ending at the store's front (drains), one
    # ending past the window end, then a segment past the window
    "partial_runs": (S.conns(rn=1, bufsz=5000), [(0, 4001, 1, S.ACK, 100)] +
                     [(0, 1 + 100 * k, 1, S.ACK, 100) for k in range(30)] +
                     [(0, 2951, 1, S.ACK, 100), (0, 3001, 1, S.ACK, 100), (0, 3050, 1, S.PSH, 100)] +
                     [(0, 3101 + 100 * k, 1, S.ACK, 100) for k in range(8)] +
                     [(0, 3851, 1, S.ACK, 150), (0, 4051, 1, S.ACK, 100)] +
                     [(0, 4151 + 100 * k, 1, S.ACK, 100) for k in range(8)] +
                     [(0, 4901, 1, S.ACK, 200), (0, 5001, 1, S.ACK, 10)]),
    # retransmitted SYNs inside in-order runs (the relay walk's check takes the reached ones as data): partial, at
    # RCV.NXT, past it, partial without ACK, partial ending at the store's front (drains), partial ending past the
    # window end, entirely old
    "syn_runs": (S.conns(rn=1, bufsz=6000), [(0, 5001, 1, S.ACK, 100)] +
                 [(0, 1 + 100 * k, 1, S.ACK, 100) for k in range(20)] +
                 [(0, 1951, 1, S.SYN | S.ACK, 100), (0, 2001, 1, S.ACK, 100), (0, 2101, 1, S.SYN | S.ACK, 50),
                  (0, 2500, 1, S.SYN | S.ACK, 10)] +
                 [(0, 2101 + 100 * k, 1, S.ACK, 100) for k in range(10)] + [(0, 3050, 1, S.SYN, 100)] +
                 [(0, 3101 + 100 * k, 1, S.ACK, 100) for k in range(18)] + [(0, 4850, 1, S.SYN | S.ACK, 150)] +
                 [(0, 5101 + 100 * k, 1, S.ACK, 100) for k in range(8)] +
                 [(0, 5850, 1, S.SYN | S.ACK, 200), (0, 100, 1, S.SYN | S.ACK, 50)]),
    # segments the key pass classifies without a walk (past the window end: OUT_OF_WINDOW; ending before the table's
    # RCV.NXT: DUPLICATE) queued behind a FIN / an RST that closes the connection become UNPROCESSED
    # (dk_tcp_fix_kernel); before the close they keep their class
    "fin_then_classified": (S.conns(rn=1001, bufsz=1000), [(0, 1001, 1, S.ACK, 10), (0, 1011, 1, S.FIN | S.ACK, 0),
                                                           (0, 5000, 1, S.ACK, 10), (0, 1, 1, S.ACK, 10)]),
    "rst_then_classified": (S.conns(rn=1001, bufsz=1000), [(0, 1001, 1, S.ACK, 10), (0, 1011, 1, S.RST, 0),
                                                           (0, 5000, 1, S.ACK, 10), (0, 1, 1, S.ACK, 10)]),
    "classified_then_close": (S.conns(rn=1001, bufsz=1000), [(0, 5000, 1, S.ACK, 10), (0, 1, 1, S.ACK, 10),
                                                             (0, 1001, 1, S.ACK, 10), (0, 1011, 1, S.FIN | S.ACK, 0),
                                                             (0, 6000, 1, S.ACK, 10)]),
}
EXPECT = {  # what the oracle says these scenarios must exercise (guards the scenarios themselves)
    "fin_then_classified": ["DELIVERED", "FIN", "UNPROCESSED", "UNPROCESSED"],
    "rst_then_classified": ["DELIVERED", "RST", "UNPROCESSED", "UNPROCESSED"],
    "classified_then_close": ["OUT_OF_WINDOW", "DUPLICATE", "DELIVERED", "FIN", "UNPROCESSED"],
}


@pytest.mark.parametrize("name", list(SCENARIOS))
def test_branch_scenarios(tcp, name):
    table, segs = SCENARIOS[name]
    if name == "skip_layout":
        table = table.copy()
        table["state"][2] = N.DK_TCP_NONE
    rx = S.batch(segs) if segs else {k: np.zeros(0, np.uint32) for k in
                                     ("meta", "flow_id", "tcp_seq", "tcp_ack", "payload")}
    exp_t = table.copy()
    exp = O.tcp_process(exp_t, rx)
    if name in EXPECT:
        assert S.acts(exp) == EXPECT[name], S.acts(exp)
    got_t, got = gpu_process(tcp, table.copy(), rx_device(rx))
    assert_same(got_t, got, exp_t, exp, name)


def test_carried_out_of_order_store(tcp):
    """A store left by one call is recovered by the next (the table is the only state between calls)."""
    t = S.conns(rn=1)
    b1 = S.batch([(0, 1001, 1, S.ACK, 1000), (0, 3001, 1, S.ACK, 1000)])
    b2 = S.batch([(0, 2001, 1, S.ACK, 1000), (0, 1, 1, S.ACK, 1000)])
    exp_t = t.copy()
    O.tcp_process(exp_t, b1)
    exp2 = O.tcp_process(exp_t, b2)
    got_t, _ = gpu_process(tcp, t.copy(), rx_device(b1))
    got_t, got2 = gpu_process(tcp, got_t, rx_device(b2))
    assert_same(got_t, got2, exp_t, exp2, "carry")
    assert int(got_t["receive_next"][0]) == 4001 and len(got2["deliv"][:got2["deliv_count"][0]]) == 4


@pytest.mark.parametrize("n,nconns,batches", [(1, 1, 1), (3000, 1, 2), (20000, 7, 2), (60000, 1000, 3),
                                              (200000, 20000, 2), (100000, 300, 1), (50000, 3, 1),
                                              (262144, 64, 1)])
def test_streams_through_rx(tcp, n, nconns, batches):
    """Frames -> dk_rx (verdicts, flow ids, seq/ack) -> dk_tcp on the GPU, against the oracle chain on the same
    frames, batch after batch with the connection table carried."""
    import torch

    flows, tr, table = synth.tcp_streams(n * batches, nconns, buffer_size=1 << 22, seed=1000 + n + nconns)
    blob, off, lens = synth.build_numpy(tr)
    synth.corrupt_numpy(blob, off, synth.corruption_plan(len(off), 0.002, tr))  # a few frames never reach TCP (holes)
    eng = RxEngine(Config(synth.BOB_IPV4), device=0)
    eng.set_sockets(flows)
    peer = OraclePeer(synth.ipv4(synth.BOB_IPV4))
    peer.set_flows(flows)
    exp_t, dev_conns = table.copy(), tcp.conns_to_device(table)
    hist = np.zeros(len(N.TCP_ACTIONS), np.int64)
    for b in range(batches):
        sl = slice(b * n, (b + 1) * n)
        boff, blens = off[sl], lens[sl]
        batch = FrameBatch.from_numpy(blob, boff, blens, device=0)
        r = eng.results(n, tcp_fields=True)
        eng.receive_batch(batch, r)
        out = TcpOut(n, len(table))
        tcp.process(r, dev_conns, out)
        torch.cuda.synchronize()
        got = out.to_numpy()
        exp_rx = peer.process(blob, boff, blens)
        exp = O.tcp_process(exp_t, exp_rx)
        got_t = tcp.conns_to_host(dev_conns)
        assert_same(got_t, got, exp_t, exp, f"batch {b}")
        hist += np.bincount(got["action"], minlength=len(N.TCP_ACTIONS))
        # the application reads everything delivered (Receiver::pop moves reader_next, ctrlblk.rs:113-129): window reopens
        exp_t["reader_next"] = exp_t["receive_next"]
        got_t["reader_next"] = got_t["receive_next"]
        dev_conns = tcp.conns_to_device(got_t)
    if n >= 20000:
        for a in ("DELIVERED", "STORED", "DUPLICATE", "OUT_OF_WINDOW", "SYN", "NO_ACK", "ACK_UNSENT", "SKIP"):
            assert hist[N.A[a]] > 0, (a, hist)
    eng.close()


def test_one_stream_gigabyte_window(tcp):
    """bench.py's tcp_rx_1conn shape: one in-order stream of 2^20 segments through a 1 GiB receive window (the largest
    TCP window scaling allows): ~70 % delivered in order, the rest past the window end; bit-exact vs the oracle."""
    n = 1 << 20
    _, tr, table = synth.tcp_streams(n, 1, 1500, buffer_size=1 << 30, reorder=0.0)
    rx = {"meta": (6 << 8 | tr.flags.astype(np.uint32) << 16 | 0x50 << 24).astype(np.uint32),
          "flow_id": tr.flow.astype(np.uint32), "tcp_seq": tr.seq, "tcp_ack": tr.ack,
          "payload": (54 | (tr.ip_len.astype(np.uint32) - 40) << 16).astype(np.uint32)}
    exp_t = table.copy()
    exp = O.tcp_process(exp_t, rx)
    got_t, got = gpu_process(tcp, table.copy(), rx_device(rx))
    assert_same(got_t, got, exp_t, exp, "1 conn, 1 GiB window")
    assert np.mean(got["action"] == N.A["DELIVERED"]) > 0.5


FUZZ = [  # (seed, segments, connections, reorder, dup, oow, rare, fin, rst, buffer)
    (1, 40000, 1, 0.0, 0.05, 0.01, 0.01, 1.0, 0.0, 1 << 30),   # one stream, many retransmissions and stray copies
    (2, 40000, 1, 2.0, 0.02, 0.005, 0.005, 1.0, 0.0, 1 << 26),  # one reordered stream: stores and drains in runs
    (7, 20000, 1, 0.0, 0.02, 0.005, 0.01, 1.0, 0.0, 1 << 16),   # a small window: full after ~45 segments
    (3, 60000, 3, 1.0, 0.03, 0.0, 0.01, 0.0, 1.0, 1 << 26),     # RSTs land mid-stream
    (4, 60000, 5, 0.5, 0.0, 0.0, 0.02, 1.0, 0.0, 1 << 22),      # rare SYN / no-ACK / unsent-ACK copies only
    (5, 80000, 40, 4.0, 0.02, 0.01, 0.002, 0.5, 0.2, 1 << 20),  # heavy reordering: the store fills and drains
    (6, 30000, 2, 0.0, 0.2, 0.0, 0.05, 1.0, 0.0, 1 << 24),      # a retransmission storm
]


@pytest.mark.parametrize("case", FUZZ, ids=[f"seed{c[0]}" for c in FUZZ])
def test_walks_fuzzed_streams(tcp, case):
    """Streams whose segments keep the state machine busy inside long runs (the relay walk's threshold check, its
    epochs and its fallback; the wave walk's parallel check): retransmission storms, stray copies with SYN / without
    ACK / with an unsent ACK, RSTs and FINs mid-batch, reordering that fills the out-of-order store, windows that
    fill; every walk bit-exact vs the oracle on the actions, views, deliveries and the connection table."""
    seed, n, nconns, reorder, dup, oow, rare, fin, rst, buf = case
    _, tr, table = synth.tcp_streams(n, nconns, 1500 if seed % 2 else None, reorder=reorder, dup=dup, oow=oow,
                                     rare=rare, fin=fin, rst=rst, buffer_size=buf, seed=500 + seed)
    rx = {"meta": (6 << 8 | tr.flags.astype(np.uint32) << 16 | 0x50 << 24).astype(np.uint32),
          "flow_id": tr.flow.astype(np.uint32), "tcp_seq": tr.seq, "tcp_ack": tr.ack,
          "payload": (54 | (tr.ip_len.astype(np.uint32) - 40) << 16).astype(np.uint32)}
    exp_t = table.copy()
    exp = O.tcp_process(exp_t, rx)
    got_t, got = gpu_process(tcp, table.copy(), rx_device(rx))
    assert_same(got_t, got, exp_t, exp, f"fuzz seed {seed}")


def test_rejects_missing_tcp_fields(tcp):
    import ctypes

    import torch

    r = RxResults(8, 1, device=torch.device("cuda", 0), tcp_fields=False, counts=False)
    conns = tcp.conns_to_device(S.conns(1))
    out = TcpOut(8, 1)
    with pytest.raises(Fail) as e:
        tcp.process(r, conns, out)
    assert e.value.errno == 22
    h = ctypes.c_void_p()
    assert tcp.lib.dk_tcp_ctx_create(-1, ctypes.byref(h)) == 22


def test_rejects_misaligned_conns(tcp):
    """The connection table must be 16-byte aligned (dk_tcp_key_kernel reads a connection's head with one 16-byte
    load): a table 4 bytes off is refused with EINVAL before any launch."""
    import ctypes

    import torch

    rx = S.batch([(0, 1, 1, S.ACK, 10)])
    r = rx_device(rx)
    buf = torch.zeros(2 * N.CONN_DTYPE.itemsize + 16, dtype=torch.uint8, device="cuda")
    out = TcpOut(1, 1)
    rs, o = r.c_struct(), out.c_struct()
    for shift in (4, 8, 12):
        rc = tcp.lib.dk_tcp_rx_process(tcp._ctx, ctypes.byref(rs), 1, ctypes.c_void_p(buf.data_ptr() + shift), 1,
                                       ctypes.byref(o), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 22, (shift, rc)
    torch.cuda.synchronize()


@pytest.mark.parametrize("nconns,reorder", [(64, 3.0), (64, 0.0), (15, 3.0), (14, 3.0), (255, 3.0), (8, 3.0)])
def test_walk_follows_stream_shape(nconns, reorder):
    """The engine's own rule (no forced walk) at the scan walk's envelope (1,024 segments per connection): the first
    call runs the scan walk; later calls run the wave walk when the last finished call stored >= 1 segment in 1,024
    out of order (in the fix kernel's sample: the call's first 16,384 segments) and the table has >= 16 connections (the
    rule's two boundaries: 16 vs 15 rows — the listener's row counts — and the stored fraction, which the oracle's STORED
    count over the same sample decides here), the scan walk otherwise (256 rows:
    the scan walk's upper bound). Every call bit-exact vs the oracle, whichever walk ran."""
    import torch

    n = 1024 * len(synth.make_flows(nconns, seed=77 + nconns))  # the table has a row per flow (the listener's too)
    _, tr, table = synth.tcp_streams(n, nconns, 1500, buffer_size=1 << 24, reorder=reorder, seed=77 + nconns)
    assert n == 1024 * len(table)
    rx = {"meta": (6 << 8 | tr.flags.astype(np.uint32) << 16 | 0x50 << 24).astype(np.uint32),
          "flow_id": tr.flow.astype(np.uint32), "tcp_seq": tr.seq, "tcp_ack": tr.ack,
          "payload": (54 | (tr.ip_len.astype(np.uint32) - 40) << 16).astype(np.uint32)}
    exp_t = table.copy()
    exp = O.tcp_process(exp_t, rx)
    sample = min(n, 64 * 256)  # the fix kernel samples its first 64 blocks (tcp_kernels.hip kShapeBlocks)
    stored = int((exp["action"][:sample] == N.A["STORED"]).sum())
    want = "wave" if stored * 1024 >= sample and len(table) >= 16 else "scan"
    r = rx_device(rx)
    tcp = TcpReceiver(0)
    walks = []
    for call in range(3):
        got_t, got = gpu_process(tcp, table.copy(), r)
        torch.cuda.synchronize()
        walks.append(tcp.last_walk)
        assert_same(got_t, got, exp_t, exp, f"{nconns} conns reorder {reorder} call {call} ({walks[-1]} walk)")
    tcp.close()
    assert walks == ["scan", want, want], (walks, stored, sample)
    if (nconns, reorder) == (64, 3.0):
        assert want == "wave"
    if reorder == 0.0:
        assert stored == 0 and want == "scan"


@pytest.mark.parametrize("nconns,reorder", [(1, 0.0), (23, 3.0), (254, 3.0), (255, 3.0), (3000, 3.0)])
def test_counting_sort_matches_radix(nconns, reorder):
    """Up to 255 table rows (tcp_kernels.hip kSortMaxRows: 2 rows + 1 <= 511 key values) the batch is ordered by one
    counting pass over the whole key (per-tile key counts, one scan that also yields the ranges, a scatter ranked by
    per-bit ballots); above, by rocPRIM's radix sort. The rule and the forced radix sort (dk_diag_tcp_set_sort) give
    bit-exact results vs the oracle at the boundary (254 / 255 flows + the listener row = 255 / 256 rows), with
    thousands of connections, and across tiles (8,192 segments per tile, a partial last one)."""
    import torch

    n = 3 * 8192 + 777
    _, tr, table = synth.tcp_streams(n, nconns, 1500, buffer_size=1 << 24, reorder=reorder, seed=91 + nconns)
    rx = {"meta": (6 << 8 | tr.flags.astype(np.uint32) << 16 | 0x50 << 24).astype(np.uint32),
          "flow_id": tr.flow.astype(np.uint32), "tcp_seq": tr.seq, "tcp_ack": tr.ack,
          "payload": (54 | (tr.ip_len.astype(np.uint32) - 40) << 16).astype(np.uint32)}
    exp_t = table.copy()
    exp = O.tcp_process(exp_t, rx)
    r = rx_device(rx)
    for radix in (False, True):
        tcp = TcpReceiver(0, radix_sort=radix)
        got_t, got = gpu_process(tcp, table.copy(), r)
        torch.cuda.synchronize()
        tcp.close()
        assert_same(got_t, got, exp_t, exp, f"{len(table)} rows reorder {reorder} radix {radix}")
