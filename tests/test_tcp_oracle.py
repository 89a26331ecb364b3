"""The TCP receive oracle (oracle/dk_tcp_oracle.cpp) against the reference's own scenarios.

Golden: the network_simulator scripts in /root/reference/network_simulator/input/tcp/ (packetdrill-style; the expected
ACK / window the stack sends after each received segment pins RCV.NXT and the receive window):
  close/close-remote.pkt:20            FIN at RCV.NXT=1            -> "ack 2 win 65534"
  close/close-out-of-order-fin.pkt:24  FIN seq 1001 before data    -> "ack 1 win 65535" (stored), then
                               :30     data seq 1(1000)            -> "ack 1002 win 64534" (data + stored FIN)
  pop/pop-push-blocking.pkt:23         data seq 1(1000)            -> "ack 1001"; :36 pure ACK -> no data
  push/push-retransmission-2.pkt:36,45 pure ACKs of sent data      -> accepted, no data
The remaining cases walk each branch of process_packet / store_out_of_order_segment (ctrlblk.rs:403-1024) with the
expected result worked out by hand from the reference code; each cites the lines it exercises.
"""
import numpy as np
import pytest

from demikernel_amd import _native as N
from oracle import oracle as O

A = N.A
ACK, PSH, FIN, SYN, RST = 0x10, 0x08, 0x01, 0x02, 0x04
HDR = 54  # payload offset of the frames (Ethernet + IPv4 + TCP, no options)
OK_TCP = 0


def conns(n=1, rn=1, snd=1, bufsz=65535, state=N.DK_TCP_ESTABLISHED, reader=None):
    t = np.zeros(n, O.TCP_CONN_DTYPE)
    t["state"] = state
    t["receive_next"] = rn
    t["reader_next"] = rn if reader is None else reader
    t["buffer_size"] = bufsz
    t["send_next"] = snd
    return t


def batch(segs):
    """segs: (flow, seq, ack, flags, payload_len[, verdict]) -> the dk_rx result arrays dko_tcp_process reads."""
    n = len(segs)
    rx = {k: np.zeros(n, np.uint32) for k in ("meta", "flow_id", "tcp_seq", "tcp_ack", "payload")}
    for i, s in enumerate(segs):
        flow, seq, ack, flags, ln = s[:5]
        v = s[5] if len(s) > 5 else OK_TCP
        rx["meta"][i] = v | 6 << 8 | flags << 16 | 0x50 << 24
        rx["flow_id"][i] = flow
        rx["tcp_seq"][i] = seq & 0xFFFFFFFF
        rx["tcp_ack"][i] = ack & 0xFFFFFFFF
        rx["payload"][i] = HDR | ln << 16
    return rx


def run(t, segs):
    out = O.tcp_process(t, batch(segs))
    return out


def deliv(out, c=0):
    s = int(out["deliv_start"][c])
    return [tuple(int(x) for x in v) for v in out["deliv"][s:s + int(out["deliv_count"][c])]]


def window(t, c=0):  # get_receive_window_size (ctrlblk.rs:786-789)
    return int(t["buffer_size"][c]) - ((int(t["receive_next"][c]) - int(t["reader_next"][c])) & 0xFFFFFFFF)


def acts(out):
    return [N.TCP_ACTIONS[a] for a in out["action"]]


EOF = (N.DK_TCP_REF_EOF, 0, 0)


def test_dtype_mirrors_match():
    assert O.TCP_CONN_DTYPE == N.CONN_DTYPE and O.TCP_VIEW_DTYPE == N.VIEW_DTYPE
    assert (O.TCP_OOO_MAX, O.TCP_DELIV_EXTRA) == (N.DK_TCP_OOO_MAX, N.DK_TCP_DELIV_EXTRA)


# ---- golden: network_simulator scripts --------------------------------------------------------------------------


def test_close_remote_pkt():
    t = conns(rn=1, snd=1)
    out = run(t, [(0, 1, 1, FIN | ACK, 0)])
    assert acts(out) == ["FIN"]
    assert int(t["receive_next"][0]) == 2 and window(t) == 65534  # "ack 2 win 65534"
    assert deliv(out) == [(0, HDR, 0), EOF]  # empty in-order buffer, then the EOF buffer (ctrlblk.rs:693, :1008)
    assert t["state"][0] == N.DK_TCP_CLOSED


def test_close_out_of_order_fin_pkt():
    t = conns(rn=1, snd=1001)
    out = run(t, [(0, 1001, 1001, FIN | ACK, 0)])
    assert acts(out) == ["STORED"]
    assert int(t["receive_next"][0]) == 1 and window(t) == 65535  # "ack 1 win 65535"
    assert (t["fin_pending"][0], t["fin_seq"][0], t["ooo_count"][0]) == (1, 1001, 0)
    out = run(t, [(0, 1, 1001, PSH | ACK, 1000)])
    assert acts(out) == ["FIN"]
    assert int(t["receive_next"][0]) == 1002 and window(t) == 64534  # "ack 1002 win 64534"
    assert deliv(out) == [(0, HDR, 1000), EOF]


def test_pop_push_blocking_pkt():
    t = conns(rn=1, snd=1)
    out = run(t, [(0, 1, 1, PSH | ACK, 1000)])
    assert acts(out) == ["DELIVERED"] and int(t["receive_next"][0]) == 1001  # "ack 1001"
    t["reader_next"] = 1001  # the pending read(501, ..., 1000) pops it: "win 65535"
    assert window(t) == 65535
    t["send_next"] = 1001  # write(501, ..., 1000) sent seq 1(1000)
    out = run(t, [(0, 1001, 1001, ACK, 0)])
    assert acts(out) == ["NO_DATA"] and int(t["receive_next"][0]) == 1001 and deliv(out) == []


def test_push_retransmission_2_pkt():
    t = conns(rn=1, snd=2001)
    out = run(t, [(0, 1, 1001, ACK, 0), (0, 1, 2001, ACK, 0)])
    assert acts(out) == ["NO_DATA", "NO_DATA"] and int(t["receive_next"][0]) == 1


# ---- check_segment_in_window (ctrlblk.rs:447-567) ---------------------------------------------------------------


def test_duplicate_and_partial_duplicate():
    t = conns(rn=1001)
    out = run(t, [(0, 1, 1, ACK, 1000), (0, 501, 1, ACK, 1000)])
    assert acts(out) == ["DUPLICATE", "DELIVERED"]  # :495-504, then the front trim :505-521
    assert tuple(out["view"][0]) == (0, HDR, 1000)
    assert tuple(out["view"][1]) == (1, HDR + 500, 500)
    assert int(t["receive_next"][0]) == 1501 and deliv(out) == [(1, HDR + 500, 500)]


def test_out_of_window_and_end_trim():
    t = conns(rn=1, bufsz=65535)
    out = run(t, [(0, 1 + 65535, 1, ACK, 10), (0, 65535, 1, ACK, 10)])
    assert acts(out) == ["OUT_OF_WINDOW", "STORED"]  # :525-535; the second is trimmed to 1 byte (:539-560)
    assert tuple(out["view"][1]) == (1, HDR, 1)
    assert t["ooo_count"][0] == 1 and t["ooo_start"][0][0] == 65535 and tuple(t["ooo"][0][0]) == (1, HDR, 1)


def test_end_trim_drops_fin():
    t = conns(rn=1, bufsz=100)
    out = run(t, [(0, 1, 1, FIN | ACK, 100)])
    assert acts(out) == ["DELIVERED"]  # the FIN lies past the window: trimmed off (:549-556)
    assert int(t["receive_next"][0]) == 101 and t["state"][0] == N.DK_TCP_ESTABLISHED


def test_zero_window_keeps_nothing():
    t = conns(rn=1001, reader=1, bufsz=1000)  # window 0
    out = run(t, [(0, 1001, 1, ACK, 10)])
    assert acts(out) == ["NO_DATA"] and tuple(out["view"][0]) == (0, HDR, 0)


def test_syn_consumes_one_sequence_number():
    t = conns(rn=100)
    out = run(t, [(0, 99, 1, SYN | ACK, 100), (0, 200, 1, SYN | ACK, 0)])
    # first: SYN at RCV.NXT-1 is trimmed off with no data loss (:510-516); second: in-window SYN (:586-604)
    assert acts(out) == ["DELIVERED", "SYN"]
    assert tuple(out["view"][0]) == (0, HDR, 100) and int(t["receive_next"][0]) == 200


def test_sequence_wraparound():
    t = conns(rn=0xFFFFFF00)
    out = run(t, [(0, 0xFFFFFF00, 1, ACK, 1000), (0, 0xFFFFFF00, 1, ACK, 1000), (0, 0x2E8, 1, ACK, 8)])
    assert acts(out) == ["DELIVERED", "DUPLICATE", "DELIVERED"]
    assert int(t["receive_next"][0]) == 0x2F0


# ---- check_rst / check_syn / process_ack (ctrlblk.rs:570-650) -----------------------------------------------------


def test_rst_closes_and_later_segments_wait():
    t = conns(rn=1)
    out = run(t, [(0, 0, 1, RST | ACK, 0), (0, 1, 1, RST, 0), (0, 1, 1, ACK, 10)])
    assert acts(out) == ["DUPLICATE", "RST", "UNPROCESSED"]  # an old RST is dropped as a duplicate first
    assert t["state"][0] == N.DK_TCP_CLOSED
    out = run(t, [(0, 11, 1, ACK, 10)])
    assert acts(out) == ["UNPROCESSED"]


def test_ack_checks_with_wraparound():
    t = conns(rn=1, snd=5)
    out = run(t, [(0, 1, 0xFFFFFFF0, ACK, 0), (0, 1, 10, ACK, 0), (0, 1, 5, PSH, 10)])
    assert acts(out) == ["NO_DATA", "ACK_UNSENT", "NO_ACK"]
    assert int(t["receive_next"][0]) == 1


# ---- process_data / out-of-order store / receive_data (ctrlblk.rs:652-1001) --------------------------------------


def test_out_of_order_recovery():
    t = conns(rn=1)
    out = run(t, [(0, 1001, 1, ACK, 1000), (0, 2001, 1, ACK, 1000), (0, 1, 1, ACK, 1000)])
    assert acts(out) == ["STORED", "STORED", "DELIVERED"]
    assert deliv(out) == [(2, HDR, 1000), (0, HDR, 1000), (1, HDR, 1000)]
    assert int(t["receive_next"][0]) == 3001 and t["ooo_count"][0] == 0
    assert not t["ooo_start"][0].any() and not t["ooo"][0].view(np.uint32).any()  # entries past the count are zero


def test_store_duplicate_and_encompass():
    t = conns(rn=1)
    out = run(t, [(0, 1501, 1, ACK, 100), (0, 1521, 1, ACK, 50), (0, 1001, 1, ACK, 1000)])
    assert acts(out) == ["STORED", "STORE_DUP", "STORED"]  # :903-908, then :880-888 drops the encompassed entry
    assert t["ooo_count"][0] == 1 and t["ooo_start"][0][0] == 1001 and tuple(t["ooo"][0][0]) == (2, HDR, 1000)


def test_end_overlap_is_one_byte_short():
    """ctrlblk.rs:910-920: the overlap adjust is stored_end - new_start (one short), the entry keeps a 1-byte overlap;
    the in-order arrival then recovers only the first entry (2000 != 2001)."""
    t = conns(rn=1)
    out = run(t, [(0, 1001, 1, ACK, 1000), (0, 1501, 1, ACK, 1000), (0, 1, 1, ACK, 1000)])
    assert acts(out) == ["STORED", "STORED", "DELIVERED"]
    assert deliv(out) == [(2, HDR, 1000), (0, HDR, 1000)]
    assert int(t["receive_next"][0]) == 2001
    assert t["ooo_count"][0] == 1 and t["ooo_start"][0][0] == 2000 and tuple(t["ooo"][0][0]) == (1, HDR + 499, 501)


def test_front_overlap_goes_to_the_back():
    """ctrlblk.rs:889-899: a segment overlapping the front of a stored one is trimmed and inserted at the END."""
    t = conns(rn=1)
    out = run(t, [(0, 2001, 1, ACK, 1000), (0, 1501, 1, ACK, 1000), (0, 1, 1, ACK, 1500)])
    assert acts(out) == ["STORED", "STORED", "DELIVERED"]
    assert deliv(out) == [(2, HDR, 1500)] and int(t["receive_next"][0]) == 1501
    assert t["ooo_count"][0] == 2
    assert list(t["ooo_start"][0][:2]) == [2001, 1501] and tuple(t["ooo"][0][1]) == (1, HDR, 500)


def test_store_keeps_sixteen():
    t = conns(rn=1)
    segs = [(0, 1001 + 200 * k, 1, ACK, 100) for k in range(17)] + [(0, 1001 - 200, 1, ACK, 100)]
    out = run(t, segs)
    assert acts(out) == ["STORED"] * 18  # the 17th is inserted and popped from the back (:932-937)
    assert t["ooo_count"][0] == 16
    assert t["ooo_start"][0][0] == 801 and t["ooo_start"][0][15] == 1001 + 200 * 14


def test_out_of_order_fin_with_data():
    t = conns(rn=1)
    out = run(t, [(0, 1001, 1, FIN | ACK, 100), (0, 1, 1, ACK, 1000), (0, 1102, 1, ACK, 5)])
    assert acts(out) == ["STORED", "FIN", "UNPROCESSED"]
    assert deliv(out) == [(1, HDR, 1000), (0, HDR, 100), EOF]
    assert int(t["receive_next"][0]) == 1102 and t["state"][0] == N.DK_TCP_CLOSED


# ---- batch layout -------------------------------------------------------------------------------------------------


def test_skip_rules_and_delivery_layout():
    t = conns(4, rn=1)
    t["state"][2] = N.DK_TCP_NONE
    segs = [(0, 1, 1, ACK, 10), (1, 1, 1, ACK, 10), (2, 1, 1, ACK, 10), (1, 11, 1, ACK, 10),
            (N.DK_FLOW_NONE, 1, 1, ACK, 10), (3, 1, 1, ACK, 10, 25), (7, 1, 1, ACK, 10), (3, 1, 1, FIN | ACK, 0)]
    out = run(t, segs)
    assert acts(out) == ["DELIVERED", "DELIVERED", "SKIP", "DELIVERED", "SKIP", "SKIP", "SKIP", "FIN"]
    assert tuple(out["view"][5]) == (5, HDR, 10)  # skipped frames keep their payload view
    # deliv_start[c] = segments of connections < c + 18 c
    assert list(out["deliv_start"]) == [0, 1 + 18, 3 + 36, 3 + 54]
    assert list(out["deliv_count"]) == [1, 2, 0, 2]
    assert deliv(out, 1) == [(1, HDR, 10), (3, HDR, 10)] and deliv(out, 3) == [(7, HDR, 0), EOF]


def test_random_streams_are_consistent():
    """Self-consistency on synthetic streams: delivered bytes are contiguous from the old RCV.NXT."""
    from demikernel_amd import synth

    flows, tr, table = synth.tcp_streams(4000, 64, seed=11)
    rx = batch([(int(tr.flow[i]), int(tr.seq[i]), int(tr.ack[i]), int(tr.flags[i]), int(tr.ip_len[i]) - 40)
                for i in range(tr.n)])
    t = table.copy()
    out = O.tcp_process(t, rx)
    assert (np.bincount(out["action"], minlength=13)[[A["DELIVERED"], A["STORED"], A["DUPLICATE"]]] > 0).all()
    for c in range(64):
        total = sum(v[2] for v in deliv(out, c) if v[0] != N.DK_TCP_REF_EOF)
        eof = sum(v[0] == N.DK_TCP_REF_EOF for v in deliv(out, c))
        assert (int(table["receive_next"][c]) + total + eof) & 0xFFFFFFFF == int(t["receive_next"][c])
