"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of oracle/libdk_oracle.so (the CPU restatement of the reference).

Used as the parity checker in tests/ and smoke(), and timed as the CPU baseline ("port") in bench.py.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_int, c_size_t, c_uint8, c_uint16, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libdk_oracle.so")

DK_V_COUNT = 39  # enum dk_verdict in include/dk_rx.h (tests/test_oracle.py checks it)
# struct dk_tcp_opts (include/dk_rx.h): the parsed [TcpOptions2; 5] list of one segment.
TCP_OPT_DTYPE = np.dtype([("kind", "u1"), ("u8", "u1"), ("u16", "<u2"), ("v0", "<u4"), ("v1", "<u4")])
TCP_OPTS_DTYPE = np.dtype([("num", "<u4"), ("opt", TCP_OPT_DTYPE, (5,)), ("sack", "<u4", (4, 2))])
assert TCP_OPT_DTYPE.itemsize == 12 and TCP_OPTS_DTYPE.itemsize == 96
FLOW_DTYPE = np.dtype([("kind", "<u4"), ("local_ip", "<u4"), ("remote_ip", "<u4"),
                       ("local_port", "<u2"), ("remote_port", "<u2")])

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        vp = c_void_p
        L.dko_peer_new.restype = vp
        L.dko_peer_new.argtypes = [c_uint32, c_int, c_int]
        L.dko_peer_free.argtypes = [vp]
        L.dko_peer_set_flows.restype = c_int
        L.dko_peer_set_flows.argtypes = [vp, vp, c_uint32]
        L.dko_process.argtypes = [vp, vp, c_uint64, vp, vp, c_uint32] + [vp] * 12
        L.dko_process_mt.restype = c_int
        L.dko_process_mt.argtypes = [vp, vp, c_uint64, vp, vp, c_uint32] + [vp] * 6 + [c_int]
        L.dko_process_par.restype = c_int
        L.dko_process_par.argtypes = [vp, vp, c_uint64, vp, vp, c_uint32] + [vp] * 12 + [c_int]
        L.dko_ipv4_parse.restype = c_int
        L.dko_ipv4_parse.argtypes = [vp, c_size_t, POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint8),
                                     POINTER(c_uint32), POINTER(c_uint32)]
        L.dko_udp_parse.restype = c_int
        L.dko_udp_parse.argtypes = [c_uint32, c_uint32, vp, c_size_t, c_int, POINTER(c_uint16), POINTER(c_uint16),
                                    POINTER(c_uint32)]
        L.dko_tcp_parse.restype = c_int
        L.dko_tcp_parse.argtypes = [c_uint32, c_uint32, vp, c_size_t, c_int, POINTER(c_int), POINTER(c_uint32)]
        L.dko_ipv4_checksum.restype = c_uint16
        L.dko_ipv4_checksum.argtypes = [vp, c_size_t]
        L.dko_tcp_checksum.restype = c_uint16
        L.dko_tcp_checksum.argtypes = [c_uint32, c_uint32, vp, c_size_t, vp, c_size_t]
        L.dko_udp_checksum.restype = c_uint16
        L.dko_udp_checksum.argtypes = [c_uint32, c_uint32, vp, vp, c_size_t]
        L.dko_generic_checksum.restype = c_uint16
        L.dko_generic_checksum.argtypes = [vp, c_size_t, c_int, c_uint32]
        L.dko_tx_fill_checksums.restype = c_int
        L.dko_tx_fill_checksums.argtypes = [vp, c_size_t]
        L.dko_tx_checksum_fields.restype = ctypes.c_uint32
        L.dko_tx_checksum_fields.argtypes = [vp, c_size_t]
        L.dko_tcp_process.restype = c_int
        L.dko_tcp_process.argtypes = [vp, c_uint32, c_uint32] + [vp] * 10
        _lib = L
    return _lib


def _buf(b: bytes):
    a = np.frombuffer(bytes(b) if b else b"\0", np.uint8)
    return a, a.ctypes.data


class OraclePeer:
    """The restated receive chain with its socket tables (dko_peer)."""

    def __init__(self, local_ipv4: int, tcp_offload: bool = False, udp_offload: bool = False):
        self._L = lib()
        self._p = self._L.dko_peer_new(local_ipv4, int(tcp_offload), int(udp_offload))
        self.nflows = 0

    def __del__(self):
        try:
            self._L.dko_peer_free(self._p)
        except Exception:
            pass

    def set_flows(self, flows: np.ndarray) -> None:
        flows = np.ascontiguousarray(flows, dtype=FLOW_DTYPE)
        rc = self._L.dko_peer_set_flows(self._p, flows.ctypes.data, len(flows))
        if rc:
            raise ValueError(f"dko_peer_set_flows: {rc}")
        self.nflows = len(flows)

    def process(self, blob: np.ndarray, off: np.ndarray, lens: np.ndarray, frames_bytes: int | None = None) -> dict:
        n = len(off)
        blob = np.ascontiguousarray(blob, np.uint8)
        off = np.ascontiguousarray(off, np.uint32)
        lens = np.ascontiguousarray(lens, np.uint16)
        out = {k: np.zeros(n, np.uint32) for k in
               ("meta", "src_ip", "dst_ip", "ports", "payload", "flow_id", "tcp_seq", "tcp_ack", "tcp_win")}
        out["flow_counts"] = np.zeros(max(self.nflows, 1), np.uint64)
        out["verdict_counts"] = np.zeros(DK_V_COUNT, np.uint64)
        out["tcp_opts"] = np.zeros(max(n, 1), TCP_OPTS_DTYPE)[:n]  # written for option-bearing TCP segments only
        fb = blob.nbytes if frames_bytes is None else frames_bytes
        self._L.dko_process(self._p, blob.ctypes.data if blob.size else None, fb, off.ctypes.data,
                            lens.ctypes.data, n,
                            *[out[k].ctypes.data for k in ("meta", "src_ip", "dst_ip", "ports", "payload", "flow_id",
                                                           "tcp_seq", "tcp_ack", "tcp_win", "flow_counts",
                                                           "verdict_counts", "tcp_opts")])
        return out

    def process_par(self, blob: np.ndarray, off: np.ndarray, lens: np.ndarray, threads: int = 0,
                    frames_bytes: int | None = None) -> dict:
        """`process` over OpenMP threads (dko_process_par): the same outputs, counters included, for whole-batch parity
        at full size. threads <= 0: the CPUs this process may use."""
        import os

        if threads <= 0:
            threads = max(1, min(len(os.sched_getaffinity(0)), 16))
        n = len(off)
        blob = np.ascontiguousarray(blob, np.uint8)
        off = np.ascontiguousarray(off, np.uint32)
        lens = np.ascontiguousarray(lens, np.uint16)
        out = {k: np.zeros(n, np.uint32) for k in
               ("meta", "src_ip", "dst_ip", "ports", "payload", "flow_id", "tcp_seq", "tcp_ack", "tcp_win")}
        out["flow_counts"] = np.zeros(max(self.nflows, 1), np.uint64)
        out["verdict_counts"] = np.zeros(DK_V_COUNT, np.uint64)
        out["tcp_opts"] = np.zeros(max(n, 1), TCP_OPTS_DTYPE)[:n]
        fb = blob.nbytes if frames_bytes is None else frames_bytes
        self._L.dko_process_par(self._p, blob.ctypes.data if blob.size else None, fb, off.ctypes.data,
                                lens.ctypes.data, n,
                                *[out[k].ctypes.data for k in ("meta", "src_ip", "dst_ip", "ports", "payload", "flow_id",
                                                               "tcp_seq", "tcp_ack", "tcp_win", "flow_counts",
                                                               "verdict_counts", "tcp_opts")], threads)
        return out

    def process_mt(self, blob, off, lens, threads: int) -> tuple[dict, int]:
        n = len(off)
        out = {k: np.zeros(n, np.uint32) for k in ("meta", "src_ip", "dst_ip", "ports", "payload", "flow_id")}
        used = self._L.dko_process_mt(self._p, blob.ctypes.data, blob.nbytes, off.ctypes.data, lens.ctypes.data, n,
                                      *[out[k].ctypes.data for k in
                                        ("meta", "src_ip", "dst_ip", "ports", "payload", "flow_id")], threads)
        return out, used


def ipv4_parse(dgram: bytes):
    """Ipv4Header::parse_and_strip on a bare datagram: (verdict or -1, (src, dst, proto, payload_off, payload_len))."""
    a, p = _buf(dgram)
    s, d, po, pl = c_uint32(), c_uint32(), c_uint32(), c_uint32()
    pr = c_uint8()
    v = lib().dko_ipv4_parse(p, len(dgram), ctypes.byref(s), ctypes.byref(d), ctypes.byref(pr), ctypes.byref(po),
                             ctypes.byref(pl))
    return v, (s.value, d.value, pr.value, po.value, pl.value)


def udp_parse(src_ip: int, dst_ip: int, seg: bytes, offload: bool):
    a, p = _buf(seg)
    sp, dp, pl = c_uint16(), c_uint16(), c_uint32()
    v = lib().dko_udp_parse(src_ip, dst_ip, p, len(seg), int(offload), ctypes.byref(sp), ctypes.byref(dp),
                            ctypes.byref(pl))
    return v, (sp.value, dp.value, pl.value)


def tcp_parse(local_ip: int, remote_ip: int, seg: bytes, offload: bool):
    a, p = _buf(seg)
    no, pl = c_int(), c_uint32()
    v = lib().dko_tcp_parse(local_ip, remote_ip, p, len(seg), int(offload), ctypes.byref(no), ctypes.byref(pl))
    return v, (no.value, pl.value)


def ipv4_checksum(hdr: bytes) -> int:
    a, p = _buf(hdr)
    return lib().dko_ipv4_checksum(p, len(hdr))


def tcp_checksum(src: int, dst: int, hdr: bytes, data: bytes) -> int:
    a, p = _buf(hdr)
    b, q = _buf(data)
    return lib().dko_tcp_checksum(src, dst, p, len(hdr), q, len(data))


def udp_checksum(src: int, dst: int, hdr8: bytes, data: bytes) -> int:
    a, p = _buf(hdr8)
    b, q = _buf(data)
    return lib().dko_udp_checksum(src, dst, p, q, len(data))


def generic_checksum(buf: bytes, start: int | None = None) -> int:
    a, p = _buf(buf)
    return lib().dko_generic_checksum(p, len(buf), 0 if start is None else 1, 0 if start is None else start)


def tx_fill_checksums(frame: bytearray) -> int:
    a = np.frombuffer(frame, np.uint8)
    return lib().dko_tx_fill_checksums(a.ctypes.data, len(frame))


def tx_checksum_fields(frame: bytes) -> int:
    """dk_tx_checksum_fields' u32 for one frame: ipv4 | l4 << 16 (0xFFFF: not filled)."""
    a = np.frombuffer(bytes(frame), np.uint8)
    return lib().dko_tx_checksum_fields(a.ctypes.data, len(frame))


# include/dk_tcp.h mirrors (tests/test_tcp_oracle.py checks them against demikernel_amd._native)
TCP_OOO_MAX, TCP_DELIV_EXTRA = 16, 18
TCP_VIEW_DTYPE = np.dtype([("ref", "<u4"), ("off", "<u4"), ("len", "<u4")])
TCP_CONN_DTYPE = np.dtype([("state", "<u4"), ("receive_next", "<u4"), ("reader_next", "<u4"), ("buffer_size", "<u4"),
                           ("send_next", "<u4"), ("fin_pending", "<u4"), ("fin_seq", "<u4"), ("ooo_count", "<u4"),
                           ("ooo_start", "<u4", (TCP_OOO_MAX,)), ("ooo", TCP_VIEW_DTYPE, (TCP_OOO_MAX,))])


def tcp_process(conns: np.ndarray, rx: dict) -> dict:
    """dko_tcp_process: the batch's TCP segments through `conns` (TCP_CONN_DTYPE, updated in place). rx holds the
    dk_rx results meta, flow_id, tcp_seq, tcp_ack, payload (u32[n]). Returns action, view, deliv, deliv_start,
    deliv_count in the dk_tcp_rx_process layout, deliv trimmed to its used span."""
    assert conns.dtype == TCP_CONN_DTYPE and conns.flags.c_contiguous
    f = {k: np.ascontiguousarray(rx[k], np.uint32) for k in ("meta", "flow_id", "tcp_seq", "tcp_ack", "payload")}
    n, nc = len(f["meta"]), len(conns)
    out = {"action": np.zeros(n, np.uint8), "view": np.zeros(n, TCP_VIEW_DTYPE),
           "deliv": np.zeros(n + TCP_DELIV_EXTRA * nc, TCP_VIEW_DTYPE),
           "deliv_start": np.zeros(nc, np.uint32), "deliv_count": np.zeros(nc, np.uint32)}
    p = lambda a: a.ctypes.data if a.size else None  # noqa: E731
    rc = lib().dko_tcp_process(p(conns), nc, n, *[p(f[k]) for k in ("meta", "flow_id", "tcp_seq", "tcp_ack", "payload")],
                               *[p(out[k]) for k in ("action", "view", "deliv", "deliv_start", "deliv_count")])
    assert rc == 0
    return out
