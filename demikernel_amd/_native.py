"""ctypes binding of include/dk_rx.h (libdk_rx.so, built in-tree for gfx950 by __graft_entry__.build()).

No fallback: if the HIP library is missing, importing the engine raises. The structures below mirror the C header
field for field; tests/test_abi.py checks their sizes and that every function the header declares is exported.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_int, c_int32, c_uint8, c_uint16, c_uint32, c_uint64, c_void_p

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libdk_rx.so")  # tuning builds (tools/variants.sh) are passed as lib_path explicitly

DK_FLOW_NONE = 0xFFFFFFFF
DK_TX_NOT_WRITTEN = 0xFFFF  # dk_tx_checksum_fields: a checksum half the in-place fill leaves untouched
DK_RX_BATCH_ALIGNED16 = 1  # dk_rx_batch.flags
DK_RX_BATCH_DEFER_COUNTS = 2
DK_RX_MAX_DEFERRED_FLOWS = 32768  # flow_counts defer only for tables up to this size (dk_rx.h)
DK_FLOW_TCP_ACTIVE, DK_FLOW_TCP_PASSIVE, DK_FLOW_UDP = 1, 2, 3

# enum dk_verdict (include/dk_rx.h), SURVEY.md Appendix A.
VERDICTS = [
    "OK_TCP", "OK_UDP", "ARP", "ICMP", "IPV6", "ETH_SHORT", "ETH_TYPE", "IP_SHORT", "IP_VERSION", "IP_IHL_SMALL",
    "IP_HDR_TRUNC", "IP_TOTLEN_SMALL", "IP_TOTLEN_BIG", "IP_EVIL", "IP_MF", "IP_FRAGOFF", "IP_TTL", "IP_PROTO",
    "IP_CSUM_FFFF", "IP_CSUM", "IP_DST", "IP_SRC", "TCP_SHORT", "TCP_DOFF_TRUNC", "TCP_DOFF_SMALL", "TCP_CSUM",
    "TCP_OPT", "TCP_OPT_EIO", "TCP_NOSOCK", "UDP_SHORT", "UDP_LEN", "UDP_CSUM", "UDP_NOSOCK", "BAD_DESC",
    "ARP_SHORT", "ARP_UNSUP", "ICMP_SHORT", "ICMP_CSUM", "ICMP_TYPE",
]
V = {name: i for i, name in enumerate(VERDICTS)}
DK_V_COUNT = len(VERDICTS)

# numpy mirror of struct dk_flow (16 bytes).
FLOW_DTYPE = np.dtype([("kind", "<u4"), ("local_ip", "<u4"), ("remote_ip", "<u4"),
                       ("local_port", "<u2"), ("remote_port", "<u2")])
assert FLOW_DTYPE.itemsize == 16


class DkRxCfg(ctypes.Structure):
    _fields_ = [("local_ipv4", c_uint32), ("tcp_rx_checksum_offload", c_uint8),
                ("udp_rx_checksum_offload", c_uint8), ("reserved", c_uint16), ("device", c_int32)]


class DkFlow(ctypes.Structure):
    _fields_ = [("kind", c_uint32), ("local_ip", c_uint32), ("remote_ip", c_uint32),
                ("local_port", c_uint16), ("remote_port", c_uint16)]


class DkRxBatch(ctypes.Structure):
    _fields_ = [("frames", c_void_p), ("frames_bytes", c_uint64), ("off", c_void_p), ("len", c_void_p),
                ("n", c_uint32), ("flags", c_uint32)]


RESULT_FIELDS = ["meta", "src_ip", "dst_ip", "ports", "payload", "flow_id", "tcp_seq", "tcp_ack", "tcp_win",
                 "flow_counts", "verdict_counts", "tcp_opts"]

# numpy mirror of struct dk_tcp_opts (96 bytes): the parsed [TcpOptions2; 5] list of one segment.
TCP_OPT_DTYPE = np.dtype([("kind", "u1"), ("u8", "u1"), ("u16", "<u2"), ("v0", "<u4"), ("v1", "<u4")])
TCP_OPTS_DTYPE = np.dtype([("num", "<u4"), ("opt", TCP_OPT_DTYPE, (5,)), ("sack", "<u4", (4, 2))])
assert TCP_OPT_DTYPE.itemsize == 12 and TCP_OPTS_DTYPE.itemsize == 96
DK_TCPOPT_MSS, DK_TCPOPT_WS, DK_TCPOPT_SACK_OK, DK_TCPOPT_SACK, DK_TCPOPT_TS = 2, 3, 4, 5, 8


class DkTcpOpt(ctypes.Structure):
    _fields_ = [("kind", c_uint8), ("u8", c_uint8), ("u16", c_uint16), ("v0", c_uint32), ("v1", c_uint32)]


class DkTcpOpts(ctypes.Structure):
    _fields_ = [("num", c_uint32), ("opt", DkTcpOpt * 5), ("sack", (c_uint32 * 2) * 4)]


class DkRxResults(ctypes.Structure):
    _fields_ = [(name, c_void_p) for name in RESULT_FIELDS]


# (name, restype, argtypes) of every function include/dk_rx.h declares.
FUNCTIONS = [
    ("dk_rx_ctx_create", c_int, [POINTER(DkRxCfg), POINTER(c_void_p)]),
    ("dk_rx_ctx_destroy", None, [c_void_p]),
    ("dk_rx_flow_table_set", c_int, [c_void_p, c_void_p, c_uint32]),
    ("dk_rx_flow_table_size", c_uint32, [c_void_p]),
    ("dk_rx_process", c_int, [c_void_p, POINTER(DkRxBatch), POINTER(DkRxResults), c_void_p]),
    ("dk_rx_process_host", c_int, [c_void_p, POINTER(DkRxBatch), POINTER(DkRxResults), c_uint32]),
    ("dk_rx_stream_forget", c_int, [c_void_p, c_void_p]),
    ("dk_rx_counts_flush", c_int, [c_void_p, c_void_p]),
    ("dk_rx_flow_counts_allreduce", c_int, [c_void_p, POINTER(DkRxResults), c_void_p, c_void_p]),
    ("dk_rx_flow_counts_allreduce_to", c_int, [c_void_p, POINTER(DkRxResults), c_void_p, c_void_p, c_void_p,
                                               c_void_p]),
    ("dk_tx_checksum", c_int, [c_void_p, c_uint64, c_void_p, c_void_p, c_uint32, c_void_p]),
    ("dk_tx_checksum_fields", c_int, [c_void_p, c_uint64, c_void_p, c_void_p, c_uint32, c_void_p, c_void_p]),
    ("dk_rx_verdict_name", c_char_p, [c_int]),
    ("dk_rx_verdict_errno", c_int, [c_int]),
    ("dk_rx_abi_version", c_uint32, []),
    ("dk_rx_build_id", c_char_p, []),
    ("dk_rx_device_count", c_int, []),
]

# include/dk_ring.h (TPACKET_V3 ring ingest)
RING_FUNCTIONS = [
    ("dk_ring_register", c_int, [c_void_p, c_uint64]),
    ("dk_ring_unregister", c_int, [c_void_p]),
    ("dk_ring_scan_tpacket3", c_int, [c_void_p, c_uint64, c_uint32, c_uint32, c_uint32, c_void_p, c_void_p, c_uint32,
                                      POINTER(c_uint32), POINTER(c_uint32)]),
    ("dk_ring_release_tpacket3", c_int, [c_void_p, c_uint64, c_uint32, c_uint32, c_uint32]),
    ("dk_rx_process_tpacket3", c_int, [c_void_p, c_void_p, c_uint64, c_uint32, c_uint32, c_uint32,
                                       POINTER(DkRxResults), c_uint32, POINTER(c_uint32), POINTER(c_uint32)]),
]

# include/dk_tcp.h (established-state TCP receive processing)
DK_TCP_OOO_MAX = 16
DK_TCP_DELIV_EXTRA = 18
DK_TCP_REF_EOF = 0xFFFFFFFF
DK_TCP_NONE, DK_TCP_ESTABLISHED, DK_TCP_CLOSED = 0, 1, 2
TCP_ACTIONS = ["SKIP", "DELIVERED", "STORED", "STORE_DUP", "NO_DATA", "FIN", "DUPLICATE", "OUT_OF_WINDOW", "RST",
               "SYN", "NO_ACK", "ACK_UNSENT", "UNPROCESSED"]
A = {name: i for i, name in enumerate(TCP_ACTIONS)}
VIEW_DTYPE = np.dtype([("ref", "<u4"), ("off", "<u4"), ("len", "<u4")])
CONN_DTYPE = np.dtype([("state", "<u4"), ("receive_next", "<u4"), ("reader_next", "<u4"), ("buffer_size", "<u4"),
                       ("send_next", "<u4"), ("fin_pending", "<u4"), ("fin_seq", "<u4"), ("ooo_count", "<u4"),
                       ("ooo_start", "<u4", (DK_TCP_OOO_MAX,)), ("ooo", VIEW_DTYPE, (DK_TCP_OOO_MAX,))])
assert CONN_DTYPE.itemsize == 288


class DkTcpView(ctypes.Structure):
    _fields_ = [("ref", c_uint32), ("off", c_uint32), ("len", c_uint32)]


class DkTcpConn(ctypes.Structure):
    _fields_ = [("state", c_uint32), ("receive_next", c_uint32), ("reader_next", c_uint32),
                ("buffer_size", c_uint32), ("send_next", c_uint32), ("fin_pending", c_uint32), ("fin_seq", c_uint32),
                ("ooo_count", c_uint32), ("ooo_start", c_uint32 * DK_TCP_OOO_MAX),
                ("ooo", DkTcpView * DK_TCP_OOO_MAX)]


class DkTcpOut(ctypes.Structure):
    _fields_ = [("action", c_void_p), ("view", c_void_p), ("deliv", c_void_p), ("deliv_start", c_void_p),
                ("deliv_count", c_void_p)]


TCP_FUNCTIONS = [
    ("dk_tcp_ctx_create", c_int, [c_int32, POINTER(c_void_p)]),
    ("dk_tcp_ctx_destroy", None, [c_void_p]),
    ("dk_tcp_rx_process", c_int, [c_void_p, POINTER(DkRxResults), c_uint32, c_void_p, c_uint32, POINTER(DkTcpOut),
                                  c_void_p]),
]

# include/dk_diag.h (diagnostics, not the receive ABI)
# include/dk_demi.h: delivered frames as demi_sgarray_t (host-side, no GPU work)
class DemiSgaseg(ctypes.Structure):
    _pack_ = 1
    _fields_ = [("sgaseg_buf", c_void_p), ("sgaseg_len", c_uint32)]


class SockaddrIn(ctypes.Structure):
    _fields_ = [("sin_family", ctypes.c_uint16), ("sin_port", ctypes.c_uint16), ("sin_addr", c_uint32),
                ("sin_zero", ctypes.c_uint8 * 8)]


class DemiSgarray(ctypes.Structure):
    _pack_ = 1
    _fields_ = [("sga_buf", c_void_p), ("sga_numsegs", c_uint32), ("sga_segs", DemiSgaseg * 1),
                ("sga_addr", SockaddrIn)]


DEMI_FUNCTIONS = [
    ("dk_rx_into_sgarrays", c_int, [c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    POINTER(DemiSgarray), c_void_p, c_uint32, POINTER(c_uint32)]),
    ("dk_tcp_into_sgarrays", c_int, [c_void_p, c_void_p, c_uint32, c_void_p, c_uint32, c_void_p, POINTER(DemiSgarray),
                                     c_uint32, POINTER(c_uint32)]),
]

# include/dk_comm.h: RCCL communicator bootstrap (the receive path's one collective is dk_rx_flow_counts_allreduce)
DK_COMM_ID_BYTES = 128
COMM_FUNCTIONS = [
    ("dk_comm_unique_id", c_int, [c_void_p]),
    ("dk_comm_init_rank", c_int, [POINTER(c_void_p), c_int32, c_void_p, c_int32, c_int32]),
    ("dk_comm_init_all", c_int, [c_void_p, c_int32, c_void_p]),
    ("dk_comm_count", c_int, [c_void_p, POINTER(c_int32)]),
    ("dk_comm_destroy", c_int, [c_void_p]),
]

DIAG_FUNCTIONS = [
    ("dk_diag_read_probe", c_int, [c_void_p, c_uint64, c_void_p, c_uint32, c_int, c_void_p]),
    ("dk_diag_rw_probe", c_int, [c_void_p, c_uint64, c_void_p, c_uint32, c_void_p, c_uint32, c_void_p]),
    ("dk_diag_patch_probe", c_int, [c_void_p, c_uint64, c_uint32, c_uint32, c_uint32, c_void_p, c_uint32, c_void_p]),
    ("dk_diag_path_stats_enable", c_int, [c_void_p, c_int]),
    ("dk_diag_path_stats_read", c_int, [c_void_p, c_void_p]),
    ("dk_diag_rx_set_tuning", c_int, [c_void_p, c_void_p, c_uint32]),
    ("dk_diag_tx_set_tuning", c_int, [c_int32, c_int32, c_int32]),
    ("dk_diag_tcp_set_walk", c_int, [c_void_p, c_int32, c_int32]),
    ("dk_diag_tcp_last_walk", c_int, [c_void_p]),
    ("dk_diag_tcp_set_sort", c_int, [c_void_p, c_int32]),
]
DK_DIAG_RX_KNOBS = ["stage", "split", "small", "sched", "grid", "grid_per_cu", "debug", "lds_table", "tail", "udp_table",
                    "host_zc"]
DK_TCP_WALKS = {"lane": 0, "wave": 1, "relay": 2, "scan": 3}

ALL_FUNCTIONS = FUNCTIONS + RING_FUNCTIONS + TCP_FUNCTIONS + DIAG_FUNCTIONS + DEMI_FUNCTIONS + COMM_FUNCTIONS

_lib = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libdk_rx.so (fails loudly: there is no CPU fallback for the product path)."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"{path} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    # One HIP runtime per process: torch ships its own libamdhip64 (SONAME libamdhip64.so.7, NEEDED as
    # "libamdhip64.so"). Loaded first, it also satisfies our NEEDED libamdhip64.so.7; loaded after us, it would be a
    # second runtime and device pointers/streams would not be shared.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    for name, restype, argtypes in ALL_FUNCTIONS:
        fn = getattr(lib, name, None)
        if fn is None:
            if path != LIB_PATH:
                continue  # tuning builds (older sources) may predate a function
            raise ImportError(f"{path}: missing {name}")
        fn.restype = restype
        fn.argtypes = argtypes
    if path == LIB_PATH:
        _lib = lib
    return lib
