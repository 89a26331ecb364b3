"""Host-side mirror of the reference's receive interface, over the C ABI (include/dk_rx.h).

The reference (Rust, src/rust/) receives frames one by one through
    PhysicalLayer::receive -> SharedLayer2Endpoint::receive -> SharedLayer3Endpoint::receive
    -> Peer::receive_batch -> TcpPeer::receive / UdpPeer::receive -> socket.receive(...)
(inetstack/protocols/layer1/mod.rs:27-33 ... layer4/tcp/peer.rs:220-255, layer4/udp/peer.rs:129-168).
`RxEngine.receive_batch` runs that whole chain for a batch on one MI355X and returns, per frame, what the chain
decides: the verdict (delivered / diverted / dropped / parse error with the reference's errno), the 4-tuple, the
payload window (the DemiBuffer after adjust/trim) and the socket (flow id). Errors follow runtime/fail.rs: a call
failure raises `Fail(errno, cause)`; per-frame failures are verdicts.

torch is used only to own device memory and to name the HIP stream; the ABI takes plain pointers.
"""
from __future__ import annotations

import ctypes
import socket
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _native as N
from ._native import DK_V_COUNT, FLOW_DTYPE, V, VERDICTS  # noqa: F401  (re-exported)


class Fail(Exception):
    """runtime/fail.rs `Fail { errno, cause }`."""

    def __init__(self, errno: int, cause: str):
        super().__init__(f"Error {errno}: {cause}")
        self.errno = errno
        self.cause = cause


def ipv4(addr: str) -> int:
    """Ipv4Addr -> u32 whose in-memory bytes are the octets (s_addr order), as the ABI takes it."""
    return int.from_bytes(socket.inet_aton(addr), "little")


def ipv4_str(a: int) -> str:
    return socket.inet_ntoa(int(a).to_bytes(4, "little"))


@dataclass
class Config:
    """The hot-path subset of the reference YAML config (demikernel/config.rs:20-48, :115, :340-346)."""

    local_ipv4_addr: str
    tcp_checksum_offload: bool = False
    udp_checksum_offload: bool = False


class SocketId:
    """Constructors for socket-table entries (runtime/network/socket/mod.rs:22-26; UDP: udp/peer.rs:38)."""

    @staticmethod
    def Active(local: tuple[str, int], remote: tuple[str, int]) -> tuple:
        return (N.DK_FLOW_TCP_ACTIVE, ipv4(local[0]), ipv4(remote[0]), local[1], remote[1])

    @staticmethod
    def Passive(local: tuple[str, int]) -> tuple:
        return (N.DK_FLOW_TCP_PASSIVE, ipv4(local[0]), 0, local[1], 0)

    @staticmethod
    def Udp(local: tuple[str, int]) -> tuple:
        return (N.DK_FLOW_UDP, ipv4(local[0]), 0, local[1], 0)


def flow_array(entries) -> np.ndarray:
    """List of SocketId tuples -> FLOW_DTYPE array (flow id = index)."""
    a = np.zeros(len(entries), dtype=FLOW_DTYPE)
    for i, (k, lip, rip, lp, rp) in enumerate(entries):
        a[i] = (k, lip, rip, lp, rp)
    return a


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise Fail(rc, what)


def _ptr(t) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr() if hasattr(t, "data_ptr") else t.ctypes.data


class FrameBatch:
    """An HBM-resident batch: packed frame blob + per-frame (u32 offset, u16 length) descriptors."""

    def __init__(self, blob, off, lens, frames_bytes: Optional[int] = None, aligned16: bool = False):
        """aligned16: the DK_RX_BATCH_ALIGNED16 hint (every frame at a 16-byte aligned address); a wrong hint only
        costs speed, never correctness."""
        import torch

        assert blob.dtype == torch.uint8 and (blob.is_cuda or blob.is_pinned()), "blob: HBM or pinned host memory"
        assert off.dtype == torch.int32 and lens.dtype == torch.int16 and off.numel() == lens.numel()
        self.blob, self.off, self.len = blob, off, lens
        self.n = off.numel()
        self.frames_bytes = blob.numel() if frames_bytes is None else frames_bytes
        self.aligned16 = aligned16

    @classmethod
    def from_numpy(cls, blob: np.ndarray, off: np.ndarray, lens: np.ndarray, device: int = 0) -> "FrameBatch":
        import torch

        dev = torch.device("cuda", device)
        b = torch.from_numpy(np.ascontiguousarray(blob, dtype=np.uint8)).to(dev)
        o = torch.from_numpy(np.ascontiguousarray(off, dtype=np.uint32).view(np.int32)).to(dev)
        ln = torch.from_numpy(np.ascontiguousarray(lens, dtype=np.uint16).view(np.int16)).to(dev)
        aligned = b.data_ptr() % 16 == 0 and bool(np.all(np.asarray(off, dtype=np.uint64) % 16 == 0))
        return cls(b, o, ln, aligned16=aligned)

    @classmethod
    def host_mapped(cls, blob_pinned, off: np.ndarray, lens: np.ndarray, device: int = 0) -> "FrameBatch":
        """Zero-copy: frames stay in page-locked host memory (a DPDK mempool registered with hipHostRegister, a
        hipHostMalloc'd NIC buffer) and the kernel reads them over PCIe through the mapped address; the descriptors
        go to HBM. `blob_pinned` is a pinned uint8 CPU tensor."""
        import torch

        dev = torch.device("cuda", device)
        o = torch.from_numpy(np.ascontiguousarray(off, dtype=np.uint32).view(np.int32)).to(dev)
        ln = torch.from_numpy(np.ascontiguousarray(lens, dtype=np.uint16).view(np.int16)).to(dev)
        aligned = blob_pinned.data_ptr() % 16 == 0 and bool(np.all(np.asarray(off, dtype=np.uint64) % 16 == 0))
        return cls(blob_pinned, o, ln, aligned16=aligned)

    def c_struct(self) -> N.DkRxBatch:
        """The ABI struct, rebuilt only when a field changed (a receive loop's per-call Python cost is what keeps a
        ~20 us kernel fed)."""
        key = (self.blob.data_ptr(), self.frames_bytes, self.off.data_ptr(), self.len.data_ptr(), self.n,
               self.aligned16)
        c = self.__dict__.get("_cs")
        if c is None or c[0] != key:
            c = (key, N.DkRxBatch(_ptr(self.blob), self.frames_bytes, _ptr(self.off), _ptr(self.len), self.n,
                                  N.DK_RX_BATCH_ALIGNED16 if self.aligned16 else 0))
            self._cs = c
        b = c[1]
        return N.DkRxBatch(b.frames, b.frames_bytes, b.off, b.len, b.n, b.flags)  # a copy: callers set flags


class RxResults:
    """Device (or host) result arrays, struct-of-arrays, int32/int64 storage reinterpreted as the ABI's u32/u64."""

    ARRAYS = ["meta", "src_ip", "dst_ip", "ports", "payload", "flow_id"]
    TCP_ARRAYS = ["tcp_seq", "tcp_ack", "tcp_win"]

    def __init__(self, n: int, nflows: int, *, device=None, tcp_fields: bool = False, counts: bool = True,
                 host: bool = False, dst_ip: bool = True, tcp_opts: bool = False):
        """dst_ip=False: the 20-byte-per-frame layout (dk_rx.h ABI 3: dst_ip not written). tcp_opts: the per-frame
        dk_tcp_opts records (written for option-bearing TCP segments only; zero-initialised here)."""
        import torch

        kw = dict(device=device) if not host else dict(pin_memory=torch.cuda.is_available())
        self.n = n
        self.t = {}
        names = [a for a in self.ARRAYS if dst_ip or a != "dst_ip"]
        for name in names + (self.TCP_ARRAYS if tcp_fields else []):
            self.t[name] = torch.zeros(n, dtype=torch.int32, **kw)
        if counts:
            self.t["flow_counts"] = torch.zeros(max(nflows, 1), dtype=torch.int64, **kw)
            self.t["verdict_counts"] = torch.zeros(DK_V_COUNT, dtype=torch.int64, **kw)
        if tcp_opts:
            self.t["tcp_opts"] = torch.zeros(max(n, 1) * N.TCP_OPTS_DTYPE.itemsize, dtype=torch.uint8, **kw)

    def c_struct(self) -> N.DkRxResults:
        """The ABI struct, rebuilt when an array was replaced: keyed on each array's name and device address (an id()
        could be reused by a replacement tensor after the old one is freed)."""
        key = tuple((k, _ptr(v)) for k, v in self.t.items())
        c = self.__dict__.get("_cs")
        if c is None or c[0] != key:
            c = (key, N.DkRxResults(*[_ptr(self.t.get(name)) for name in N.RESULT_FIELDS]))
            self._cs = c
        return c[1]

    def zero_counts(self) -> None:
        for k in ("flow_counts", "verdict_counts"):
            if k in self.t:
                self.t[k].zero_()

    def to_numpy(self) -> dict:
        out = {}
        for k, v in self.t.items():
            a = v.cpu().numpy()
            if k == "tcp_opts":
                out[k] = a.view(N.TCP_OPTS_DTYPE)[: self.n]
            else:
                out[k] = a.view(np.uint64) if a.dtype == np.int64 else a.view(np.uint32)
        return out


class RxEngine:
    """Batch receive path on one GPU (the drop-in for layer2..layer4 receive + demux, see module docstring)."""

    def __init__(self, config: Config, device: int = 0, lib_path: Optional[str] = None,
                 tuning: Optional[dict] = None):
        """tuning: diagnostic overrides passed to set_tuning right after the context is created (tests and A/B tools;
        the engine's own rule otherwise — the process environment is never consulted)."""
        self.lib = N.load_library() if lib_path is None else N.load_library(lib_path)
        self.config = config
        self.device = device
        cfg = N.DkRxCfg(ipv4(config.local_ipv4_addr), int(config.tcp_checksum_offload),
                        int(config.udp_checksum_offload), 0, device)
        h = ctypes.c_void_p()
        _check(self.lib.dk_rx_ctx_create(ctypes.byref(cfg), ctypes.byref(h)), "dk_rx_ctx_create")
        self._ctx = h
        self.nflows = 0
        # stream handle -> the RxResults of that stream's deferred launch: its pending counter rows hold raw pointers
        # to the counter arrays (dk_rx.h DK_RX_BATCH_DEFER_COUNTS), so the arrays are kept alive until the next launch
        # on the stream, a flush, forget_stream or close
        self._pending = {}
        if tuning:
            self.set_tuning(**tuning)

    @property
    def flow_counts_deferred(self) -> bool:
        """Whether DK_RX_BATCH_DEFER_COUNTS also defers flow_counts for the installed table (dk_rx.h: tables up to
        DK_RX_MAX_DEFERRED_FLOWS entries; larger ones count flows inside the launch itself)."""
        return self.nflows <= N.DK_RX_MAX_DEFERRED_FLOWS

    def close(self) -> None:
        if self._ctx:
            self.lib.dk_rx_ctx_destroy(self._ctx)  # completes every pending row set first
            self._ctx = None
        self._pending = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_sockets(self, flows: np.ndarray) -> None:
        flows = np.ascontiguousarray(flows, dtype=FLOW_DTYPE)
        _check(self.lib.dk_rx_flow_table_set(self._ctx, flows.ctypes.data, len(flows)), "dk_rx_flow_table_set")
        self.nflows = len(flows)

    def results(self, n: int, *, tcp_fields: bool = False, counts: bool = True, dst_ip: bool = True,
                tcp_opts: bool = False) -> RxResults:
        import torch

        return RxResults(n, self.nflows, device=torch.device("cuda", self.device), tcp_fields=tcp_fields,
                         counts=counts, dst_ip=dst_ip, tcp_opts=tcp_opts)

    def receive_batch(self, batch: FrameBatch, results: RxResults, stream=None, defer_counts: bool = False) -> None:
        """Asynchronous on `stream` (a torch.cuda.Stream; default: the current stream). defer_counts: the
        DK_RX_BATCH_DEFER_COUNTS flag — this batch's counter increments land with the next receive_batch on the same
        stream (inside its kernel) or flush_counts()."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        b, r = batch.c_struct(), results.c_struct()
        if defer_counts:
            b.flags |= N.DK_RX_BATCH_DEFER_COUNTS
        _check(self.lib.dk_rx_process(self._ctx, ctypes.byref(b), ctypes.byref(r), ctypes.c_void_p(s.cuda_stream)),
               "dk_rx_process")
        # This launch completes the stream's previous deferred rows (inside its kernel) and leaves its own pending. The
        # previous arrays may be released now that the launch is queued: record_stream keeps the caching allocator
        # from reusing their memory before the work queued on `s` (this kernel) has run — unless they are this
        # launch's own arrays, which stay pending (a receive loop over one result set).
        cnt = [results.t[k] for k in ("flow_counts", "verdict_counts") if k in results.t] if defer_counts else []
        prev = self._pending.get(s.cuda_stream)
        if prev is not None and cnt and len(prev[0]) == len(cnt) and all(a is b for a, b in zip(prev[0], cnt)):
            return
        self._release_pending(s)
        if cnt:
            self._pending[s.cuda_stream] = (cnt, s)

    def _release_pending(self, s) -> None:
        prev = self._pending.pop(s.cuda_stream, None)
        if prev is not None:
            for t in prev[0]:
                if t.is_cuda:
                    t.record_stream(s)

    def flush_counts(self, stream=None) -> None:
        """dk_rx_counts_flush: the counters of a deferred batch on `stream` become current (one small launch)."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _check(self.lib.dk_rx_counts_flush(self._ctx, ctypes.c_void_p(s.cuda_stream)), "dk_rx_counts_flush")
        self._release_pending(s)  # the flush launch is queued on `s`

    def build_id(self) -> str:
        return self.lib.dk_rx_build_id().decode()

    def forget_stream(self, stream) -> None:
        """dk_rx_stream_forget: release this context's scratch of `stream` (a torch.cuda.Stream or a raw hipStream_t
        handle) before the stream is destroyed."""
        h = stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)
        _check(self.lib.dk_rx_stream_forget(self._ctx, ctypes.c_void_p(h)), "dk_rx_stream_forget")
        self._pending.pop(h, None)  # flushed and waited for by dk_rx_stream_forget

    def receive_batch_host(self, blob: np.ndarray, off: np.ndarray, lens: np.ndarray, results: RxResults,
                           chunk_frames: int = 0, aligned16: Optional[bool] = None) -> None:
        """Host-resident batch (NIC ring / socket buffer): pipelined H2D -> kernel -> D2H. Synchronous.
        aligned16 (DK_RX_BATCH_ALIGNED16 hint; offsets are what matters, the staging keeps them mod 16): by default
        computed from `off`."""
        if aligned16 is None:
            aligned16 = bool(np.all(np.asarray(off, dtype=np.uint64) % 16 == 0))
        b = N.DkRxBatch(blob.ctypes.data, blob.nbytes, off.ctypes.data, lens.ctypes.data, len(off),
                        N.DK_RX_BATCH_ALIGNED16 if aligned16 else 0)
        r = results.c_struct()
        _check(self.lib.dk_rx_process_host(self._ctx, ctypes.byref(b), ctypes.byref(r), chunk_frames),
               "dk_rx_process_host")

    def path_stats(self, enable: Optional[bool] = None) -> Optional[np.ndarray]:
        """Diagnostics (dk_diag.h): enable/disable per-path frame counters, or read them ([4] u64)."""
        if enable is not None:
            _check(self.lib.dk_diag_path_stats_enable(self._ctx, int(enable)), "dk_diag_path_stats_enable")
            return None
        out = np.zeros(4, np.uint64)
        _check(self.lib.dk_diag_path_stats_read(self._ctx, out.ctypes.data), "dk_diag_path_stats_read")
        return out

    def set_tuning(self, **knobs) -> None:
        """Diagnostics (dk_diag.h): override the engine's kernel family / schedule / grid choices (-1 = its rule);
        unnamed knobs go back to the rule. Names: N.DK_DIAG_RX_KNOBS (stage, split, small, sched, grid, grid_per_cu, debug,
        lds_table, tail, udp_table, host_zc)."""
        bad = set(knobs) - set(N.DK_DIAG_RX_KNOBS)
        assert not bad, bad
        arr = (ctypes.c_int32 * len(N.DK_DIAG_RX_KNOBS))(*[int(knobs.get(k, -1)) for k in N.DK_DIAG_RX_KNOBS])
        _check(self.lib.dk_diag_rx_set_tuning(self._ctx, arr, len(N.DK_DIAG_RX_KNOBS)), "dk_diag_rx_set_tuning")

    def counts_allreduce(self, results: RxResults, comm: int, stream=None) -> None:
        """dk_rx_flow_counts_allreduce: sum this batch's device counters over every rank of `comm` (an RCCL
        communicator from dk_comm.h), in place, on `stream`."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        r = results.c_struct()
        _check(self.lib.dk_rx_flow_counts_allreduce(self._ctx, ctypes.byref(r), ctypes.c_void_p(comm),
                                                    ctypes.c_void_p(s.cuda_stream)), "dk_rx_flow_counts_allreduce")

    def counts_allreduce_to(self, results: RxResults, flow_out, verdict_out, comm: int, stream=None) -> None:
        """dk_rx_flow_counts_allreduce_to: the node-wide sums of this rank's (accumulating) counters into separate
        device tensors (u64[flow table size], u64[DK_V_COUNT]), on `stream`."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        r = results.c_struct()
        _check(self.lib.dk_rx_flow_counts_allreduce_to(
            self._ctx, ctypes.byref(r), ctypes.c_void_p(flow_out.data_ptr() if flow_out is not None else 0),
            ctypes.c_void_p(verdict_out.data_ptr() if verdict_out is not None else 0), ctypes.c_void_p(comm),
            ctypes.c_void_p(s.cuda_stream)), "dk_rx_flow_counts_allreduce_to")

    def tx_checksum(self, batch: FrameBatch, stream=None) -> None:
        """Fill IPv4/TCP/UDP checksums in place (serialize_and_attach with tx offload off)."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _check(self.lib.dk_tx_checksum(_ptr(batch.blob), batch.frames_bytes, _ptr(batch.off), _ptr(batch.len),
                                       batch.n, ctypes.c_void_p(s.cuda_stream)), "dk_tx_checksum")


    def tx_checksum_fields(self, batch: FrameBatch, fields=None, stream=None):
        """dk_tx_checksum_fields: the same checksums returned, not written — an int32 device tensor of n entries, each
        ipv4 | l4 << 16 (as u32; N.DK_TX_NOT_WRITTEN for a half the in-place fill leaves untouched). The frames are
        only read."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        if fields is None:
            fields = torch.empty(max(batch.n, 1), dtype=torch.int32, device=batch.off.device)
        _check(self.lib.dk_tx_checksum_fields(_ptr(batch.blob), batch.frames_bytes, _ptr(batch.off), _ptr(batch.len),
                                              batch.n, _ptr(fields), ctypes.c_void_p(s.cuda_stream)),
               "dk_tx_checksum_fields")
        return fields


def tx_tuning(split: int = -1, sched: int = -1, grid_per_cu: int = -1) -> None:
    """Diagnostics (dk_diag.h): TX kernel overrides for the process (-1 = the engine's rule)."""
    _check(N.load_library().dk_diag_tx_set_tuning(split, sched, grid_per_cu), "dk_diag_tx_set_tuning")


class Comm:
    """An RCCL communicator (include/dk_comm.h) for the receive path's one collective."""

    def __init__(self, handle: int):
        self.handle = handle

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_uint8 * N.DK_COMM_ID_BYTES)()
        _check(N.load_library().dk_comm_unique_id(buf), "dk_comm_unique_id")
        return bytes(buf)

    @classmethod
    def init_rank(cls, nranks: int, uid: bytes, rank: int, device: int) -> "Comm":
        h = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * N.DK_COMM_ID_BYTES).from_buffer_copy(uid)
        _check(N.load_library().dk_comm_init_rank(ctypes.byref(h), nranks, buf, rank, device), "dk_comm_init_rank")
        return cls(h.value)

    @classmethod
    def init_all(cls, devices) -> list:
        hs = (ctypes.c_void_p * len(devices))()
        devs = (ctypes.c_int32 * len(devices))(*devices)
        _check(N.load_library().dk_comm_init_all(hs, len(devices), devs), "dk_comm_init_all")
        return [cls(h) for h in hs]

    def count(self) -> int:
        n = ctypes.c_int32()
        _check(N.load_library().dk_comm_count(ctypes.c_void_p(self.handle), ctypes.byref(n)), "dk_comm_count")
        return n.value

    def destroy(self) -> None:
        if self.handle:
            _check(N.load_library().dk_comm_destroy(ctypes.c_void_p(self.handle)), "dk_comm_destroy")
            self.handle = 0


def verdict_errno(v: int) -> int:
    return N.load_library().dk_rx_verdict_errno(v)


def raise_for_verdict(v: int) -> None:
    """Turn an error verdict back into the reference's Fail (errno from the reference line it mirrors)."""
    if v in (V["OK_TCP"], V["OK_UDP"]):
        return
    raise Fail(verdict_errno(v), VERDICTS[v])
