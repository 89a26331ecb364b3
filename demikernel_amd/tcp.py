"""Established-state TCP receive processing on the GPU (include/dk_tcp.h).

What ControlBlock::poll does to each segment TcpPeer::receive queued for an established socket (tcp/socket.rs:308-314
-> tcp/established/ctrlblk.rs:350-440: in-window checks and trims, RST / SYN / ACK checks, in-order delivery, the
out-of-order store, remote FIN), run for every connection of a dk_rx batch at once. The connection table is a device
array of struct dk_tcp_conn (CONN_DTYPE) indexed by the flow_id dk_rx assigns, updated in place across batches.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _native as N
from .rx import RxResults, _check, _ptr

CONN_DTYPE, VIEW_DTYPE = N.CONN_DTYPE, N.VIEW_DTYPE
ACTIONS, A = N.TCP_ACTIONS, N.A
NONE, ESTABLISHED, CLOSED = N.DK_TCP_NONE, N.DK_TCP_ESTABLISHED, N.DK_TCP_CLOSED
REF_EOF, OOO_MAX, DELIV_EXTRA = N.DK_TCP_REF_EOF, N.DK_TCP_OOO_MAX, N.DK_TCP_DELIV_EXTRA


def conn_table(nconns: int, *, receive_next=0, send_next=0, buffer_size=65535, state=ESTABLISHED) -> np.ndarray:
    """Host connection table (CONN_DTYPE): every connection established at the given RCV.NXT / SND.NXT, reader caught
    up (reader_next = RCV.NXT), empty out-of-order store. Scalars or per-connection arrays."""
    t = np.zeros(nconns, CONN_DTYPE)
    t["state"] = state
    t["receive_next"] = np.asarray(receive_next, np.int64).astype(np.uint32)
    t["reader_next"] = t["receive_next"]
    t["buffer_size"] = buffer_size
    t["send_next"] = np.asarray(send_next, np.int64).astype(np.uint32)
    return t


class TcpOut:
    """Device output arrays of one dk_tcp_rx_process call (dk_tcp_out)."""

    def __init__(self, n: int, nconns: int, device: int = 0):
        import torch

        dev = torch.device("cuda", device)
        self.n, self.nconns = n, nconns
        self.action = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev)
        self.view = torch.zeros(max(n, 1) * 3, dtype=torch.int32, device=dev)
        self.deliv = torch.zeros(max(n + DELIV_EXTRA * nconns, 1) * 3, dtype=torch.int32, device=dev)
        self.deliv_start = torch.zeros(max(nconns, 1), dtype=torch.int32, device=dev)
        self.deliv_count = torch.zeros(max(nconns, 1), dtype=torch.int32, device=dev)

    def c_struct(self) -> N.DkTcpOut:
        return N.DkTcpOut(_ptr(self.action), _ptr(self.view), _ptr(self.deliv), _ptr(self.deliv_start),
                          _ptr(self.deliv_count))

    def to_numpy(self) -> dict:
        v = lambda t, k: t.cpu().numpy().view(np.uint32).view(VIEW_DTYPE)[:k]  # noqa: E731
        return {"action": self.action.cpu().numpy()[:self.n], "view": v(self.view, self.n),
                "deliv": v(self.deliv, self.n + DELIV_EXTRA * self.nconns),
                "deliv_start": self.deliv_start.cpu().numpy().view(np.uint32)[:self.nconns],
                "deliv_count": self.deliv_count.cpu().numpy().view(np.uint32)[:self.nconns]}

    def delivered(self, c: int, host: Optional[dict] = None) -> np.ndarray:
        """Connection c's pushed buffers (views, DK_TCP_REF_EOF for the EOF buffer), in receive-queue order."""
        h = self.to_numpy() if host is None else host
        s = int(h["deliv_start"][c])
        return h["deliv"][s:s + int(h["deliv_count"][c])]


class TcpReceiver:
    """Per-GPU TCP receive processing over a device connection table (the ControlBlock receive halves)."""

    def __init__(self, device: int = 0, lib_path: str | None = None, walk: str | None = None, relay_waves: int = 8,
                 radix_sort: bool = False):
        """walk: a diagnostic override of the engine's walk choice ("lane", "wave", "relay", "scan"; None = the rule),
        set through dk_diag_tcp_set_walk; radix_sort: order the batch with the radix sort even where the rule takes
        the counting sort (dk_diag_tcp_set_sort)."""
        self.lib = N.load_library(lib_path) if lib_path else N.load_library()
        self.device = device
        h = ctypes.c_void_p()
        _check(self.lib.dk_tcp_ctx_create(device, ctypes.byref(h)), "dk_tcp_ctx_create")
        self._ctx = h
        if walk is not None or relay_waves != 8:
            _check(self.lib.dk_diag_tcp_set_walk(self._ctx, N.DK_TCP_WALKS[walk] if walk else -1, relay_waves),
                   "dk_diag_tcp_set_walk")
        if radix_sort:
            _check(self.lib.dk_diag_tcp_set_sort(self._ctx, 1), "dk_diag_tcp_set_sort")

    @property
    def last_walk(self) -> Optional[str]:
        """The walk the last process() call ran (dk_diag_tcp_last_walk), None before the first."""
        w = self.lib.dk_diag_tcp_last_walk(self._ctx)
        return {v: k for k, v in N.DK_TCP_WALKS.items()}.get(w)

    def close(self) -> None:
        if self._ctx:
            self.lib.dk_tcp_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def conns_to_device(self, table: np.ndarray):
        import torch

        t = np.ascontiguousarray(table, CONN_DTYPE)
        return torch.from_numpy(t.view(np.uint8).copy()).to(torch.device("cuda", self.device))

    @staticmethod
    def conns_to_host(dev) -> np.ndarray:
        return dev.cpu().numpy().view(CONN_DTYPE).copy()

    def process(self, rx: RxResults, conns, out: TcpOut, stream=None) -> None:
        """Run the TCP segments of the dk_rx batch `rx` (made with tcp_fields=True) through `conns` (a uint8 device
        tensor of nconns * 288 bytes, updated in place). Asynchronous on `stream` (default: the current stream)."""
        import torch

        assert conns.dtype == torch.uint8 and conns.numel() % CONN_DTYPE.itemsize == 0
        nconns = conns.numel() // CONN_DTYPE.itemsize
        assert out.n == rx.n and out.nconns == nconns
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        r, o = rx.c_struct(), out.c_struct()
        _check(self.lib.dk_tcp_rx_process(self._ctx, ctypes.byref(r), rx.n, _ptr(conns), nconns, ctypes.byref(o),
                                          ctypes.c_void_p(s.cuda_stream)), "dk_tcp_rx_process")
