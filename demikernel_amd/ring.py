"""TPACKET_V3 receive rings (include/dk_ring.h): the batch L1 ingest that replaces catpowder's
one-recvfrom-per-frame receive (catpowder/linux/mod.rs:138-159) and RECEIVE_BATCH_SIZE = 4 (runtime/network/consts.rs:42).

`build_tpacket3` lays frames out the way the Linux kernel fills a PACKET_RX_RING in TPACKET_V3 mode: a 48-byte block
descriptor, then packets at 8-byte alignment, each a 48-byte tpacket3_hdr with the Ethernet header at tp_mac = 82
(tp_net = TPACKET_ALIGN(TPACKET3_HDRLEN + 16) = 96), so frames sit at 2 mod 16 like NIC buffers. It is how the tests and
the bench make rings without a raw socket; `TpacketRing` drives the engine over a ring's blocks.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _native as N
from .rx import Fail, RxResults, _check

TP_STATUS_KERNEL, TP_STATUS_USER = 0, 1
TPACKET_V3 = 2
BLOCK_DESC_BYTES = 48  # sizeof(struct tpacket_block_desc)
PKT_HDR_BYTES = 48  # sizeof(struct tpacket3_hdr)
TP_MAC, TP_NET = 82, 96


def _check_blocks(rc: int, what: str, blocks: int) -> None:
    """Fail with the blocks the call consumed (a malformed first block counts as consumed: release it too)."""
    if rc != 0:
        e = Fail(rc, what)
        e.blocks = blocks
        raise e


def gpu_numa_node(device: int = 0) -> int:
    """The host NUMA node the GPU's PCIe root sits on (/sys/bus/pci/devices/<bdf>/numa_node), -1 if unknown."""
    import torch

    p = torch.cuda.get_device_properties(device)
    bdf = f"{getattr(p, 'pci_domain_id', 0):04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    try:
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return -1


def _mbind(addr: int, nbytes: int, node: int) -> bool:
    """Bind [addr, addr + nbytes) to one NUMA node before its first touch (mbind MPOL_BIND; x86_64 syscall 237)."""
    libc = ctypes.CDLL(None, use_errno=True)
    mask = (ctypes.c_ulong * 16)()
    mask[node // 64] = 1 << (node % 64)
    return libc.syscall(237, ctypes.c_void_p(addr), ctypes.c_ulong(nbytes), 2, mask, ctypes.c_ulong(16 * 64), 0) == 0


def page_aligned_empty(nbytes: int, numa_node: int = -1) -> np.ndarray:
    """Anonymous-mmap backed u8 array (page aligned, like a PACKET_RX_RING mapping; hipHostRegister-able). numa_node
    >= 0: its pages are placed on that node (the GPU's, gpu_numa_node: a ring the kernel reads over PCIe from the other
    socket's memory lost 5 % in tools/ring_numa.py), as a LibOS gets by creating the ring from a thread
    on the GPU's node."""
    import mmap

    m = mmap.mmap(-1, max(nbytes, 1), flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    a = np.frombuffer(m, np.uint8, count=nbytes)
    if numa_node >= 0 and nbytes:
        _mbind(a.ctypes.data, nbytes, numa_node)  # best effort: placement is a speed property only
    return a


def build_tpacket3(blob: np.ndarray, off: np.ndarray, lens: np.ndarray, block_size: int = 1 << 20,
                   nblocks: Optional[int] = None, seq0: int = 1, numa_node: int = -1):
    """Pack frames blob[off[i]:off[i]+lens[i]] into TPACKET_V3 blocks, every used block closed (TP_STATUS_USER).
    Returns (ring u8 array, blocks used, expected off u32[], expected len u16[]): the descriptors a scan must give.
    numa_node: see page_aligned_empty."""
    lens = np.asarray(lens, np.int64)
    n = len(lens)
    need = (TP_MAC + lens + 7) & ~7  # TOTAL_PKT_LEN_INCL_ALIGN (8-byte packet alignment)
    assert n == 0 or int(need.max()) <= block_size - BLOCK_DESC_BYTES, "a frame does not fit a block"
    block_of = np.zeros(n, np.int64)
    pos = np.zeros(n, np.int64)
    b, cur = 0, BLOCK_DESC_BYTES
    for i, nd in enumerate(need.tolist()):
        if cur + nd > block_size:
            b, cur = b + 1, BLOCK_DESC_BYTES
        block_of[i], pos[i] = b, cur
        cur += nd
    used = b + 1 if n else 0
    nblocks = used if nblocks is None else nblocks
    assert nblocks >= used
    ring = page_aligned_empty(nblocks * block_size, numa_node)
    ring[:] = 0
    start = block_of * block_size + pos
    exp_off = (start + TP_MAC).astype(np.uint32)
    src = np.asarray(off, np.int64)
    for i in range(n):
        L = int(lens[i])
        ring[int(exp_off[i]):int(exp_off[i]) + L] = blob[int(src[i]):int(src[i]) + L]
    last = np.ones(n, bool)
    last[:-1] = block_of[1:] != block_of[:-1]
    hdr = np.zeros((n, PKT_HDR_BYTES // 4), np.uint32)
    hdr[:, 0] = np.where(last, 0, need)  # tp_next_offset (0 on a block's last packet)
    hdr[:, 3] = lens  # tp_snaplen
    hdr[:, 4] = lens  # tp_len
    hdr[:, 5] = TP_STATUS_USER  # tp_status
    hdr[:, 6] = TP_MAC | (TP_NET << 16)  # tp_mac, tp_net
    if n:
        ring[start[:, None] + np.arange(PKT_HDR_BYTES)] = hdr.view(np.uint8).reshape(n, PKT_HDR_BYTES)
    for k in range(used):
        sel = block_of == k
        d = np.zeros(BLOCK_DESC_BYTES // 4, np.uint32)
        d[0] = TPACKET_V3  # version
        d[1] = BLOCK_DESC_BYTES  # offset_to_priv
        d[2] = TP_STATUS_USER  # hdr.bh1.block_status
        d[3] = int(sel.sum())  # num_pkts
        d[4] = BLOCK_DESC_BYTES  # offset_to_first_pkt
        d[5] = int(pos[sel][-1] + need[sel][-1])  # blk_len
        d[6] = (seq0 + k) & 0xFFFFFFFF  # seq_num (low word)
        ring[k * block_size:k * block_size + BLOCK_DESC_BYTES] = d.view(np.uint8)
    return ring, used, exp_off, lens.astype(np.uint16)


class TpacketRing:
    """A TPACKET_V3 ring in host memory (mmap'd from a PACKET_RX_RING socket, or built by build_tpacket3), read by the
    receive engine a block range at a time."""

    def __init__(self, ring: np.ndarray, block_size: int, register: bool = True):
        self.lib = N.load_library()
        self.ring = ring
        self.block_size = block_size
        self.nblocks = ring.nbytes // block_size
        self.registered = False
        if register:
            _check(self.lib.dk_ring_register(ring.ctypes.data, ring.nbytes), "dk_ring_register")
            self.registered = True

    def close(self) -> None:
        if self.registered:
            self.lib.dk_ring_unregister(self.ring.ctypes.data)
            self.registered = False

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def scan(self, first_block: int, nblocks: int, cap: int):
        """Descriptors of the ready blocks: (off u32[], len u16[], blocks consumed)."""
        off = np.zeros(max(cap, 1), np.uint32)
        ln = np.zeros(max(cap, 1), np.uint16)
        nf, nb = ctypes.c_uint32(), ctypes.c_uint32()
        rc = self.lib.dk_ring_scan_tpacket3(self.ring.ctypes.data, self.ring.nbytes, self.block_size, first_block,
                                            nblocks, off.ctypes.data, ln.ctypes.data, cap, ctypes.byref(nf),
                                            ctypes.byref(nb))
        _check_blocks(rc, "dk_ring_scan_tpacket3", nb.value)
        return off[:nf.value], ln[:nf.value], nb.value

    def release(self, first_block: int, nblocks: int) -> None:
        _check(self.lib.dk_ring_release_tpacket3(self.ring.ctypes.data, self.ring.nbytes, self.block_size,
                                                 first_block, nblocks), "dk_ring_release_tpacket3")

    def receive(self, engine, first_block: int, nblocks: int, results: RxResults) -> tuple[int, int]:
        """Process the ready blocks through `engine` (host pipeline); results are host arrays, in ring order.
        Returns (frames, blocks consumed)."""
        nf, nb = ctypes.c_uint32(), ctypes.c_uint32()
        r = results.c_struct()
        rc = self.lib.dk_rx_process_tpacket3(engine._ctx, self.ring.ctypes.data, self.ring.nbytes, self.block_size,
                                             first_block, nblocks, ctypes.byref(r), results.n, ctypes.byref(nf),
                                             ctypes.byref(nb))
        _check_blocks(rc, "dk_rx_process_tpacket3", nb.value)
        return nf.value, nb.value


class PacketSocketRing:
    """A live Linux receive ring: an AF_PACKET / SOCK_RAW socket (ETH_P_ALL) with PACKET_RX_RING in TPACKET_V3 mode,
    mmap'd, bound to one interface — catpowder's RawSocket::new (catpowder/linux/rawsocket/rawsocket.rs:27-39: AF_PACKET,
    SOCK_RAW | SOCK_NONBLOCK, ETH_P_ALL) with the kernel's block ring in place of one recvfrom per frame. `ring` is the
    mapping as a u8 array, for TpacketRing. Needs CAP_NET_RAW (PermissionError otherwise)."""

    SOL_PACKET, PACKET_RX_RING, PACKET_VERSION, PACKET_IGNORE_OUTGOING = 263, 5, 10, 23
    ETH_P_ALL = 3

    def __init__(self, ifname: str = "lo", block_size: int = 1 << 16, nblocks: int = 64, retire_ms: int = 4):
        import mmap
        import socket
        import struct

        s = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(self.ETH_P_ALL))
        try:
            s.setsockopt(self.SOL_PACKET, self.PACKET_VERSION, TPACKET_V3)
            try:  # only what the interface receives (a loopback send is seen again as outgoing otherwise)
                s.setsockopt(self.SOL_PACKET, self.PACKET_IGNORE_OUTGOING, 1)
            except OSError:
                pass
            frame_size = 2048
            # struct tpacket_req3: block_size, block_nr, frame_size, frame_nr, retire_blk_tov, sizeof_priv,
            # feature_req_word
            req = struct.pack("7I", block_size, nblocks, frame_size, block_size * nblocks // frame_size, retire_ms, 0, 0)
            s.setsockopt(self.SOL_PACKET, self.PACKET_RX_RING, req)
            self.mm = mmap.mmap(s.fileno(), block_size * nblocks, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
            s.bind((ifname, self.ETH_P_ALL))
        except Exception:
            s.close()
            raise
        self.sock = s
        self.ifname = ifname
        self.block_size = block_size
        self.nblocks = nblocks
        self.ring = np.frombuffer(self.mm, np.uint8)

    def block_ready(self, k: int) -> bool:
        return bool(int(self.ring[k * self.block_size + 8: k * self.block_size + 12].view(np.uint32)[0]) & TP_STATUS_USER)

    def close(self) -> None:
        self.ring = None
        try:
            self.mm.close()
        except BufferError:  # a numpy view is still alive; the mapping goes with the socket
            pass
        self.sock.close()


def inject(ifname: str, frames: list) -> None:
    """Send raw Ethernet frames out of `ifname` (loopback: they come back in as received frames)."""
    import socket

    s = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(PacketSocketRing.ETH_P_ALL))
    try:
        s.bind((ifname, 0))
        for f in frames:
            s.send(f)
    finally:
        s.close()
