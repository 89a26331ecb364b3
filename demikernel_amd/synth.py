"""Synthetic receive traffic (test and bench tooling; not on the product path).

Frames are built the way the reference's stack would serialize them (Ethernet2 -> IPv4 IHL 5, DF -> TCP without
options or UDP), addressed to the configured local IPv4 from a set of remote flows. Layout: a packed blob with
64-byte aligned frame slots and per-frame (u32 offset, u16 length) descriptors.

Checksums are filled either by `fill_checksums_numpy` — an independent RFC 1071 implementation (sum from 0, end-around
carry), deliberately not the oracle's code — or on the GPU by the product's TX kernel (dk_tx_checksum).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ._native import DK_FLOW_TCP_ACTIVE, DK_FLOW_TCP_PASSIVE, DK_FLOW_UDP, FLOW_DTYPE
from .rx import ipv4

# inetstack/test_helpers/mod.rs:16-21
ALICE_MAC = bytes([0x12, 0x23, 0x45, 0x67, 0x89, 0xAB])
BOB_MAC = bytes([0xAB, 0x89, 0x67, 0x45, 0x23, 0x12])
ALICE_IPV4 = "192.168.1.1"
BOB_IPV4 = "192.168.1.2"
LOCAL_PORT = 12345  # tcp-echo server port used by the reference CI (tools/ci/job/linux.py:145)
SEED = 0xDE31CE1
ETH_MIN_FRAME = 60  # minimum Ethernet frame without FCS: shorter IPv4 packets carry pad bytes


def make_flows(nflows: int, local_ip: str = BOB_IPV4, kind: str = "tcp", seed: int = SEED,
               passive: bool = True) -> np.ndarray:
    """Socket table: `nflows` established TCP connections (Active) plus a Passive listener, or UDP binds."""
    rng = np.random.default_rng(seed)
    lip = ipv4(local_ip)
    if kind == "tcp":
        a = np.zeros(nflows + (1 if passive else 0), dtype=FLOW_DTYPE)
        k = np.arange(nflows, dtype=np.uint32)
        # remote 10.x.y.z (never 0.0.0.0 / broadcast / multicast)
        octs = np.stack([np.full(nflows, 10, np.uint32), (k >> 16) & 255, (k >> 8) & 255, (k & 255) | 1], axis=1)
        rip = (octs[:, 0] | octs[:, 1] << 8 | octs[:, 2] << 16 | octs[:, 3] << 24).astype(np.uint32)
        rport = rng.permutation(np.arange(1024, 65535, dtype=np.uint32))[:nflows].astype(np.uint16) \
            if nflows <= 64511 else rng.integers(1024, 65535, nflows, dtype=np.uint16)
        a["kind"][:nflows] = DK_FLOW_TCP_ACTIVE
        a["local_ip"][:nflows] = lip
        a["remote_ip"][:nflows] = rip
        a["local_port"][:nflows] = LOCAL_PORT
        a["remote_port"][:nflows] = rport
        if passive:
            a[nflows] = (DK_FLOW_TCP_PASSIVE, lip, 0, LOCAL_PORT, 0)
        return a
    a = np.zeros(nflows, dtype=FLOW_DTYPE)
    a["kind"] = DK_FLOW_UDP
    a["local_ip"] = lip
    if kind == "udp_random_ports":  # binds spread over the port space (no two on one cache line of the port table)
        a["local_port"] = rng.permutation(np.arange(1024, 65536, dtype=np.uint32))[:nflows].astype(np.uint16)
    else:
        a["local_port"] = (5000 + np.arange(nflows)).astype(np.uint16)
    return a


@dataclass
class Traffic:
    """Per-frame header fields (numpy arrays of length n)."""

    ip_len: np.ndarray  # IPv4 total_length (u16)
    frame_len: np.ndarray  # frame length L (u16), >= 14 + ip_len (Ethernet pad)
    proto: np.ndarray  # 6 or 17 (u8)
    src_ip: np.ndarray
    dst_ip: np.ndarray
    sport: np.ndarray
    dport: np.ndarray
    seq: np.ndarray
    ack: np.ndarray
    flags: np.ndarray
    window: np.ndarray
    ip_id: np.ndarray
    ttl: np.ndarray
    flow: np.ndarray  # index of the flow each frame belongs to

    @property
    def n(self) -> int:
        return len(self.ip_len)


def traffic(n: int, ip_len, flows: np.ndarray, local_ip: str = BOB_IPV4, seed: int = SEED) -> Traffic:
    """Data segments of the given IPv4 total lengths, spread uniformly over the Active TCP / UDP flows."""
    rng = np.random.default_rng(seed)
    ip_len = np.broadcast_to(np.asarray(ip_len, dtype=np.uint16), (n,)).copy()
    frame_len = np.maximum(ip_len.astype(np.int64) + 14, ETH_MIN_FRAME).astype(np.uint16)
    data_flows = np.nonzero(flows["kind"] != DK_FLOW_TCP_PASSIVE)[0]
    fidx = data_flows[rng.integers(0, len(data_flows), n)]
    fl = flows[fidx]
    is_tcp = fl["kind"] == DK_FLOW_TCP_ACTIVE
    proto = np.where(is_tcp, 6, 17).astype(np.uint8)
    # UDP remotes: 10.1.x.y with random source ports
    udp_src = (10 | 1 << 8 | rng.integers(0, 256, n, dtype=np.uint32) << 16
               | (rng.integers(0, 255, n, dtype=np.uint32) + 1) << 24).astype(np.uint32)
    src = np.where(is_tcp, fl["remote_ip"], udp_src).astype(np.uint32)
    sport = np.where(is_tcp, fl["remote_port"], rng.integers(1024, 65535, n, dtype=np.uint16)).astype(np.uint16)
    return Traffic(
        ip_len=ip_len, frame_len=frame_len, proto=proto, src_ip=src,
        dst_ip=np.full(n, ipv4(local_ip), dtype=np.uint32), sport=sport, dport=fl["local_port"].astype(np.uint16),
        seq=rng.integers(0, 2**32, n, dtype=np.uint32), ack=rng.integers(0, 2**32, n, dtype=np.uint32),
        flags=np.full(n, 0x18, np.uint8), window=rng.integers(0, 65536, n, dtype=np.uint16),
        ip_id=rng.integers(0, 65536, n, dtype=np.uint16), ttl=np.full(n, 64, np.uint8), flow=fidx.astype(np.int64))


def tcp_streams(n: int, nconns: int, ip_len=None, *, reorder: float = 3.0, dup: float = 0.02, oow: float = 0.005,
                fin: float = 0.3, rare: float = 0.002, rst: float = 0.05, buffer_size: int = 65535,
                seed: int = SEED):
    """Established TCP byte streams for the dk_tcp path: `n` data segments over `nconns` Active connections, each
    connection's segments contiguous in sequence space from a random RCV.NXT (wrapping included), arriving with local
    reordering (each segment displaced by up to ~`reorder` places within its connection), plus a `dup` fraction of
    retransmissions from earlier stream offsets (duplicates and partial overlaps) and an `oow` fraction of strays far
    beyond the window (neither takes stream bytes, so the streams stay gap-free), FIN on the last
    segment of a `fin` fraction of the connections, RST on about a `rst` fraction of the connections, and a `rare`
    fraction of extra copies with SYN / ACK bit clear / ack beyond SND.NXT. Returns (flows, Traffic, host connection table for
    dk_tcp (one row per flow; the Passive listener's row is DK_TCP_NONE))."""
    from .tcp import CONN_DTYPE, ESTABLISHED

    rng = np.random.default_rng(seed + 7)
    flows = make_flows(nconns, seed=seed)
    tr = traffic(n, 40 if ip_len is None else ip_len, flows, seed=seed)
    if ip_len is None:
        tr.ip_len = (40 + rng.integers(0, 1461, n)).astype(np.uint16)
        tr.frame_len = np.maximum(tr.ip_len.astype(np.int64) + 14, ETH_MIN_FRAME).astype(np.uint16)
    plen = tr.ip_len.astype(np.int64) - 40
    f = tr.flow
    isn = rng.integers(0, 2**32, nconns, dtype=np.uint64)
    isn[: min(nconns, 4)] = 2**32 - 3000  # a few streams wrap inside the batch
    snd = rng.integers(0, 2**32, nconns, dtype=np.uint64)
    # stream order: arrival rank within the connection plus noise, re-ranked
    arr = np.arange(n)
    r = rng.random(n)
    d = r < dup
    o = (r >= dup) & (r < dup + oow)
    x = (r >= dup + oow) & (r < dup + oow + 3 * rare)  # copies that the SYN / ACK checks will drop
    key = np.lexsort((arr + rng.uniform(0, reorder + 1e-9, n), f))  # frames sorted by (conn, noisy arrival)
    order_len = np.where((d | o | x)[key], 0, plen[key])  # resent / stray segments take no new stream bytes
    csum = np.cumsum(order_len)
    first = np.ones(n, bool)
    first[1:] = f[key][1:] != f[key][:-1]
    base = np.maximum.accumulate(np.where(first, csum - order_len, 0))
    stream_off = np.empty(n, np.int64)
    stream_off[key] = csum - order_len - base
    seq = (isn[f] + stream_off.astype(np.uint64)) & 0xFFFFFFFF
    seq[d] = (seq[d] - rng.integers(1, 3000, int(d.sum())).astype(np.uint64)) & 0xFFFFFFFF
    seq[o] = (seq[o] + np.uint64(buffer_size) + rng.integers(0, 1 << 20, int(o.sum())).astype(np.uint64)) & 0xFFFFFFFF
    tr.seq = seq.astype(np.uint32)
    tr.ack = ((snd[f] - rng.integers(0, 4096, n).astype(np.uint64)) & 0xFFFFFFFF).astype(np.uint32)
    flags = np.full(n, 0x18, np.uint8)  # PSH | ACK
    last = np.zeros(n, bool)
    last_key = np.ones(n, bool)
    last_key[:-1] = f[key][1:] != f[key][:-1]
    last[key[last_key]] = True
    fin_conn = rng.random(nconns) < fin
    flags[last & fin_conn[f]] |= 0x01
    # segments the checks drop carry no stream bytes of their own (rare SYN / no-ACK / unsent-ACK copies), so they
    # leave no holes; RST closes its connection wherever it lands
    extra = d | o | x
    flags[extra & (rng.random(n) < 0.2)] |= 0x02  # SYN
    flags[extra & (rng.random(n) < 0.2)] &= ~np.uint8(0x10)  # ACK bit clear
    flags[rng.random(n) < rst * nconns / max(n, 1)] |= 0x04  # RST: about `rst` of the connections get one
    unsent = extra & (rng.random(n) < 0.2)
    tr.ack[unsent] = ((snd[f[unsent]] + rng.integers(1, 1 << 20, int(unsent.sum())).astype(np.uint64))
                      & 0xFFFFFFFF).astype(np.uint32)
    tr.flags = flags
    table = np.zeros(len(flows), CONN_DTYPE)
    table["state"][:nconns] = ESTABLISHED
    table["receive_next"][:nconns] = isn.astype(np.uint32)
    table["reader_next"][:nconns] = isn.astype(np.uint32)
    table["buffer_size"][:nconns] = buffer_size
    table["send_next"][:nconns] = snd.astype(np.uint32)
    return flows, tr, table


def imix_ip_lengths(n: int, seed: int = SEED) -> np.ndarray:
    """Simple IMIX: IPv4 total lengths 40 / 576 / 1500 in ratio 7:4:1, shuffled."""
    rng = np.random.default_rng(seed + 1)
    return rng.choice(np.array([40, 576, 1500], np.uint16), size=n, p=[7 / 12, 4 / 12, 1 / 12])


def layout(frame_len: np.ndarray, align: int = 64) -> tuple[np.ndarray, int]:
    slots = (frame_len.astype(np.int64) + align - 1) // align * align
    off = np.zeros(len(frame_len), np.int64)
    np.cumsum(slots[:-1], out=off[1:])
    total = int(off[-1] + slots[-1]) if len(frame_len) else 0
    assert total <= 0xFFFFFF00, "a batch blob is limited to DK_RX_MAX_BLOB = 4 GiB - 256 (u32 offsets)"
    return off.astype(np.uint32), total


HDR_TCP, HDR_UDP = 54, 42


def headers(tr: Traffic) -> np.ndarray:
    """(n, 54) header bytes (UDP rows use the first 42), checksum fields zero."""
    n = tr.n
    h = np.zeros((n, HDR_TCP), np.uint8)
    h[:, 0:6] = np.frombuffer(BOB_MAC, np.uint8)
    h[:, 6:12] = np.frombuffer(ALICE_MAC, np.uint8)
    h[:, 12], h[:, 13] = 0x08, 0x00
    h[:, 14], h[:, 15] = 0x45, 0x00

    def be16(col, v):
        h[:, col] = (v >> 8) & 255
        h[:, col + 1] = v & 255

    def be32(col, v):
        for k in range(4):
            h[:, col + k] = (v >> (24 - 8 * k)) & 255

    be16(16, tr.ip_len.astype(np.uint32))
    be16(18, tr.ip_id.astype(np.uint32))
    h[:, 20], h[:, 21] = 0x40, 0x00  # DF
    h[:, 22] = tr.ttl
    h[:, 23] = tr.proto
    h[:, 26:30] = tr.src_ip.astype("<u4").view(np.uint8).reshape(n, 4)
    h[:, 30:34] = tr.dst_ip.astype("<u4").view(np.uint8).reshape(n, 4)
    be16(34, tr.sport.astype(np.uint32))
    be16(36, tr.dport.astype(np.uint32))
    tcp = tr.proto == 6
    be32(38, tr.seq.astype(np.uint64))
    be32(42, tr.ack.astype(np.uint64))
    h[:, 46] = 0x50
    h[:, 47] = tr.flags
    be16(48, tr.window.astype(np.uint32))
    # UDP rows: bytes 38..41 = length, checksum 0; bytes 42.. are payload (overwritten below by the caller's blob)
    udp = ~tcp
    seglen = tr.ip_len.astype(np.uint32) - 20
    h[udp, 38] = (seglen[udp] >> 8) & 255
    h[udp, 39] = seglen[udp] & 255
    h[udp, 40] = 0
    h[udp, 41] = 0
    return h


def _fold_complement(s: np.ndarray) -> np.ndarray:
    s = s.astype(np.uint64)
    while np.any(s > 0xFFFF):
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def fill_checksums_numpy(blob: np.ndarray, off: np.ndarray, tr: Traffic, chunk: int = 8192) -> None:
    """Independent RFC 1071 checksums (IPv4 header, TCP/UDP with pseudo-header), vectorised per size group."""
    key = tr.ip_len.astype(np.int64) * 32 + tr.proto
    for k in np.unique(key):
        idx_all = np.nonzero(key == k)[0]
        tot, proto = int(k // 32), int(k % 32)
        S, E = 34, 14 + tot
        for c in range(0, len(idx_all), chunk):
            idx = idx_all[c:c + chunk]
            o = off[idx].astype(np.int64)
            hdr = blob[o[:, None] + np.arange(14, 34)].astype(np.uint32)
            w = hdr[:, 0::2] << 8 | hdr[:, 1::2]
            w[:, 5] = 0
            ipc = _fold_complement(w.sum(axis=1))
            blob[o + 24] = (ipc >> 8).astype(np.uint8)
            blob[o + 25] = (ipc & 255).astype(np.uint8)
            if E - S < (20 if proto == 6 else 8):
                continue
            seg = blob[o[:, None] + np.arange(S, E)].astype(np.uint32)
            cs = 16 if proto == 6 else 6
            seg[:, cs] = 0
            seg[:, cs + 1] = 0
            if seg.shape[1] % 2:
                seg = np.concatenate([seg, np.zeros((len(idx), 1), np.uint32)], axis=1)
            words = (seg[:, 0::2] << 8 | seg[:, 1::2]).sum(axis=1, dtype=np.uint64)
            src, dst = tr.src_ip[idx].astype(np.uint64), tr.dst_ip[idx].astype(np.uint64)

            def hl(a):  # BE words of an octet-order address
                return ((a & 255) << 8 | (a >> 8) & 255) + (((a >> 16) & 255) << 8 | (a >> 24) & 255)

            pseudo = hl(src) + hl(dst) + proto + (E - S)
            c4 = _fold_complement(words + pseudo)
            blob[o + S + cs] = (c4 >> 8).astype(np.uint8)
            blob[o + S + cs + 1] = (c4 & 255).astype(np.uint8)


def build_numpy(tr: Traffic, align: int = 64, seed: int = SEED, checksums: bool = True):
    """Host blob for tests: random payload, headers, independent checksums. Returns (blob, off, len)."""
    off, total = layout(tr.frame_len, align)
    rng = np.random.default_rng(seed + 2)
    blob = np.frombuffer(rng.bytes(total), np.uint8).copy()
    h = headers(tr)
    tcp = tr.proto == 6
    for hl, sel in ((HDR_TCP, tcp), (HDR_UDP, ~tcp)):
        idx = np.nonzero(sel)[0]
        if len(idx):
            blob[off[idx].astype(np.int64)[:, None] + np.arange(hl)] = h[idx, :hl]
    # Ethernet padding beyond the IPv4 datagram: zero bytes, as a NIC would deliver them
    pad = tr.frame_len.astype(np.int64) - 14 - tr.ip_len.astype(np.int64)
    for i in np.nonzero(pad > 0)[0]:
        blob[off[i] + 14 + int(tr.ip_len[i]): off[i] + int(tr.frame_len[i])] = 0
    if checksums:
        fill_checksums_numpy(blob, off, tr)
    return blob, off, tr.frame_len.copy()


def build_device(tr: Traffic, engine, align: int = 64, seed: int = SEED):
    """HBM blob for the bench: payload from torch's device RNG, headers scattered from the host, checksums by the
    product TX kernel (dk_tx_checksum). Returns a FrameBatch."""
    import torch

    from .rx import FrameBatch

    dev = torch.device("cuda", engine.device)
    off, total = layout(tr.frame_len, align)
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    blob = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
    off_t = torch.from_numpy(off.astype(np.int64)).to(dev)
    h = torch.from_numpy(headers(tr)).to(dev)
    tcp = torch.from_numpy(tr.proto == 6).to(dev)
    for p in range(HDR_TCP):
        if p < HDR_UDP:
            blob[off_t + p] = h[:, p]
        else:
            sel = off_t[tcp] + p
            blob[sel] = h[tcp, p]
    pad = (tr.frame_len.astype(np.int64) - 14 - tr.ip_len.astype(np.int64))
    if np.any(pad > 0):
        for d in np.unique(pad[pad > 0]):
            sel = np.nonzero(pad == d)[0]
            base = torch.from_numpy((off[sel].astype(np.int64) + 14 + tr.ip_len[sel].astype(np.int64))).to(dev)
            for k in range(int(d)):
                blob[base + k] = 0
    batch = FrameBatch(blob, torch.from_numpy(off.view(np.int32)).to(dev),
                       torch.from_numpy(tr.frame_len.view(np.int16)).to(dev),
                       aligned16=blob.data_ptr() % 16 == 0)  # 64-byte slots
    engine.tx_checksum(batch)
    return batch


# Corruptions applied to a `frac` tail of frames after checksums (exercise verdict parity).
CORRUPTIONS = [
    ("payload_flip", lambda L, tot: (14 + tot - 1, 0x5A)),  # -> TCP/UDP checksum mismatch
    ("ip_csum_flip", lambda L, tot: (25, 0x01)),            # -> IPv4 header checksum mismatch
    ("mf_flag", lambda L, tot: (20, 0x20)),                 # -> MF (fragmentation unsupported)
    ("ttl_zero", lambda L, tot: (22, None)),                # -> TTL 0
    ("totlen_big", lambda L, tot: (16, 0x40)),              # -> total_length > datagram
    ("ethertype", lambda L, tot: (12, 0x11)),               # -> unsupported ethertype
    ("version", lambda L, tot: (14, 0x10)),                 # -> IP version 5
    ("doff_small", lambda L, tot: (46, 0x50 ^ 0x30)),       # -> TCP data offset 3 (TCP) / payload (UDP)
]


def corruption_plan(n: int, frac: float, tr: Traffic, seed: int = SEED):
    """(frame index, byte position, xor mask or None=zero) for a deterministic `frac` of the frames."""
    rng = np.random.default_rng(seed + 3)
    m = int(round(n * frac))
    idx = np.sort(rng.choice(n, size=m, replace=False)) if m else np.zeros(0, np.int64)
    kinds = rng.integers(0, len(CORRUPTIONS), m)
    plan = []
    for i, k in zip(idx, kinds):
        pos, mask = CORRUPTIONS[k][1](int(tr.frame_len[i]), int(tr.ip_len[i]))
        plan.append((int(i), pos, mask))
    return plan


def corrupt_numpy(blob: np.ndarray, off: np.ndarray, plan) -> None:
    for i, pos, mask in plan:
        a = int(off[i]) + pos
        blob[a] = 0 if mask is None else blob[a] ^ mask


def corrupt_device(batch, off: np.ndarray, plan) -> None:
    import torch

    if not plan:
        return
    dev = batch.blob.device
    zero = [int(off[i]) + p for i, p, m in plan if m is None]
    flip = [(int(off[i]) + p, m) for i, p, m in plan if m is not None]
    if zero:
        batch.blob[torch.tensor(zero, dtype=torch.int64, device=dev)] = 0
    if flip:
        a = torch.tensor([x for x, _ in flip], dtype=torch.int64, device=dev)
        m = torch.tensor([y for _, y in flip], dtype=torch.uint8, device=dev)
        batch.blob[a] = batch.blob[a] ^ m
