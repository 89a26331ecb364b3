"""Single-frame builders for tests (pure Python; checksums by an independent RFC 1071 implementation).

`ipv4_header` mirrors the reference test helper build_ipv4_header (src/rust/inetstack/protocols/layer3/ipv4/
tests.rs:22-72), including its quirk of computing the checksum with Ipv4Header::compute_checksum (first 20 bytes only).
"""
from __future__ import annotations

import random
import struct

from demikernel_amd.rx import ipv4
from demikernel_amd.synth import ALICE_IPV4, ALICE_MAC, BOB_IPV4, BOB_MAC


def rfc1071(data: bytes, start: int = 0) -> int:
    """One's-complement checksum, RFC 1071 style (sum from 0, end-around carry, complement)."""
    if len(data) % 2:
        data = data + b"\0"
    s = start + sum(struct.unpack(f"!{len(data) // 2}H", data))
    while s > 0xFFFF:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def ref_checksum(words_sum_be: int) -> int:
    """The reference's form: state = 0xFFFF + sum; while state > 0xFFFF: state -= 0xFFFF; !state."""
    s = 0xFFFF + words_sum_be
    while s > 0xFFFF:
        s -= 0xFFFF
    return (~s) & 0xFFFF


def ip_bytes(a: str | int) -> bytes:
    return (ipv4(a) if isinstance(a, str) else a).to_bytes(4, "little")


def ipv4_header(version=4, ihl=5, dscp=0, ecn=0, total_length=20, ident=0, flags=0x2, frag=0, ttl=64, proto=6,
                src=ALICE_IPV4, dst=BOB_IPV4, checksum=None, options=b"") -> bytes:
    h = bytearray(max(ihl, 5) * 4 if not options else 20 + len(options))
    h[0] = ((version & 0xF) << 4) | (ihl & 0xF)
    h[1] = ((dscp & 0x3F) << 2) | (ecn & 0x3)
    h[2:4] = struct.pack("!H", total_length & 0xFFFF)
    h[4:6] = struct.pack("!H", ident)
    h[6:8] = struct.pack("!H", ((flags & 7) << 13) | (frag & 0x1FFF))
    h[8] = ttl
    h[9] = proto
    h[12:16] = ip_bytes(src)
    h[16:20] = ip_bytes(dst)
    if options:
        h[20:20 + len(options)] = options
    if checksum is None:
        # Ipv4Header::compute_checksum: 9 words of the first 20 bytes (ipv4/header.rs:280-301)
        w = struct.unpack("!10H", bytes(h[:20]))
        checksum = ref_checksum(sum(w) - w[5])
    h[10:12] = struct.pack("!H", checksum)
    return bytes(h)


def eth_header(ethertype=0x0800, dst=BOB_MAC, src=ALICE_MAC) -> bytes:
    return bytes(dst) + bytes(src) + struct.pack("!H", ethertype)


def pseudo(src, dst, proto, seglen) -> int:
    s, d = ip_bytes(src), ip_bytes(dst)
    return sum(struct.unpack("!4H", s + d)) + proto + seglen


def tcp_segment(src=ALICE_IPV4, dst=BOB_IPV4, sport=40000, dport=12345, seq=1, ack=2, flags=0x18, window=4096,
                urg=0, options=b"", payload=b"", doff=None, checksum=None, b12_extra=0) -> bytes:
    options = options + b"\0" * (-len(options) % 4)  # pad with EOL to a 32-bit boundary
    hl = 20 + len(options)
    if doff is None:
        doff = hl // 4
    h = bytearray(struct.pack("!HHIIBBHHH", sport, dport, seq, ack, (doff << 4) | b12_extra, flags, window, 0, urg))
    seg = bytes(h) + options + payload
    if checksum is None:
        checksum = rfc1071(seg, pseudo(src, dst, 6, len(seg)))
    return seg[:16] + struct.pack("!H", checksum) + seg[18:]


def udp_segment(src=ALICE_IPV4, dst=BOB_IPV4, sport=40000, dport=5000, payload=b"", length=None,
                checksum=None) -> bytes:
    L = 8 + len(payload) if length is None else length
    seg = struct.pack("!HHHH", sport, dport, L & 0xFFFF, 0) + payload
    if checksum is None:
        checksum = rfc1071(seg, pseudo(src, dst, 17, len(seg)))
    return seg[:6] + struct.pack("!H", checksum) + seg[8:]


def frame(l4: bytes = b"", proto=6, src=ALICE_IPV4, dst=BOB_IPV4, ip_options=b"", pad=0, ethertype=0x0800,
          **ip_kw) -> bytes:
    ihl = 5 + len(ip_options) // 4
    tot = ip_kw.pop("total_length", ihl * 4 + len(l4))
    ip = ipv4_header(ihl=ip_kw.pop("ihl", ihl), total_length=tot, proto=proto, src=src, dst=dst,
                     options=ip_options, **ip_kw)
    return eth_header(ethertype) + ip + l4 + b"\0" * pad


def tcp_frame(payload=b"", src=ALICE_IPV4, dst=BOB_IPV4, options=b"", sport=40000, dport=12345, pad=0,
              ip_options=b"", tcp_kw=None, **ip_kw) -> bytes:
    seg = tcp_segment(src=src, dst=dst, sport=sport, dport=dport, options=options, payload=payload,
                      **(tcp_kw or {}))
    return frame(seg, 6, src, dst, ip_options=ip_options, pad=pad, **ip_kw)


def udp_frame(payload=b"", src=ALICE_IPV4, dst=BOB_IPV4, sport=40000, dport=5000, pad=0, udp_kw=None,
              **ip_kw) -> bytes:
    seg = udp_segment(src=src, dst=dst, sport=sport, dport=dport, payload=payload, **(udp_kw or {}))
    return frame(seg, 17, src, dst, pad=pad, **ip_kw)


def icmp_message(type_=8, code=0, ident=0x1234, seq=1, payload=b"", checksum=None) -> bytes:
    """Icmpv4Header::serialize_and_attach (icmpv4/header.rs:71-84): type, code, checksum, rest-of-header (id, seq)."""
    m = bytes([type_, code, 0, 0]) + struct.pack("!HH", ident, seq) + payload
    if checksum is None:
        checksum = rfc1071(m)
    return m[:2] + struct.pack("!H", checksum) + m[4:]


def icmp_frame(type_=8, code=0, ident=0x1234, seq=1, payload=b"", checksum=None, src=ALICE_IPV4, dst=BOB_IPV4,
               **kw) -> bytes:
    return frame(icmp_message(type_, code, ident, seq, payload, checksum), 1, src, dst, **kw)


def arp_frame(op=1, sha=ALICE_MAC, spa=ALICE_IPV4, tha=(0,) * 6, tpa=BOB_IPV4, htype=1, ptype=0x0800, hlen=6, plen=4,
              pad=0) -> bytes:
    """ArpHeader::create_and_serialize (arp/header.rs:117-135) behind an Ethernet header, as build_arp_query
    (arp/tests.rs:199-213) builds a query."""
    pdu = struct.pack("!HHBBH", htype, ptype, hlen, plen, op) + bytes(sha) + ip_bytes(spa) + bytes(tha) + ip_bytes(tpa)
    return eth_header(0x0806, dst=(0xFF,) * 6) + pdu + b"\0" * pad


def pack(frames: list[bytes], align: int = 64, misalign: list[int] | None = None):
    """Pack frames into a blob with aligned slots (+ optional per-frame misalignment). Returns numpy arrays."""
    import numpy as np

    offs, pos = [], 0
    for i, f in enumerate(frames):
        pos = (pos + align - 1) // align * align
        if misalign:
            pos += misalign[i % len(misalign)]
        offs.append(pos)
        pos += len(f)
    blob = np.zeros(max(pos, 1), np.uint8)
    for o, f in zip(offs, frames):
        blob[o:o + len(f)] = np.frombuffer(f, np.uint8)
    return blob, np.array(offs, np.uint32), np.array([len(f) for f in frames], np.uint16)


# ---------------------------------------------------------------------------------------------------------------------
# A corpus that reaches every Appendix A branch, with the verdict each frame is built to produce.
# ---------------------------------------------------------------------------------------------------------------------
def tcp_opt_cases():
    """(options bytes, expected verdict name or None=ok) — tcp/header.rs:215-302."""
    ts = bytes([8, 10]) + b"\x00\x00\x00\x01\x00\x00\x00\x02"
    return [
        (bytes([2, 4, 0x05, 0xB4]), None),                       # MSS
        (bytes([1, 1, 3, 3, 7, 0]), None),                       # NOP NOP WS EOL (pad)
        (bytes([4, 2, 1, 1]), None),                             # SACKP
        (bytes([1, 1]) + ts, None),                              # NOP NOP TS
        (bytes([5, 10]) + bytes(8) + bytes([0, 0]), None),       # SACK 1 block + EOL pad
        (bytes([0, 2, 4, 0x05]), None),                          # EOL first: rest ignored
        (bytes([2, 3, 0, 0]), "TCP_OPT"),                        # MSS len != 4
        (bytes([3, 4, 0, 0]), "TCP_OPT"),                        # WS len != 3
        (bytes([4, 3, 0, 0]), "TCP_OPT"),                        # SACKP len != 2
        (bytes([5, 11]) + bytes(10), "TCP_OPT"),                 # SACK invalid size
        (bytes([8, 9]) + bytes(10), "TCP_OPT"),                  # TS len != 10
        (bytes([9, 2, 0, 0]), "TCP_OPT"),                        # unknown kind
        (bytes([4, 2]) * 6, "TCP_OPT"),                          # six options -> too many
        (bytes([4, 2]) * 5 + bytes([1, 1]), None),               # five options + NOPs: ok
        (bytes([1, 1, 1, 2]), "TCP_OPT_EIO"),                    # MSS kind, length byte missing
        (bytes([1, 1, 2, 4]), "TCP_OPT_EIO"),                    # MSS body missing
        (bytes([1, 5, 18]) + bytes(9), "TCP_OPT_EIO"),           # SACK claims 2 blocks, has 1
        (bytes([1, 1, 1, 8, 10]) + bytes(3), "TCP_OPT_EIO"),     # TS truncated
        (bytes([1, 1, 1, 3]), "TCP_OPT_EIO"),                    # WS length missing
    ]


def verdict_corpus(seed: int = 7):
    """List of (name, frame bytes, expected verdict name, config overrides). Local IP = BOB, flows from flows()."""
    rng = random.Random(seed)
    pl = bytes(rng.randrange(256) for _ in range(100))
    C = []
    add = lambda name, f, v: C.append((name, f, v))  # noqa: E731
    add("ok_tcp", tcp_frame(pl), "OK_TCP")
    add("ok_tcp_odd_payload", tcp_frame(pl[:33]), "OK_TCP")
    add("ok_tcp_empty_payload", tcp_frame(b""), "OK_TCP")
    add("ok_tcp_eth_pad", tcp_frame(b"", pad=6), "OK_TCP")
    add("ok_tcp_passive", tcp_frame(pl, sport=55555), "OK_TCP")  # no Active match -> Passive listener
    add("tcp_nosock", tcp_frame(pl, dport=999), "TCP_NOSOCK")
    add("ok_udp", udp_frame(pl), "OK_UDP")
    add("ok_udp_odd", udp_frame(pl[:7]), "OK_UDP")
    add("ok_udp_csum0", udp_frame(pl, udp_kw=dict(checksum=0)), "OK_UDP")
    add("ok_udp_wildcard", udp_frame(pl, dport=7000), "OK_UDP")
    add("udp_nosock", udp_frame(pl, dport=7001), "UDP_NOSOCK")
    add("ok_udp_broadcast_csum0", udp_frame(pl, dst="255.255.255.255", udp_kw=dict(checksum=0)), "OK_UDP")
    # broadcast dst with a real checksum: the pseudo-header uses the configured local IP (udp/peer.rs:134) -> U3
    add("udp_broadcast_csum", udp_frame(pl, dst="255.255.255.255"), "UDP_CSUM")
    add("eth_short", eth_header()[:13], "ETH_SHORT")
    add("eth_empty", b"", "ETH_SHORT")
    add("eth_type", eth_header(0x1234) + bytes(40), "ETH_TYPE")
    add("arp_zero_pdu", eth_header(0x0806) + bytes(28), "ARP_UNSUP")
    add("arp_request", arp_frame(), "ARP")
    add("arp_reply", arp_frame(op=2, sha=BOB_MAC, spa=BOB_IPV4, tha=ALICE_MAC, tpa=ALICE_IPV4), "ARP")
    add("arp_padded", arp_frame(pad=18), "ARP")
    add("arp_short", arp_frame()[:14 + 27], "ARP_SHORT")
    add("arp_empty", eth_header(0x0806), "ARP_SHORT")
    add("arp_htype", arp_frame(htype=6), "ARP_UNSUP")
    add("arp_ptype", arp_frame(ptype=0x86DD), "ARP_UNSUP")
    add("arp_hlen", arp_frame(hlen=8), "ARP_UNSUP")
    add("arp_plen", arp_frame(plen=16), "ARP_UNSUP")
    add("arp_op", arp_frame(op=3), "ARP_UNSUP")
    add("arp_op0", arp_frame(op=0), "ARP_UNSUP")
    add("ipv6", eth_header(0x86DD) + bytes(40), "IPV6")
    add("ip_short", eth_header() + bytes(19), "IP_SHORT")
    add("ip_version", frame(tcp_segment(), version=6), "IP_VERSION")
    add("ip_ihl_small", frame(tcp_segment(), ihl=4), "IP_IHL_SMALL")
    add("ip_hdr_trunc", eth_header() + ipv4_header(ihl=15, total_length=60)[:24], "IP_HDR_TRUNC")
    add("ip_totlen_small", frame(tcp_segment(), total_length=19), "IP_TOTLEN_SMALL")
    add("ip_totlen_big", frame(tcp_segment(), total_length=200), "IP_TOTLEN_BIG")
    add("ip_evil", frame(tcp_segment(), flags=0x4), "IP_EVIL")
    add("ip_mf", frame(tcp_segment(), flags=0x1), "IP_MF")
    add("ip_fragoff", frame(tcp_segment(), frag=1), "IP_FRAGOFF")
    add("ip_ttl", frame(tcp_segment(), ttl=0), "IP_TTL")
    add("ip_proto", frame(tcp_segment(), proto=47), "IP_PROTO")
    add("ip_csum_ffff", frame(tcp_segment(), checksum=0xFFFF), "IP_CSUM_FFFF")
    add("ip_csum", frame(tcp_segment(), checksum=0x0001), "IP_CSUM")
    add("ip_dst", tcp_frame(pl, dst="192.168.1.3"), "IP_DST")
    add("ip_src_bcast", tcp_frame(pl, src="255.255.255.255"), "IP_SRC")
    add("ip_src_mcast", tcp_frame(pl, src="224.0.0.1"), "IP_SRC")
    add("ip_src_zero", tcp_frame(pl, src="0.0.0.0"), "IP_SRC")
    add("icmp_zero_csum", frame(bytes([8, 0, 0, 0]) + bytes(4), proto=1), "ICMP_CSUM")
    add("icmp_echo_request", icmp_frame(payload=pl[:56]), "ICMP")
    add("icmp_echo_reply", icmp_frame(0, ident=7, seq=65535, payload=pl[:56]), "ICMP")
    add("icmp_dest_unreach", icmp_frame(3, code=1, ident=0, seq=0, payload=pl[:28]), "ICMP")
    add("icmp_odd_payload", icmp_frame(payload=pl[:33]), "ICMP")
    add("icmp_header_only", icmp_frame(13), "ICMP")
    add("icmp_big", icmp_frame(payload=pl * 10), "ICMP")
    add("icmp_eth_pad", icmp_frame(payload=pl[:4], pad=10), "ICMP")
    add("icmp_ip_options", icmp_frame(payload=pl[:20], ip_options=bytes([1, 1, 1, 0])), "ICMP")
    add("icmp_short", frame(icmp_message()[:7], proto=1), "ICMP_SHORT")
    add("icmp_empty", frame(b"", proto=1), "ICMP_SHORT")
    add("icmp_csum", icmp_frame(payload=pl[:56], checksum=0x1111), "ICMP_CSUM")
    add("icmp_type_6", icmp_frame(6), "ICMP_TYPE")
    add("icmp_type_15", icmp_frame(15, payload=pl[:9]), "ICMP_TYPE")
    add("icmp_type_255", icmp_frame(255), "ICMP_TYPE")
    add("icmp_dst_not_local", icmp_frame(dst="192.168.1.3"), "IP_DST")
    add("ip_options_ok", tcp_frame(pl, ip_options=bytes([1, 1, 1, 0])), "OK_TCP")
    f = bytearray(tcp_frame(pl, ip_options=bytes([1, 1, 1, 0])))
    f[34:38] = bytes([7, 7, 7, 7])  # IPv4 options are not checksummed (ipv4/header.rs:289-296, quirk 1)
    add("ip_options_not_summed", bytes(f), "OK_TCP")
    add("tcp_short", frame(bytes(19), proto=6), "TCP_SHORT")
    add("tcp_doff_trunc", frame(tcp_segment(doff=6), proto=6), "TCP_DOFF_TRUNC")
    add("tcp_doff_small", frame(tcp_segment(doff=4), proto=6), "TCP_DOFF_SMALL")
    add("tcp_csum", tcp_frame(pl, tcp_kw=dict(checksum=0x1234)), "TCP_CSUM")
    add("tcp_csum_ffff", tcp_frame(pl, tcp_kw=dict(checksum=0xFFFF)), "TCP_CSUM")
    for k, (opts, v) in enumerate(tcp_opt_cases()):
        add(f"tcp_opt_{k}", tcp_frame(pl[:10], options=opts), v or "OK_TCP")
    add("tcp_opt_bad_csum_first", tcp_frame(pl, options=bytes([9, 2, 0, 0]), tcp_kw=dict(checksum=1)), "TCP_CSUM")
    add("udp_short", frame(bytes(7), proto=17), "UDP_SHORT")
    add("udp_len", udp_frame(pl, udp_kw=dict(length=50)), "UDP_LEN")
    add("udp_csum", udp_frame(pl, udp_kw=dict(checksum=0x4321)), "UDP_CSUM")
    return C


def corpus_flows():
    """Socket table for verdict_corpus(): Active (BOB:12345 <- ALICE:40000), Passive BOB:12345, UDP BOB:5000 and
    wildcard 0.0.0.0:7000."""
    from demikernel_amd.rx import SocketId, flow_array

    return flow_array([
        SocketId.Active((BOB_IPV4, 12345), (ALICE_IPV4, 40000)),
        SocketId.Passive((BOB_IPV4, 12345)),
        SocketId.Udp((BOB_IPV4, 5000)),
        SocketId.Udp(("0.0.0.0", 7000)),
    ])
