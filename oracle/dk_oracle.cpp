// =====================================================================================================================
// dk_oracle.cpp — TEST INFRASTRUCTURE ONLY. Not part of the product; never linked into libdk_rx.so.
//
// A CPU restatement of the Demikernel receive path (reference microsoft/demikernel @ 2024-10-24, mounted read-only at
// /root/reference; paths below are relative to src/rust/). It exists to (1) check the MI355X engine bit for bit and
// (2) be timed as the CPU baseline ("port") in bench.py. Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load it.
//
// It follows the reference function by function, keeping its check order, its scalar big-endian word loops, its
// subtraction-loop fold and its HashMap demux (std::unordered_map here). The reference is Rust and cannot be built in
// this image (no cargo/rustc), so it is pinned by the reference's own unit-test vectors (tests/golden, tests/
// test_oracle.py): IPv4 parse verdicts (layer3/ipv4/tests.rs), the UDP header KAT (layer4/udp/header.rs:206-252),
// plus the RFC 1071 known answer and serialize->parse round trips. TCP/UDP checksum values have no known-answer vector
// in the reference; they are cross-checked against an independent numpy implementation.
// =====================================================================================================================

#include "../include/dk_rx.h"

#include <cstdint>
#include <cstring>
#include <unordered_map>
#include <vector>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

// errno per verdict (EBADMSG 74, ENOTSUP 95, EIO 5) is tabulated in tests/ and in the product (dk_rx_verdict_errno).

// ---------------------------------------------------------------------------------------------------------------------
// DemiBuffer view: data pointer + length. adjust()/trim() as runtime/memory/demibuffer.rs:515-590 (fail if n > len).
// ---------------------------------------------------------------------------------------------------------------------
struct Buf {
    const uint8_t* p;
    size_t len;
    size_t off;  // bytes adjusted away from the frame start (payload offset bookkeeping)
    bool adjust(size_t n) {
        if (n > len) return false;
        p += n;
        len -= n;
        off += n;
        return true;
    }
    bool trim(size_t n) {
        if (n > len) return false;
        len -= n;
        return true;
    }
};

inline uint16_t be16(const uint8_t* b) { return (uint16_t)(((uint16_t)b[0] << 8) | b[1]); }
inline uint32_t be32(const uint8_t* b) {
    return ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
}
inline uint32_t octets_u32(const uint8_t* b) { uint32_t v; std::memcpy(&v, b, 4); return v; }  // s_addr order
inline void octets_of(uint32_t a, uint8_t o[4]) { std::memcpy(o, &a, 4); }

// protocols/mod.rs:66-71 fold16 / the identical `while state > 0xFFFF { state -= 0xFFFF }` loops.
inline uint16_t fold16(uint32_t state) {
    while (state > 0xFFFF) state -= 0xFFFF;
    return (uint16_t)~state;
}

// ---------------------------------------------------------------------------------------------------------------------
// Layer 2: Ethernet2Header::parse_and_strip (layer2/ethernet2/header.rs:50-65), EtherType2::try_from (protocol.rs:35-41)
// ---------------------------------------------------------------------------------------------------------------------
enum EtherType2 { ARP = 0x0806, IPV4 = 0x0800, IPV6 = 0x86dd };

int eth_parse_and_strip(Buf& buf, uint16_t* ether_type) {
    if (buf.len < 14) return DK_V_ETH_SHORT;                      // header.rs:51-53 "frame too small"
    uint16_t et = be16(buf.p + 12);
    if (et != ARP && et != IPV4 && et != IPV6) return DK_V_ETH_TYPE;  // protocol.rs:35-41 ENOTSUP
    buf.adjust(14);                                               // header.rs:62
    *ether_type = et;
    return -1;
}

// ---------------------------------------------------------------------------------------------------------------------
// Layer 3: Ipv4Header (layer3/ipv4/header.rs)
// ---------------------------------------------------------------------------------------------------------------------
struct Ipv4Header {
    uint8_t ihl;
    uint16_t total_length;
    uint8_t protocol;
    uint32_t src, dst;  // octet order
};

// header.rs:280-301 — only the first 20 bytes, checksum word skipped, state starts at 0xFFFF.
uint16_t ipv4_compute_checksum(const uint8_t* buf, size_t len) {
    uint32_t state = 0xffff;
    if (len < 20) return 0;  // :284-288 "should not happen by construction"
    for (int i = 0; i < 5; i++) state += be16(buf + 2 * i);
    for (int i = 6; i < 10; i++) state += be16(buf + 2 * i);
    while (state > 0xffff) state -= 0xffff;
    return (uint16_t)~state;
}

// header.rs:111-225
int ipv4_parse_and_strip(Buf& buf, Ipv4Header* out) {
    if (buf.len < 20) return DK_V_IP_SHORT;                       // :113-115
    uint8_t version = buf.p[0] >> 4;
    if (version != 4) return DK_V_IP_VERSION;                     // :117-120
    uint8_t ihl = buf.p[0] & 0xF;
    uint16_t hdr_size = (uint16_t)ihl << 2;
    if (hdr_size < 20) return DK_V_IP_IHL_SMALL;                  // :123-127
    if (buf.len < hdr_size) return DK_V_IP_HDR_TRUNC;             // :128-130
    const uint8_t* h = buf.p;
    // dscp / ecn: warn only (:134-143)
    uint16_t total_length = be16(h + 2);
    if (total_length < hdr_size) return DK_V_IP_TOTLEN_SMALL;     // :145-148
    if ((size_t)total_length > buf.len) return DK_V_IP_TOTLEN_BIG;  // :150-152
    uint8_t flags = h[6] >> 5;
    if (flags & 0x4) return DK_V_IP_EVIL;                         // :168-172
    if (flags & 0x1) return DK_V_IP_MF;                           // :175-178
    uint16_t fragment_offset = be16(h + 6) & 0x1fff;
    if (fragment_offset != 0) return DK_V_IP_FRAGOFF;             // :180-185
    if (h[8] == 0) return DK_V_IP_TTL;                            // :187-190
    uint8_t proto = h[9];
    if (proto != 0x01 && proto != 0x06 && proto != 0x11) return DK_V_IP_PROTO;  // :192, ip/protocol.rs:34-41
    uint16_t header_checksum = be16(h + 10);
    if (header_checksum == 0xffff) return DK_V_IP_CSUM_FFFF;      // :194-197
    if (header_checksum != ipv4_compute_checksum(h, hdr_size)) return DK_V_IP_CSUM;  // :198-200
    out->ihl = ihl;
    out->total_length = total_length;
    out->protocol = proto;
    out->src = octets_u32(h + 12);
    out->dst = octets_u32(h + 16);
    size_t padding_bytes = buf.len - total_length;                // :206-208
    buf.adjust(hdr_size);
    buf.trim(padding_bytes);
    return -1;
}

inline bool is_broadcast(uint32_t a) { return a == 0xFFFFFFFFu; }
inline bool is_multicast(uint32_t a) { uint8_t o[4]; octets_of(a, o); return (o[0] & 0xF0) == 224; }  // 224/4
inline bool is_unspecified(uint32_t a) { return a == 0; }

// ---------------------------------------------------------------------------------------------------------------------
// Layer 4: TCP (layer4/tcp/header.rs)
// ---------------------------------------------------------------------------------------------------------------------
struct TcpHeader {
    uint16_t src_port, dst_port;
    uint32_t seq, ack;
    uint8_t b12, b13;
    uint16_t window, urgent;
    uint32_t data_offset;
    int num_options;
    dk_tcp_opts opts;  // the option list (tcp/header.rs:212-302) in the dk_rx.h record layout
};

// tcp/header.rs:433-509, restated word for word.
uint16_t tcp_checksum(uint32_t src_ip, uint32_t dst_ip, const uint8_t* header, size_t hlen, const uint8_t* data,
                      size_t dlen) {
    uint32_t state = 0xffff;
    uint8_t s[4], d[4];
    octets_of(src_ip, s);
    octets_of(dst_ip, d);
    state += be16(s);
    state += be16(s + 2);
    state += be16(d);
    state += be16(d + 2);
    state += 0x0006;                      // [0, IpProtocol::TCP]
    state += (uint32_t)(hlen + dlen);     // segment length
    const uint8_t* f = header;
    state += be16(f + 0);
    state += be16(f + 2);
    state += be16(f + 4);
    state += be16(f + 6);
    state += be16(f + 8);
    state += be16(f + 10);
    state += be16(f + 12);
    state += be16(f + 14);
    state += 0;                           // checksum field as zero
    state += be16(f + 18);
    if (hlen > 20)                        // options: data_offset is a multiple of 4, no remainder
        for (size_t i = 20; i + 2 <= hlen; i += 2) state += be16(header + i);
    size_t i = 0;
    for (; i + 2 <= dlen; i += 2) state += be16(data + i);
    if (i < dlen) state += (uint32_t)data[i] << 8;  // remainder [b, 0]
    while (state > 0xFFFF) state -= 0xFFFF;
    return (uint16_t)~state;
}

// std::io::Cursor::read_exact semantics over hdr_buf[20..data_offset]: fail (-> EIO) when short.
struct Cursor {
    const uint8_t* p;
    size_t len, pos;
    bool read_exact(uint8_t* out, size_t n) {
        if (len - pos < n) { pos = len; return false; }  // io::ErrorKind::UnexpectedEof
        std::memcpy(out, p + pos, n);
        pos += n;
        return true;
    }
};

// tcp/header.rs:162-327 (local_ipv4_addr/remote_ipv4_addr are passed as tcp/peer.rs:223-228 passes them).
int tcp_parse_and_strip(uint32_t local_ipv4_addr, uint32_t remote_ipv4_addr, Buf& buf, bool rx_checksum_offload,
                        TcpHeader* out) {
    if (buf.len < 20) return DK_V_TCP_SHORT;                          // :168-170
    size_t data_offset = (size_t)(buf.p[12] >> 4) * 4;
    if (buf.len < data_offset) return DK_V_TCP_DOFF_TRUNC;            // :171-174
    if (data_offset < 20) return DK_V_TCP_DOFF_SMALL;                 // :175-177
    if (data_offset > 60) return DK_V_TCP_DOFF_SMALL;                 // :178-180 (unreachable: 4-bit field)
    const uint8_t* hdr = buf.p;
    const uint8_t* data = buf.p + data_offset;
    size_t dlen = buf.len - data_offset;
    out->src_port = be16(hdr + 0);
    out->dst_port = be16(hdr + 2);
    out->seq = be32(hdr + 4);
    out->ack = be32(hdr + 8);
    out->b12 = hdr[12];
    out->b13 = hdr[13];
    out->window = be16(hdr + 14);
    if (!rx_checksum_offload) {                                       // :203-207
        uint16_t checksum = be16(hdr + 16);
        if (checksum != tcp_checksum(local_ipv4_addr, remote_ipv4_addr, hdr, data_offset, data, dlen))
            return DK_V_TCP_CSUM;
    }
    out->urgent = be16(hdr + 18);
    int num_options = 0;
    std::memset(&out->opts, 0, sizeof out->opts);
    uint32_t nsack = 0;
    if (data_offset > 20) {                                           // :215-302
        Cursor rdr{hdr + 20, data_offset - 20, 0};
        while (rdr.pos < data_offset - 20) {
            uint8_t kind;
            if (!rdr.read_exact(&kind, 1)) return DK_V_TCP_OPT_EIO;
            uint8_t t1, t2[2], t4[4];
            dk_tcp_opt e{kind, 0, 0, 0, 0};
            switch (kind) {
                case 0: goto done;                                    // EndOfOptionsList: break
                case 1: continue;                                     // NoOperation: not counted
                case 2:                                               // MaximumSegmentSize(mss)
                    if (!rdr.read_exact(&t1, 1)) return DK_V_TCP_OPT_EIO;
                    if (t1 != 4) return DK_V_TCP_OPT;
                    if (!rdr.read_exact(t2, 2)) return DK_V_TCP_OPT_EIO;
                    e.u16 = be16(t2);
                    break;
                case 3:                                               // WindowScale(scale)
                    if (!rdr.read_exact(&t1, 1)) return DK_V_TCP_OPT_EIO;
                    if (t1 != 3) return DK_V_TCP_OPT;
                    if (!rdr.read_exact(&t1, 1)) return DK_V_TCP_OPT_EIO;
                    e.u8 = t1;
                    break;
                case 4:                                               // SelectiveAcknowlegementPermitted
                    if (!rdr.read_exact(&t1, 1)) return DK_V_TCP_OPT_EIO;
                    if (t1 != 2) return DK_V_TCP_OPT;
                    break;
                case 5: {                                             // SelectiveAcknowlegement
                    if (!rdr.read_exact(&t1, 1)) return DK_V_TCP_OPT_EIO;
                    size_t num_sacks;
                    switch (t1) {
                        case 10: case 18: case 26: case 34: num_sacks = ((size_t)t1 - 2) / 8; break;
                        default: return DK_V_TCP_OPT;
                    }
                    e.u8 = (uint8_t)num_sacks;
                    e.u16 = (uint16_t)nsack;
                    for (size_t k = 0; k < num_sacks; k++) {
                        uint8_t b4[4];
                        if (!rdr.read_exact(t4, 4)) return DK_V_TCP_OPT_EIO;
                        if (!rdr.read_exact(b4, 4)) return DK_V_TCP_OPT_EIO;
                        if (nsack < 4) {
                            out->opts.sack[nsack][0] = be32(t4);
                            out->opts.sack[nsack][1] = be32(b4);
                            nsack++;
                        }
                    }
                    break;
                }
                case 8: {                                             // Timestamp
                    if (!rdr.read_exact(&t1, 1)) return DK_V_TCP_OPT_EIO;
                    if (t1 != 10) return DK_V_TCP_OPT;
                    uint8_t b4[4];
                    if (!rdr.read_exact(t4, 4)) return DK_V_TCP_OPT_EIO;
                    if (!rdr.read_exact(b4, 4)) return DK_V_TCP_OPT_EIO;
                    e.v0 = be32(t4);
                    e.v1 = be32(b4);
                    break;
                }
                default: return DK_V_TCP_OPT;                         // "invalid TCP option"
            }
            if (num_options >= 5) return DK_V_TCP_OPT;                // "too many TCP options provided"
            out->opts.opt[num_options] = e;                           // option_list[num_options] = option
            num_options++;
        }
    }
done:
    out->num_options = num_options;
    out->opts.num = (uint32_t)num_options;
    out->data_offset = (uint32_t)data_offset;
    buf.adjust(data_offset);                                          // :306-307
    return -1;
}

// ---------------------------------------------------------------------------------------------------------------------
// Layer 4: UDP (layer4/udp/header.rs)
// ---------------------------------------------------------------------------------------------------------------------
// udp/header.rs:140-193
uint16_t udp_checksum(uint32_t src_ip, uint32_t dst_ip, const uint8_t* udp_hdr, const uint8_t* data, size_t dlen) {
    uint32_t state = 0xffff;
    uint8_t s[4], d[4];
    octets_of(src_ip, s);
    octets_of(dst_ip, d);
    state += be16(s);
    state += be16(s + 2);
    state += be16(d);
    state += be16(d + 2);
    state += 0x0011;                      // [0, IpProtocol::UDP]
    state += (uint32_t)(8 + dlen);        // UDP segment length
    state += be16(udp_hdr + 0);
    state += be16(udp_hdr + 2);
    state += be16(udp_hdr + 4);
    state += 0;                           // checksum field as zero
    size_t i = 0;
    for (; i + 2 <= dlen; i += 2) state += be16(data + i);
    if (i < dlen) state += (uint32_t)data[i] << 8;
    while (state > 0xFFFF) state -= 0xFFFF;
    return (uint16_t)~state;
}

struct UdpHeader { uint16_t src_port, dst_port; };

// udp/header.rs:57-94
int udp_parse_and_strip(uint32_t src_ipv4_addr, uint32_t dst_ipv4_addr, Buf& buf, bool checksum_offload,
                        UdpHeader* out) {
    if (buf.len < 8) return DK_V_UDP_SHORT;                           // :64-66
    const uint8_t* hdr = buf.p;
    out->src_port = be16(hdr);
    out->dst_port = be16(hdr + 2);
    size_t length = be16(hdr + 4);
    if (length != buf.len) return DK_V_UDP_LEN;                       // :72-75
    if (!checksum_offload) {                                          // :78-88
        uint16_t checksum = be16(hdr + 6);
        if (checksum != 0)
            if (checksum != udp_checksum(src_ipv4_addr, dst_ipv4_addr, hdr, hdr + 8, buf.len - 8))
                return DK_V_UDP_CSUM;
    }
    buf.adjust(8);
    return -1;
}

// ---------------------------------------------------------------------------------------------------------------------
// Diverted control-plane frames: the parse the ARP / ICMPv4 peers run on what layer 3 hands
// them (arp/peer.rs:140-147, icmpv4/peer.rs:114-121).
// ---------------------------------------------------------------------------------------------------------------------
// protocols/mod.rs:47-64 compute_generic_checksum: BE words, odd tail [b, 0], state seeded with 0xFFFF unless given.
uint32_t compute_generic_checksum(const uint8_t* buf, size_t len, const uint32_t* start) {
    uint32_t state = start ? *start : 0xFFFF;
    size_t i = 0;
    for (; i + 2 <= len; i += 2) state += be16(buf + i);
    if (i < len) state += (uint32_t)buf[i] << 8;
    return state;
}

struct Icmpv4Header { uint8_t type, code; uint16_t id, seq; };

// icmpv4/header.rs:47-66 parse_and_strip; Icmpv4Type2::parse (icmpv4/protocol.rs:35-58).
int icmpv4_parse_and_strip(Buf& buf, Icmpv4Header* out) {
    if (buf.len < 8) return DK_V_ICMP_SHORT;                            // :48-50
    const uint8_t* hdr = buf.p;
    // compute_checksum (:88-93): generic sum of the 8-byte header (checksum field included) then of the body
    uint32_t state = compute_generic_checksum(hdr, 8, nullptr);
    state = compute_generic_checksum(hdr + 8, buf.len - 8, &state);
    if (fold16(state) != 0) return DK_V_ICMP_CSUM;                      // :55-57
    switch (hdr[0]) {                                                   // protocol.rs:37-56
        case 0: case 3: case 4: case 5: case 8: case 9: case 10: case 11: case 12: case 13: case 14: break;
        default: return DK_V_ICMP_TYPE;                                 // "invalid type byte"
    }
    out->type = hdr[0];
    out->code = hdr[1];
    out->id = be16(hdr + 4);
    out->seq = be16(hdr + 6);
    buf.adjust(8);                                                      // :61
    return -1;
}

struct ArpHeader { uint16_t op; uint32_t sender_ip, target_ip; };

// arp/header.rs:80-111 parse_and_consume; ArpOperation::try_from (:161-166).
int arp_parse_and_consume(const Buf& buf, ArpHeader* out) {
    if (buf.len < 28) return DK_V_ARP_SHORT;                            // :81-83
    const uint8_t* b = buf.p;
    if (be16(b) != 1) return DK_V_ARP_UNSUP;                            // HTYPE Ethernet2 (:85-88)
    if (be16(b + 2) != 0x0800) return DK_V_ARP_UNSUP;                   // PTYPE IPv4 (:89-92)
    if (b[4] != 6) return DK_V_ARP_UNSUP;                               // HLEN (:93-96)
    if (b[5] != 4) return DK_V_ARP_UNSUP;                               // PLEN (:97-100)
    uint16_t op = be16(b + 6);
    if (op != 1 && op != 2) return DK_V_ARP_UNSUP;                      // Request / Reply only (:161-166)
    out->op = op;
    out->sender_ip = octets_u32(b + 14);
    out->target_ip = octets_u32(b + 24);
    return -1;
}

// ---------------------------------------------------------------------------------------------------------------------
// Demux tables: HashMap<SocketId, SharedTcpSocket> (tcp/peer.rs) and HashMap<SocketAddrV4, SharedUdpSocket>
// (udp/peer.rs:38). The hash function is irrelevant to results; lookup order is what matters.
// ---------------------------------------------------------------------------------------------------------------------
struct Key {
    uint32_t kind, lip, rip;
    uint16_t lport, rport;
    bool operator==(const Key& o) const {
        return kind == o.kind && lip == o.lip && rip == o.rip && lport == o.lport && rport == o.rport;
    }
};
struct KeyHash {
    size_t operator()(const Key& k) const {
        uint64_t h = k.kind * 0x9E3779B97F4A7C15ull;
        h ^= k.lip + 0x632BE59BD9B4E019ull + (h << 6) + (h >> 2);
        h ^= k.rip + 0x8CB92BA72F3D8DD7ull + (h << 6) + (h >> 2);
        h ^= ((uint64_t)k.lport << 16 | k.rport) + (h << 6) + (h >> 2);
        return (size_t)h;
    }
};

}  // namespace

struct dko_peer {
    uint32_t local_ipv4;
    bool tcp_offload, udp_offload;
    std::unordered_map<Key, uint32_t, KeyHash> tcp;  // SocketId -> flow id
    std::unordered_map<Key, uint32_t, KeyHash> udp;  // SocketAddrV4 -> flow id
    uint32_t nflows;
};

namespace {

// The whole per-frame chain: layer2/mod.rs:56-79 -> layer3/mod.rs:71-120 -> layer4/mod.rs:97-107 ->
// tcp/peer.rs:220-255 | udp/peer.rs:129-168. Writes the dk_rx.h result record for frame i.
void receive_one(const dko_peer& peer, const uint8_t* frame, size_t len, uint32_t* meta, uint32_t* src, uint32_t* dst,
                 uint32_t* ports, uint32_t* payload, uint32_t* flow, uint32_t* seq, uint32_t* ack, uint32_t* win,
                 dk_tcp_opts* opts) {
    *meta = 0; *src = 0; *dst = 0; *ports = 0; *payload = 0; *flow = DK_FLOW_NONE; *seq = 0; *ack = 0; *win = 0;
    Buf buf{frame, len, 0};
    uint16_t et;
    int v = eth_parse_and_strip(buf, &et);
    if (v >= 0) { *meta = (uint32_t)v; return; }
    // dst MAC mismatch is warn-only (layer2/mod.rs:69-75): no verdict.
    if (et == ARP) {                                                // layer3/mod.rs:75-78 -> arp/peer.rs:140
        ArpHeader ah;
        v = arp_parse_and_consume(buf, &ah);
        if (v >= 0) { *meta = (uint32_t)v; return; }
        *meta = DK_V_ARP | (uint32_t)ah.op << 16;
        *src = ah.sender_ip; *dst = ah.target_ip;
        *payload = (uint32_t)buf.off | (uint32_t)buf.len << 16;
        return;
    }
    if (et == IPV6) { *meta = DK_V_IPV6; return; }                 // layer3/mod.rs:116
    Ipv4Header ip;
    v = ipv4_parse_and_strip(buf, &ip);
    if (v >= 0) { *meta = (uint32_t)v; return; }
    if (ip.dst != peer.local_ipv4 && !is_broadcast(ip.dst)) { *meta = DK_V_IP_DST; return; }   // :91-95
    if (is_broadcast(ip.src) || is_multicast(ip.src) || is_unspecified(ip.src)) { *meta = DK_V_IP_SRC; return; }
    if (ip.protocol == 0x01) {                                     // :109-112 -> icmpv4/peer.rs:114
        Icmpv4Header ih;
        v = icmpv4_parse_and_strip(buf, &ih);
        if (v >= 0) { *meta = (uint32_t)v; return; }
        *meta = DK_V_ICMP | 0x01u << 8 | (uint32_t)ih.type << 16 | (uint32_t)ih.code << 24;
        *src = ip.src; *dst = ip.dst;
        *ports = (uint32_t)ih.id | (uint32_t)ih.seq << 16;
        *payload = (uint32_t)buf.off | (uint32_t)buf.len << 16;
        return;
    }
    if (ip.protocol == 0x06) {
        // TcpPeer::receive (tcp/peer.rs:220-255): parse_and_strip(&src_ipv4_addr, &self.local_ipv4_addr, ...)
        TcpHeader th;
        v = tcp_parse_and_strip(ip.src, peer.local_ipv4, buf, peer.tcp_offload, &th);
        if (v >= 0) { *meta = (uint32_t)v; return; }
        uint32_t fid = DK_FLOW_NONE;
        Key active{DK_FLOW_TCP_ACTIVE, peer.local_ipv4, ip.src, th.dst_port, th.src_port};
        auto it = peer.tcp.find(active);
        if (it != peer.tcp.end()) fid = it->second;
        else {
            Key passive{DK_FLOW_TCP_PASSIVE, peer.local_ipv4, 0, th.dst_port, 0};
            auto it2 = peer.tcp.find(passive);
            if (it2 != peer.tcp.end()) fid = it2->second;
        }
        v = fid == DK_FLOW_NONE ? DK_V_TCP_NOSOCK : DK_V_OK_TCP;
        *meta = (uint32_t)v | 0x06u << 8 | (uint32_t)th.b13 << 16 | (uint32_t)th.b12 << 24;
        *src = ip.src; *dst = ip.dst;
        *ports = (uint32_t)th.src_port | (uint32_t)th.dst_port << 16;
        *payload = (uint32_t)buf.off | (uint32_t)buf.len << 16;
        *flow = fid;
        *seq = th.seq; *ack = th.ack; *win = (uint32_t)th.window | (uint32_t)th.urgent << 16;
        if (opts && th.data_offset > 20) *opts = th.opts;  // option-bearing segment (dk_rx.h tcp_opts)
        return;
    }
    // UdpPeer::receive (udp/peer.rs:129-168): parse_and_strip(&src_ipv4_addr, &self.local_ipv4_addr, ...)
    UdpHeader uh;
    v = udp_parse_and_strip(ip.src, peer.local_ipv4, buf, peer.udp_offload, &uh);
    if (v >= 0) { *meta = (uint32_t)v; return; }
    uint32_t fid = DK_FLOW_NONE;
    Key local{DK_FLOW_UDP, peer.local_ipv4, 0, uh.dst_port, 0};
    auto it = peer.udp.find(local);
    if (it != peer.udp.end()) fid = it->second;
    else {
        Key wildcard{DK_FLOW_UDP, 0, 0, uh.dst_port, 0};              // Ipv4Addr::UNSPECIFIED
        auto it2 = peer.udp.find(wildcard);
        if (it2 != peer.udp.end()) fid = it2->second;
    }
    v = fid == DK_FLOW_NONE ? DK_V_UDP_NOSOCK : DK_V_OK_UDP;
    *meta = (uint32_t)v | 0x11u << 8;
    *src = ip.src; *dst = ip.dst;
    *ports = (uint32_t)uh.src_port | (uint32_t)uh.dst_port << 16;
    *payload = (uint32_t)buf.off | (uint32_t)buf.len << 16;
    *flow = fid;
}

}  // namespace

// =====================================================================================================================
// C ABI for ctypes (tests / bench cpu_baseline).
// =====================================================================================================================
extern "C" {

dko_peer* dko_peer_new(uint32_t local_ipv4, int tcp_offload, int udp_offload) {
    dko_peer* p = new dko_peer();
    p->local_ipv4 = local_ipv4;
    p->tcp_offload = tcp_offload != 0;
    p->udp_offload = udp_offload != 0;
    p->nflows = 0;
    return p;
}

void dko_peer_free(dko_peer* p) { delete p; }

// Socket table: HashMap::insert semantics (last duplicate wins). Returns 0 or EINVAL.
int dko_peer_set_flows(dko_peer* p, const dk_flow* flows, uint32_t n) {
    p->tcp.clear();
    p->udp.clear();
    for (uint32_t i = 0; i < n; i++) {
        const dk_flow& f = flows[i];
        if (f.kind == DK_FLOW_TCP_ACTIVE) p->tcp[Key{f.kind, f.local_ip, f.remote_ip, f.local_port, f.remote_port}] = i;
        else if (f.kind == DK_FLOW_TCP_PASSIVE) p->tcp[Key{f.kind, f.local_ip, 0, f.local_port, 0}] = i;
        else if (f.kind == DK_FLOW_UDP) p->udp[Key{f.kind, f.local_ip, 0, f.local_port, 0}] = i;
        else return 22;
    }
    p->nflows = n;
    return 0;
}

// Process frames [begin, end) of a host batch. Result arrays are full-length [n]; optional ones may be NULL.
static void dko_range(const dko_peer* p, const uint8_t* frames, uint64_t frames_bytes, const uint32_t* off,
                      const uint16_t* len, uint32_t begin, uint32_t end, uint32_t* meta, uint32_t* src, uint32_t* dst,
                      uint32_t* ports, uint32_t* payload, uint32_t* flow, uint32_t* seq, uint32_t* ack, uint32_t* win,
                      uint64_t* flow_counts, uint64_t* verdict_counts, dk_tcp_opts* opts) {
    for (uint32_t i = begin; i < end; i++) {
        uint32_t s_, a_, w_;
        if ((uint64_t)off[i] + len[i] > frames_bytes) {
            meta[i] = DK_V_BAD_DESC; src[i] = dst[i] = ports[i] = payload[i] = 0; flow[i] = DK_FLOW_NONE;
            s_ = a_ = w_ = 0;
        } else {
            receive_one(*p, frames + off[i], len[i], &meta[i], &src[i], &dst[i], &ports[i], &payload[i], &flow[i],
                        &s_, &a_, &w_, opts ? opts + i : nullptr);
        }
        if (seq) seq[i] = s_;
        if (ack) ack[i] = a_;
        if (win) win[i] = w_;
        if (verdict_counts) verdict_counts[meta[i] & 0xFF]++;
        if (flow_counts && flow[i] != DK_FLOW_NONE && ((meta[i] & 0xFF) <= DK_V_OK_UDP)) flow_counts[flow[i]]++;
    }
}

void dko_process(const dko_peer* p, const uint8_t* frames, uint64_t frames_bytes, const uint32_t* off,
                 const uint16_t* len, uint32_t n, uint32_t* meta, uint32_t* src, uint32_t* dst, uint32_t* ports,
                 uint32_t* payload, uint32_t* flow, uint32_t* seq, uint32_t* ack, uint32_t* win,
                 uint64_t* flow_counts, uint64_t* verdict_counts, dk_tcp_opts* opts) {
    dko_range(p, frames, frames_bytes, off, len, 0, n, meta, src, dst, ports, payload, flow, seq, ack, win,
              flow_counts, verdict_counts, opts);
}

// Scaled CPU baseline: packet shards over `threads` OpenMP threads (counts merged after the loop). Returns the
// number of threads actually used.
int dko_process_mt(const dko_peer* p, const uint8_t* frames, uint64_t frames_bytes, const uint32_t* off,
                   const uint16_t* len, uint32_t n, uint32_t* meta, uint32_t* src, uint32_t* dst, uint32_t* ports,
                   uint32_t* payload, uint32_t* flow, int threads) {
#ifdef _OPENMP
    int used = 1;
#pragma omp parallel num_threads(threads)
    {
        int t = omp_get_thread_num(), nt = omp_get_num_threads();
#pragma omp single
        used = nt;
        uint32_t b = (uint32_t)((uint64_t)n * t / nt), e = (uint32_t)((uint64_t)n * (t + 1) / nt);
        dko_range(p, frames, frames_bytes, off, len, b, e, meta, src, dst, ports, payload, flow, nullptr, nullptr,
                  nullptr, nullptr, nullptr, nullptr);
    }
    return used;
#else
    (void)threads;
    dko_range(p, frames, frames_bytes, off, len, 0, n, meta, src, dst, ports, payload, flow, nullptr, nullptr, nullptr,
              nullptr, nullptr, nullptr);
    return 1;
#endif
}

// Whole-batch parity checker for full-size GPU tests: every output dko_process writes (all nine result arrays, the
// option records and both counter arrays), over `threads` OpenMP threads on contiguous frame ranges. Counters are
// accumulated per thread and added after the loop (the same counting rule as dko_range). Returns the threads used.
int dko_process_par(const dko_peer* p, const uint8_t* frames, uint64_t frames_bytes, const uint32_t* off,
                    const uint16_t* len, uint32_t n, uint32_t* meta, uint32_t* src, uint32_t* dst, uint32_t* ports,
                    uint32_t* payload, uint32_t* flow, uint32_t* seq, uint32_t* ack, uint32_t* win,
                    uint64_t* flow_counts, uint64_t* verdict_counts, dk_tcp_opts* opts, int threads) {
    const uint32_t nf = p->nflows ? p->nflows : 1;
    int used = 1;
#ifdef _OPENMP
#pragma omp parallel num_threads(threads > 0 ? threads : 1)
    {
        const int t = omp_get_thread_num(), nt = omp_get_num_threads();
#pragma omp single
        used = nt;
        std::vector<uint64_t> fc(nf, 0), vc(DK_V_COUNT, 0);
        const uint32_t b = (uint32_t)((uint64_t)n * t / nt), e = (uint32_t)((uint64_t)n * (t + 1) / nt);
        dko_range(p, frames, frames_bytes, off, len, b, e, meta, src, dst, ports, payload, flow, seq, ack, win,
                  fc.data(), vc.data(), opts);
#pragma omp critical
        {
            for (uint32_t i = 0; i < nf; i++) flow_counts[i] += fc[i];
            for (uint32_t i = 0; i < DK_V_COUNT; i++) verdict_counts[i] += vc[i];
        }
    }
#else
    (void)threads;
    dko_range(p, frames, frames_bytes, off, len, 0, n, meta, src, dst, ports, payload, flow, seq, ack, win,
              flow_counts, verdict_counts, opts);
#endif
    return used;
}

// ---- per-layer entry points, so the reference's unit tests can be restated layer by layer -----------------------
// Ipv4Header::parse_and_strip on a bare datagram: returns -1 on success (payload window in *poff/*plen) or a verdict.
int dko_ipv4_parse(const uint8_t* dgram, size_t len, uint32_t* src, uint32_t* dst, uint8_t* proto, uint32_t* poff,
                   uint32_t* plen) {
    Buf b{dgram, len, 0};
    Ipv4Header h;
    int v = ipv4_parse_and_strip(b, &h);
    if (v >= 0) return v;
    *src = h.src; *dst = h.dst; *proto = h.protocol; *poff = (uint32_t)b.off; *plen = (uint32_t)b.len;
    return -1;
}

// UdpHeader::parse_and_strip on a bare segment.
int dko_udp_parse(uint32_t src_ip, uint32_t dst_ip, const uint8_t* seg, size_t len, int offload, uint16_t* sport,
                  uint16_t* dport, uint32_t* plen) {
    Buf b{seg, len, 0};
    UdpHeader h;
    int v = udp_parse_and_strip(src_ip, dst_ip, b, offload != 0, &h);
    if (v >= 0) return v;
    *sport = h.src_port; *dport = h.dst_port; *plen = (uint32_t)b.len;
    return -1;
}

// TcpHeader::parse_and_strip on a bare segment; returns -1 or a verdict, options count in *nopt.
int dko_tcp_parse(uint32_t local_ip, uint32_t remote_ip, const uint8_t* seg, size_t len, int offload, int* nopt,
                  uint32_t* plen) {
    Buf b{seg, len, 0};
    TcpHeader h;
    int v = tcp_parse_and_strip(local_ip, remote_ip, b, offload != 0, &h);
    if (v >= 0) return v;
    *nopt = h.num_options; *plen = (uint32_t)b.len;
    return -1;
}

// Checksum primitives (the reference's own functions, restated).
uint16_t dko_ipv4_checksum(const uint8_t* hdr, size_t len) { return ipv4_compute_checksum(hdr, len); }
uint16_t dko_tcp_checksum(uint32_t src, uint32_t dst, const uint8_t* hdr, size_t hlen, const uint8_t* data,
                          size_t dlen) {
    return tcp_checksum(src, dst, hdr, hlen, data, dlen);
}
uint16_t dko_udp_checksum(uint32_t src, uint32_t dst, const uint8_t* hdr8, const uint8_t* data, size_t dlen) {
    return udp_checksum(src, dst, hdr8, data, dlen);
}
// compute_generic_checksum + fold16 (protocols/mod.rs:47-71): start = 0xFFFF unless `has_start`.
uint16_t dko_generic_checksum(const uint8_t* buf, size_t len, int has_start, uint32_t start) {
    uint32_t state = has_start ? start : 0xFFFF;
    size_t i = 0;
    for (; i + 2 <= len; i += 2) state += be16(buf + i);
    if (i < len) state += (uint32_t)buf[i] << 8;
    return fold16(state);
}

// serialize_and_attach restatement (TX, offload off): fill the IPv4 header checksum and the TCP/UDP checksum of a full
// Ethernet frame in place, using the frame's own src/dst (ipv4/header.rs:229-266, tcp/header.rs:397-404,
// udp/header.rs:97-130). Returns bit 0 = the IPv4 checksum was written, bit 1 = the L4 checksum was written (at *l4_at).
static int tx_fill(uint8_t* f, size_t len, size_t* l4_at) {
    if (len < 34 || be16(f + 12) != IPV4) return 0;
    uint8_t* ip = f + 14;
    size_t ihl = (size_t)(ip[0] & 0xF) * 4;
    size_t tot = be16(ip + 2);
    if (ihl < 20 || 14 + tot > len || tot < ihl) return 0;
    ip[10] = ip[11] = 0;
    uint16_t c = ipv4_compute_checksum(ip, ihl);
    ip[10] = (uint8_t)(c >> 8); ip[11] = (uint8_t)c;
    uint32_t src = octets_u32(ip + 12), dst = octets_u32(ip + 16);
    uint8_t* l4 = ip + ihl;
    size_t seg = tot - ihl;
    if (ip[9] == 0x06) {
        if (seg < 20) return 1;
        size_t doff = (size_t)(l4[12] >> 4) * 4;
        if (doff < 20 || doff > seg) return 1;
        l4[16] = l4[17] = 0;
        c = tcp_checksum(src, dst, l4, doff, l4 + doff, seg - doff);
        l4[16] = (uint8_t)(c >> 8); l4[17] = (uint8_t)c;
        *l4_at = 14 + ihl + 16;
        return 3;
    }
    if (ip[9] == 0x11) {
        if (seg < 8) return 1;
        l4[6] = l4[7] = 0;
        c = udp_checksum(src, dst, l4, l4 + 8, seg - 8);
        l4[6] = (uint8_t)(c >> 8); l4[7] = (uint8_t)c;
        *l4_at = 14 + ihl + 6;
        return 3;
    }
    return 1;
}

// Returns 0, or -1 if the frame is not Eth/IPv4/{TCP,UDP} with a consistent length.
int dko_tx_fill_checksums(uint8_t* f, size_t len) {
    size_t at = 0;
    return tx_fill(f, len, &at) == 3 ? 0 : -1;
}

// The same checksums as dk_tx_checksum_fields reports them (include/dk_rx.h): ipv4 | l4 << 16, 0xFFFF for a field the
// in-place fill leaves untouched; the frame itself is not modified.
uint32_t dko_tx_checksum_fields(const uint8_t* f, size_t len) {
    std::vector<uint8_t> g(f, f + len);
    size_t at = 0;
    const int m = tx_fill(g.data(), len, &at);
    const uint32_t ip = (m & 1) ? be16(g.data() + 24) : 0xFFFFu;
    const uint32_t l4 = (m & 2) ? be16(g.data() + at) : 0xFFFFu;
    return ip | l4 << 16;
}

}  // extern "C"
