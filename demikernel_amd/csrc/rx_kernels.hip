// rx_kernels.hip — CDNA4 (gfx950) kernels for the Demikernel receive-path transform.
//
// One kernel, dk_rx_kernel, does for a whole batch what the reference does frame by frame in
//   Ethernet2Header::parse_and_strip  (src/rust/inetstack/protocols/layer2/ethernet2/header.rs:50-65)
//   Ipv4Header::parse_and_strip       (layer3/ipv4/header.rs:111-225, compute_checksum :280-301)
//   SharedLayer3Endpoint::receive     (layer3/mod.rs:71-120: dst/src filters, ICMP/ARP diversion)
//   TcpHeader::parse_and_strip        (layer4/tcp/header.rs:162-327, tcp_checksum :433-509)
//   UdpHeader::parse_and_strip        (layer4/udp/header.rs:57-94, checksum :140-193)
//   TcpPeer::receive / UdpPeer::receive demux (layer4/tcp/peer.rs:220-255, layer4/udp/peer.rs:129-168)
//
// Work decomposition (persistent grid; one 256-thread workgroup = 4 waves processes 256-frame tiles):
//   Phase A, lane per frame: descriptor; frames of <= 64 bytes load straight into registers (4 x dwordx4).
//   Phase B, quarter-wave per frame: every frame of > 64 bytes is streamed once, whole, by 16 lanes (6 x dwordx4 in
//     flight per lane, 1.5 KB per quarter per round, 4 frames per wave per round); its blocks are summed, its header
//     window and last 32 bytes are deposited in LDS for the owning lane, and the quarter's sum is reduced with 4
//     lane shuffles.
//   Phase C, lane per frame: parse every header field from registers in Appendix A order (IPv4 header checksum
//     included), close the L4 one's-complement sum (pseudo-header, stored field removed), T4/U3 verdicts, TCP option
//     walk (T5, byte loads: only option-bearing segments), hash-table demux, SoA result stores, counters.
// Frames whose start is not 16-byte aligned, or whose IPv4 IHL != 5, are parsed and summed by a per-lane byte-load
// path that implements the same checks.
//
// Checksum arithmetic: the reference sums big-endian 16-bit words into a u32 seeded with
// 0xFFFF and folds by repeated subtraction of 0xFFFF. We sum little-endian 16-bit halves of dwords with
// v_dot2_u32_u16 (x . {1,1}), in any order and grouping (the true integer sum, < 2^31 for 64 KiB), reduce mod 0xFFFF,
// byte-swap (sum_BE == 256 * sum_LE mod 0xFFFF), add the pseudo-header and map the residue back to the reference's
// result (0 -> 0, m -> 0xFFFF - m). Bit-exactness against the CPU restatement is tested, not assumed.
#include <hip/hip_runtime.h>

#include "rx_common.h"
#include "rx_diag.h"

namespace dk {
namespace {

constexpr uint32_t kNone = 0xFFu;      // not yet decided
constexpr uint32_t kPendTcp = 0xF0u;   // TCP header parsed; awaiting T4/T5/demux
constexpr uint32_t kPendUdp = 0xF1u;   // UDP header parsed; awaiting U3/demux
constexpr uint32_t kPendIcmp = 0xF2u;  // ICMPv4 message >= 8 bytes; awaiting its checksum and type checks
// ICMPv4 type bytes Icmpv4Type2::parse accepts (icmpv4/protocol.rs:37-56): 0, 3, 4, 5, 8 .. 14.
constexpr uint32_t kIcmpTypes = (1u << 0) | (1u << 3) | (1u << 4) | (1u << 5) | (0x7Fu << 8);
// Tuning knobs (compile-time; defaults are the measured best, see DESIGN.md "Tuning log").
#ifndef DK_COOP_U
#define DK_COOP_U 6
#endif
#ifndef DK_HDR_TEMPORAL_U
#define DK_HDR_TEMPORAL_U 1  // loads u < this of a frame's first iteration take the default policy (kHdrT)
#endif
#ifndef DK_HDR_TEMPORAL
#define DK_HDR_TEMPORAL 0  // 1: the receive kernels too load each frame's first 256 bytes with the default policy
#endif
#ifndef DK_NT_LOADS
#define DK_NT_LOADS 1
#endif
#ifndef DK_MIN_WAVES
#define DK_MIN_WAVES 4  // waves per SIMD the register budget must admit (128 VGPRs)
#endif
constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
static_assert(kWaves == (int)kStagedWaves, "the host computes the dynamic tail's boundary with kStagedWaves");
constexpr uint32_t kCoopU = DK_COOP_U; // dwordx4 loads per lane per phase-B round
constexpr uint32_t kCoopSpan = 16 * kCoopU;  // 16-byte blocks one quarter-wave covers per round
#ifndef DK_ROUNDS_PER_STEP
#define DK_ROUNDS_PER_STEP 2
#endif
constexpr uint32_t kRoundsPerStep = DK_ROUNDS_PER_STEP;  // phase-B rounds whose loads are in flight together
// The result-staging kernel (mixed sizes, IMIX) streams one round of large frames per step: half the load registers
// for twice the steps, which pays for 9 staged chunks (round 3).
#ifndef DK_ROUNDS_STAGED
#define DK_ROUNDS_STAGED 1
#endif
constexpr uint32_t kRoundsStaged = DK_ROUNDS_STAGED;

typedef unsigned short us2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t hsum2(uint32_t x, uint32_t acc) {  // acc + lo16(x) + hi16(x)
    const us2 one = {1, 1};
    return __builtin_amdgcn_udot2(__builtin_bit_cast(us2, x), one, acc, false);
}
__device__ __forceinline__ uint32_t block_sum(const uint4& b, uint32_t acc) {
    acc = hsum2(b.x, acc);
    acc = hsum2(b.y, acc);
    acc = hsum2(b.z, acc);
    return hsum2(b.w, acc);
}
// Mask of bytes [l, h) of one dword, 0 <= l, h <= 4 (empty when h <= l).
__device__ __forceinline__ uint32_t bytes_mask(int l, int h) {
    const uint32_t mh = h >= 4 ? 0xFFFFFFFFu : ((1u << (8 * h)) - 1u);
    const uint32_t ml = l >= 4 ? 0xFFFFFFFFu : ((1u << (8 * l)) - 1u);
    return mh & ~ml;
}
__device__ __forceinline__ int clamp4(int x) { return min(max(x, 0), 4); }
// Sum of the LE halves of bytes [lo, hi) of a 16-byte block given as 4 dwords (lo even; bytes outside zeroed).
__device__ __forceinline__ uint32_t block_sum_masked(uint32_t a, uint32_t b, uint32_t c, uint32_t d, int lo, int hi,
                                                     uint32_t acc) {
    acc = hsum2(a & bytes_mask(clamp4(lo), clamp4(hi)), acc);
    acc = hsum2(b & bytes_mask(clamp4(lo - 4), clamp4(hi - 4)), acc);
    acc = hsum2(c & bytes_mask(clamp4(lo - 8), clamp4(hi - 8)), acc);
    return hsum2(d & bytes_mask(clamp4(lo - 12), clamp4(hi - 12)), acc);
}

__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }
// x mod 0xFFFF in [0, 0xFFFE].
__device__ __forceinline__ uint32_t mod_ffff(uint32_t x) {
    x = (x & 0xFFFFu) + (x >> 16);
    x = (x & 0xFFFFu) + (x >> 16);
    return x == 0xFFFFu ? 0u : x;
}
// The reference's `!fold(0xFFFF + S)` given m = S mod 0xFFFF (S = sum of BE words incl. pseudo-header).
__device__ __forceinline__ uint32_t csum_from_residue(uint32_t m) { return m == 0 ? 0u : 0xFFFFu - m; }
// BE residue of a LE-half sum.
__device__ __forceinline__ uint32_t be_residue(uint32_t le_sum) { return bswap16(mod_ffff(le_sum)); }

// ---------------------------------------------------------------------------------------------------------------------
// Byte accessors: registers (fast path, constant offsets < 64 after inlining) or global memory (slow path).
// ---------------------------------------------------------------------------------------------------------------------
struct RegAcc {
    uint32_t w[16];  // frame bytes [0, 64), little-endian dwords
    __device__ __forceinline__ uint32_t b8(uint32_t k) const { return (w[k >> 2] >> ((k & 3) * 8)) & 0xFFu; }
    __device__ __forceinline__ uint32_t le16(uint32_t k) const { return (w[k >> 2] >> ((k & 2) * 8)) & 0xFFFFu; }
    __device__ __forceinline__ uint32_t be16(uint32_t k) const { return bswap16(le16(k)); }
    __device__ __forceinline__ uint32_t u32(uint32_t k) const {
        return (k & 2) ? ((w[k >> 2] >> 16) | (w[(k >> 2) + 1] << 16)) : w[k >> 2];
    }
    __device__ __forceinline__ uint32_t be32(uint32_t k) const { return __builtin_bswap32(u32(k)); }
};
struct MemAcc {
    const uint8_t* f;
    __device__ __forceinline__ uint32_t b8(uint32_t k) const { return f[k]; }
    __device__ __forceinline__ uint32_t le16(uint32_t k) const { return (uint32_t)f[k] | ((uint32_t)f[k + 1] << 8); }
    __device__ __forceinline__ uint32_t be16(uint32_t k) const { return ((uint32_t)f[k] << 8) | f[k + 1]; }
    __device__ __forceinline__ uint32_t u32(uint32_t k) const { return le16(k) | (le16(k + 2) << 16); }
    __device__ __forceinline__ uint32_t be32(uint32_t k) const { return (be16(k) << 16) | be16(k + 2); }
    // LE-half sum over frame bytes [s, e), s even, odd tail padded with zero (tcp/header.rs:497-499).
    __device__ uint32_t sum_le16(uint32_t s, uint32_t e) const {
        uint32_t acc = 0, k = s;
        if ((reinterpret_cast<uintptr_t>(f) & 1) == 0) {
            const uint16_t* h = reinterpret_cast<const uint16_t*>(f);
            for (; k + 2 <= e; k += 2) acc += h[k >> 1];
        } else {
            for (; k + 2 <= e; k += 2) acc += le16(k);
        }
        if (k < e) acc += f[k];
        return acc;
    }
};

// Per-frame state carried from phase A to phase C.
struct Lane {
    uint32_t v;       // verdict or kPend*
    uint32_t src, dst;
    uint32_t ports;   // src_port | dst_port << 16
    uint32_t mhi;     // result meta bits 8..31 (protocol and protocol bytes, dk_rx.h)
    uint32_t seq, ack, winurg;
    uint32_t S, E;    // L4 region [S, E), frame-relative
    uint32_t hlen;    // TCP data offset / 8 for UDP
    uint32_t stored;  // stored L4 checksum (BE value)
    uint32_t need;    // L4 checksum must be verified
    uint32_t lsum;    // LE-half sum of the part of [S, E) summed in-lane
};

// Everything up to (not including) the L4 checksum, in Appendix A order (slow path: any alignment, any IHL, bytes
// read from global memory; the fast path is parse_fast below).
template <class A>
__device__ __forceinline__ void parse_headers(const A& a, uint32_t len, const RxParams& P, Lane& L) {
    L.v = kNone;
    if (len < 14) { L.v = DK_V_ETH_SHORT; return; }                          // E1
    const uint32_t et = a.be16(12);
    if (et != 0x0806u && et != 0x0800u && et != 0x86ddu) { L.v = DK_V_ETH_TYPE; return; }  // E2
    if (et == 0x0806u) {  // ArpHeader::parse_and_consume (arp/header.rs:80-111, :161-166)
        if (len - 14 < 28) { L.v = DK_V_ARP_SHORT; return; }
        const uint32_t op = a.be16(20);
        if (a.be16(14) != 1u || a.be16(16) != 0x0800u || a.b8(18) != 6u || a.b8(19) != 4u || (op != 1u && op != 2u)) {
            L.v = DK_V_ARP_UNSUP;
            return;
        }
        L.v = DK_V_ARP;
        L.mhi = op << 8;
        L.src = a.u32(28);
        L.dst = a.u32(38);
        L.S = 14;
        L.E = len;
        return;
    }
    if (et == 0x86ddu) { L.v = DK_V_IPV6; return; }
    const uint32_t iplen = len - 14;
    if (iplen < 20) { L.v = DK_V_IP_SHORT; return; }                         // I1
    const uint32_t b14 = a.b8(14);
    if ((b14 >> 4) != 4) { L.v = DK_V_IP_VERSION; return; }                  // I2
    const uint32_t hs = (b14 & 15u) * 4;
    if (hs < 20) { L.v = DK_V_IP_IHL_SMALL; return; }                        // I3
    if (iplen < hs) { L.v = DK_V_IP_HDR_TRUNC; return; }                     // I4
    const uint32_t tot = a.be16(16);
    if (tot < hs) { L.v = DK_V_IP_TOTLEN_SMALL; return; }                    // I5
    if (tot > iplen) { L.v = DK_V_IP_TOTLEN_BIG; return; }                   // I6
    const uint32_t flags = a.b8(20) >> 5;
    if (flags & 4u) { L.v = DK_V_IP_EVIL; return; }                          // I7
    if (flags & 1u) { L.v = DK_V_IP_MF; return; }                            // I8
    if (a.be16(20) & 0x1FFFu) { L.v = DK_V_IP_FRAGOFF; return; }             // I9
    if (a.b8(22) == 0) { L.v = DK_V_IP_TTL; return; }                        // I10
    const uint32_t proto = a.b8(23);
    if (proto != 1u && proto != 6u && proto != 17u) { L.v = DK_V_IP_PROTO; return; }  // I11
    const uint32_t ipcs = a.be16(24);
    if (ipcs == 0xFFFFu) { L.v = DK_V_IP_CSUM_FFFF; return; }                // I12
    // compute_checksum: 9 words of the first 20 bytes, checksum word skipped (ipv4/header.rs:280-301).
    const uint32_t hsum = a.le16(14) + a.le16(16) + a.le16(18) + a.le16(20) + a.le16(22) + a.le16(26) + a.le16(28) +
                          a.le16(30) + a.le16(32);
    if (csum_from_residue(be_residue(hsum)) != ipcs) { L.v = DK_V_IP_CSUM; return; }  // I13
    const uint32_t src = a.u32(26), dst = a.u32(30);
    if (dst != P.local_ip && dst != 0xFFFFFFFFu) { L.v = DK_V_IP_DST; return; }       // F1
    if (src == 0xFFFFFFFFu || (src & 0xF0u) == 0xE0u || src == 0) { L.v = DK_V_IP_SRC; return; }  // F2
    const uint32_t S = 14u + hs;
    const uint32_t seg = tot - hs;
    L.src = src;
    L.dst = dst;
    L.S = S;
    L.E = 14 + tot;
    if (proto == 1u) {  // Icmpv4Header::parse_and_strip (icmpv4/header.rs:47-66)
        if (seg < 8) { L.v = DK_V_ICMP_SHORT; return; }
        L.ports = a.be16(S + 4) | (a.be16(S + 6) << 16);
        L.mhi = 1u | (a.b8(S) << 8) | (a.b8(S + 1) << 16);
        L.hlen = 8;
        L.need = 1;
        L.v = kPendIcmp;
        return;
    }
    if (proto == 6u) {
        if (seg < 20) { L.v = DK_V_TCP_SHORT; return; }                      // T1
        const uint32_t b12 = a.b8(S + 12);
        const uint32_t doff = (b12 >> 4) * 4;
        if (seg < doff) { L.v = DK_V_TCP_DOFF_TRUNC; return; }               // T2
        if (doff < 20) { L.v = DK_V_TCP_DOFF_SMALL; return; }                // T3
        L.ports = a.be16(S) | (a.be16(S + 2) << 16);
        L.seq = a.be32(S + 4);
        L.ack = a.be32(S + 8);
        L.mhi = 6u | (a.b8(S + 13) << 8) | (b12 << 16);
        L.winurg = a.be16(S + 14) | (a.be16(S + 18) << 16);
        L.stored = a.be16(S + 16);
        L.hlen = doff;
        L.need = P.tcp_offload ? 0u : 1u;
        L.v = kPendTcp;
    } else {
        if (seg < 8) { L.v = DK_V_UDP_SHORT; return; }                       // U1
        if (a.be16(S + 4) != seg) { L.v = DK_V_UDP_LEN; return; }            // U2
        L.ports = a.be16(S) | (a.be16(S + 2) << 16);
        L.stored = a.be16(S + 6);
        L.hlen = 8;
        L.mhi = 17u;
        L.need = (!P.udp_offload && L.stored != 0) ? 1u : 0u;                // U3 precondition (udp/header.rs:78-82)
        L.v = kPendUdp;
    }
}

// parse_headers<true> restated without branches for the register window (IHL == 5, len >= 34, every offset < 64):
// each check is one compare + select, applied last-to-first so the first failing check in Appendix A order wins. The
// early-return form made the compiler re-materialise every zeroed Lane field on each of its ~25 exits, i.e. ~12
// v_mov per check per wave on the path every valid frame takes. I3/I4 (hs < 20, iplen < hs) cannot fire here.
__device__ __forceinline__ void parse_fast(const RegAcc& a, uint32_t len, const RxParams& P, Lane& L) {
    const uint32_t et = a.be16(12);
    const uint32_t iplen = len - 14;
    const uint32_t b14 = a.b8(14);
    const uint32_t tot = a.be16(16);
    const uint32_t frag = a.be16(20);
    const uint32_t proto = a.b8(23);
    const uint32_t ipcs = a.be16(24);
    // the 9 words of compute_checksum, whole dwords through v_dot2 (words at 16..22 and 28..30 are dwords 4, 5, 7)
    const uint32_t hsum = hsum2(a.w[7], hsum2(a.w[5], hsum2(a.w[4], (a.w[3] >> 16) + (a.w[6] >> 16) + (a.w[8] & 0xFFFFu))));
    const uint32_t src = a.u32(26), dst = a.u32(30);
    const uint32_t seg = tot - 20;
    const uint32_t b12 = a.b8(46);
    const uint32_t doff = (b12 >> 4) * 4;
    const bool tcp = proto == 6u;
    const uint32_t stored = tcp ? a.be16(50) : a.be16(40);

    uint32_t v4 = tcp ? (seg < 20 ? (uint32_t)DK_V_TCP_SHORT                                  // T1
                         : seg < doff ? (uint32_t)DK_V_TCP_DOFF_TRUNC                         // T2
                         : doff < 20 ? (uint32_t)DK_V_TCP_DOFF_SMALL : kPendTcp)              // T3
                      : (seg < 8 ? (uint32_t)DK_V_UDP_SHORT                                   // U1
                         : a.be16(38) != seg ? (uint32_t)DK_V_UDP_LEN : kPendUdp);            // U2
    const bool icmp = proto == 1u;
    uint32_t v = icmp ? (seg < 8 ? (uint32_t)DK_V_ICMP_SHORT : kPendIcmp) : v4;
    v = (src == 0xFFFFFFFFu || (src & 0xF0u) == 0xE0u || src == 0) ? (uint32_t)DK_V_IP_SRC : v;   // F2
    v = (dst != P.local_ip && dst != 0xFFFFFFFFu) ? (uint32_t)DK_V_IP_DST : v;                   // F1
    v = csum_from_residue(be_residue(hsum)) != ipcs ? (uint32_t)DK_V_IP_CSUM : v;                // I13
    v = ipcs == 0xFFFFu ? (uint32_t)DK_V_IP_CSUM_FFFF : v;                                       // I12
    v = (proto != 1u && proto != 6u && proto != 17u) ? (uint32_t)DK_V_IP_PROTO : v;              // I11
    v = a.b8(22) == 0 ? (uint32_t)DK_V_IP_TTL : v;                                               // I10
    v = (frag & 0x1FFFu) ? (uint32_t)DK_V_IP_FRAGOFF : v;                                        // I9
    v = (frag & 0x2000u) ? (uint32_t)DK_V_IP_MF : v;                                             // I8
    v = (frag & 0x8000u) ? (uint32_t)DK_V_IP_EVIL : v;                                           // I7
    v = tot > iplen ? (uint32_t)DK_V_IP_TOTLEN_BIG : v;                                          // I6
    v = tot < 20 ? (uint32_t)DK_V_IP_TOTLEN_SMALL : v;                                           // I5
    v = (b14 >> 4) != 4 ? (uint32_t)DK_V_IP_VERSION : v;                                         // I2
    v = et == 0x86ddu ? (uint32_t)DK_V_IPV6 : v;
    v = et == 0x0806u ? (uint32_t)DK_V_ARP : v;
    v = (et != 0x0806u && et != 0x0800u && et != 0x86ddu) ? (uint32_t)DK_V_ETH_TYPE : v;        // E2

    const bool pend = v == kPendTcp || v == kPendUdp || v == kPendIcmp;
    L.v = v;
    L.src = src;
    L.dst = dst;
    L.S = 34;
    L.E = 14 + tot;
    L.ports = icmp ? a.be16(38) | (a.be16(40) << 16) : a.be16(34) | (a.be16(36) << 16);
    L.seq = a.be32(38);
    L.ack = a.be32(42);
    L.mhi = tcp ? 6u | (a.b8(47) << 8) | (b12 << 16) : icmp ? 1u | (a.b8(34) << 8) | (a.b8(35) << 16) : 17u;
    L.winurg = a.be16(48) | (a.be16(52) << 16);
    L.stored = stored;
    L.hlen = tcp ? doff : 8u;
    L.need = pend && (tcp ? !P.tcp_offload : icmp ? true : (!P.udp_offload && stored != 0)) ? 1u : 0u;  // U3 :78-82
}

// TCP option walk (tcp/header.rs:215-302), over the option bytes in global memory. Returns 0 (ok), DK_V_TCP_OPT
// (EBADMSG) or DK_V_TCP_OPT_EIO (truncated read: std::io::Cursor::read_exact -> io::Error -> EIO). With `out`, the
// parsed list (the reference's [TcpOptions2; 5]) is written there when the walk succeeds.
__device__ __forceinline__ uint32_t opt_be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
__device__ __noinline__ uint32_t tcp_options(const uint8_t* o, uint32_t n, dk_tcp_opts* out) {
    dk_tcp_opts r;
    uint32_t* rw = reinterpret_cast<uint32_t*>(&r);
    for (int k = 0; k < 24; k++) rw[k] = 0;
    uint32_t pos = 0, nopt = 0, nsack = 0;
    while (pos < n) {
        const uint32_t kind = o[pos++];
        if (kind == 0) break;
        if (kind == 1) continue;
        dk_tcp_opt e{(uint8_t)kind, 0, 0, 0, 0};
        if (kind == 2 || kind == 3 || kind == 4 || kind == 5 || kind == 8) {
            if (pos >= n) return DK_V_TCP_OPT_EIO;
            const uint32_t l = o[pos++];
            uint32_t body;
            if (kind == 2) { if (l != 4) return DK_V_TCP_OPT; body = 2; }
            else if (kind == 3) { if (l != 3) return DK_V_TCP_OPT; body = 1; }
            else if (kind == 4) { if (l != 2) return DK_V_TCP_OPT; body = 0; }
            else if (kind == 5) {
                if (l != 10 && l != 18 && l != 26 && l != 34) return DK_V_TCP_OPT;
                body = l - 2;  // num_sacks * 8, read in 4-byte pieces
            } else { if (l != 10) return DK_V_TCP_OPT; body = 8; }
            if (n - pos < body) return DK_V_TCP_OPT_EIO;
            const uint8_t* b = o + pos;
            if (kind == 2) e.u16 = (uint16_t)((b[0] << 8) | b[1]);
            else if (kind == 3) e.u8 = b[0];
            else if (kind == 8) { e.v0 = opt_be32(b); e.v1 = opt_be32(b + 4); }
            else if (kind == 5) {
                const uint32_t ns = body / 8;
                e.u8 = (uint8_t)ns;
                e.u16 = (uint16_t)nsack;
                for (uint32_t k = 0; k < ns && nsack < 4; k++, nsack++) {
                    r.sack[nsack][0] = opt_be32(b + 8 * k);
                    r.sack[nsack][1] = opt_be32(b + 8 * k + 4);
                }
            }
            pos += body;
        } else {
            return DK_V_TCP_OPT;
        }
        if (nopt >= 5) return DK_V_TCP_OPT;  // "too many TCP options provided"
        r.opt[nopt] = e;
        nopt++;
    }
    if (out) {
        r.num = nopt;
        uint32_t* ow = reinterpret_cast<uint32_t*>(out);
        for (int k = 0; k < 24; k++) ow[k] = rw[k];
    }
    return 0;
}

// Open-addressing probe of the device socket table (see rx_common.h), split so that the first slot's load can be issued
// as soon as the key is parsed and consumed after the checksum work (its L2 latency is otherwise exposed per chunk:
// -17 % on IMIX without the probe).
struct ProbeKey {
    uint32_t kind, lip, rip, lport_rport;
};
__device__ __forceinline__ uint32_t probe_slot(const RxParams& P, const ProbeKey& k) {
    return flow_hash(k.kind, k.lip, k.rip, k.lport_rport) & P.table_mask;
}
__device__ __forceinline__ uint32_t probe_finish(const RxParams& P, const ProbeKey& k, uint32_t h, uint4 s) {
    const uint4* T = reinterpret_cast<const uint4*>(P.table);
    for (uint32_t i = 0; i <= P.table_mask; i++) {
        if (s.x == 0) break;
        if ((s.x >> 24) == k.kind && s.y == k.lip && s.z == k.rip && s.w == k.lport_rport) return s.x & 0xFFFFFFu;
        h = (h + 1) & P.table_mask;
        s = T[h];
    }
    return DK_FLOW_NONE;
}
// UDP binds and TCP listeners: one exact load of the port table (rx_common.h).
__device__ __forceinline__ uint32_t port_lookup(const RxParams& P, uint32_t base, uint32_t port) {
    return P.port_tab[base + port];
}
// The bind on (local_ip, port), issued ahead of the checksum work: kUb (the small-frame kernel's instantiation with
// the compact bind table in LDS, rx_common.h) its two buckets' words in s, else the port table's word in s.x;
// udp_local_finish reads the flow id out once it is needed.
extern __shared__ __attribute__((aligned(16))) uint32_t dk_dyn_lds[];
template <bool kUb>
__device__ __forceinline__ void udp_local_issue(const RxParams& P, uint32_t port, uint4& s) {
    if (kUb) {
        const uint2* T = reinterpret_cast<const uint2*>(dk_dyn_lds + P.ub_off);
        const uint32_t h = ub_hash(port, P.ub_seed);
        const uint2 a = T[h & P.ub_mask], b = T[(h >> 16) & P.ub_mask];
        s = make_uint4(a.x, a.y, b.x, b.y);
    } else {
        s.x = P.port_tab[kPortUdpLocal + port];
    }
}
template <bool kUb>
__device__ __forceinline__ uint32_t udp_local_finish(uint32_t port, const uint4& s) {
    return kUb ? ub_pick(s.x, s.y, s.z, s.w, port) : s.x;
}
// The LDS copy of the compact bind table (before the workgroup's first barrier).
__device__ __forceinline__ void ub_load(const RxParams& P, uint32_t tid, uint32_t nthreads) {
    const uint4* src = reinterpret_cast<const uint4*>(P.ub);
    uint4* dst = reinterpret_cast<uint4*>(dk_dyn_lds + P.ub_off);
    for (uint32_t k = tid; k < P.ub_words / 4; k += nthreads) dst[k] = src[k];
}

// The LDS Active table (rx_common.h): copied from global memory at the kernel start (before the workgroup's first
// barrier), then a lookup is two dependent LDS reads and a key compare. Returns the slot the global probe would have
// hit first ({kind << 24 | flow_id, local_ip, remote_ip, ports}), or zeros (an empty slot: probe_finish stops there,
// and the Passive lookup follows as it would after a miss in the global table).
__device__ __forceinline__ void lt_load(const RxParams& P, uint32_t tid, uint32_t nthreads) {
    const uint4* src = reinterpret_cast<const uint4*>(P.lt);
    uint4* dst = reinterpret_cast<uint4*>(dk_dyn_lds + P.lt_off);
    for (uint32_t k = tid; k < P.lt_words / 4; k += nthreads) dst[k] = src[k];
}
__device__ __forceinline__ uint4 lt_lookup(const RxParams& P, uint32_t rip, uint32_t ports) {
    const uint32_t* T = dk_dyn_lds + P.lt_off;
    const uint32_t h = flow_hash(DK_FLOW_TCP_ACTIVE, P.local_ip, rip, ports);
    const uint32_t n = P.lt_n;
    const uint32_t sl = lt_slot(h, T[3 * n + lt_bucket(h, P.lt_b)], n);
    const uint32_t kr = T[sl], kp = T[n + sl], fid = T[2 * n + sl];
    return kr == rip && kp == ports ? make_uint4(DK_FLOW_TCP_ACTIVE << 24 | fid, P.local_ip, rip, ports)
                                    : make_uint4(0, 0, 0, 0);
}

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// One quarter-wave's frame in a phase-B step.
struct CoopSlot {
    uint32_t boff;  // byte offset of the frame's first granule in the blob
    uint32_t nb, j, acc;
    bool has;
};

// Frame-blob granule loads: buffer_load_dwordx4 (SGPR resource + 32-bit lane offset). With the nontemporal policy it
// streams ~12 % faster than global_load_dwordx4 on gfx950 (dk_diag_read_probe modes 6 vs 3), needs one offset VGPR
// instead of a 64-bit address, and its range check is the phase-B mask: the resource covers the blob rounded up to
// 16 bytes (a granule holding a frame byte is loaded whole; it never crosses a page), so a load at kOob returns zeros
// without touching memory — no exec masking, no branch around each load. Blobs are <= DK_RX_MAX_BLOB (dk_rx.h).
constexpr uint32_t kOob = 0xFFFFFFF0u;
struct Blob {
    __amdgpu_buffer_rsrc_t rs;
    __device__ __forceinline__ Blob(const uint8_t* frames, uint64_t frames_bytes)
        : rs(__builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(frames), 0,
                                               (int)(uint32_t)((frames_bytes + 15) & ~15ull), 0x00020000)) {}
    template <bool kNt>
    __device__ __forceinline__ uint4 ld(uint32_t byte_off) const {
        const auto r = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)byte_off, 0, kNt ? 2 : 0);
        return make_uint4(r[0], r[1], r[2], r[3]);
    }
};

// A stride of 5 uint4 spreads the owner lanes' ds_read_b128 of hdr over the banks. The LDS bank
// conflicts left in the staged kernel are the LDS Active table's random lookups (76 %) and the counter
// atomics (20 %), by ablation (profiles/r04g_lds_conflicts.json).
constexpr uint32_t kHdrStride = 5;
struct WaveLds {
    uint2 rec[64];              // phase B: per rank {owner lane | granules << 8, offset of the frame's first granule}
    uint32_t csum[64];          // phase B: whole-frame LE-half sums by owner lane
    uint4 hdr[64][kHdrStride];  // phase B -> C: granules 0..4 of each big frame (bytes [0, 64) + shift)
    uint4 tail[64];             // phase B -> C: the last granule of each big frame
    uint32_t cb[16];            // staged kernel: the first frame of each chunk staged since the last flush
};
typedef __attribute__((address_space(3))) void lds_void;


// The bytes of one 64-frame chunk (phases A and B), shared by the RX and TX kernels:
//   Phase A (lane): descriptor; frames of <= 64 bytes load their bytes straight into registers.
//   Phase B (quarter-wave per frame, 4 frames per wave per round): frames of > 64 bytes are streamed whole, once, by
//     16 lanes (kCoopU x dwordx4 in flight each): granules summed with v_dot2_u32_u16, the header window and the last
//     granule deposited in LDS for the owner lane, the quarter's sum reduced by a DPP row scan. Reading each frame in
//     one contiguous pass keeps DRAM rows open (a separate 64-byte header read per frame cost 8 %).
// Any even frame address takes this vector path: granules are the 16-byte blocks from a = f - sh (sh = f mod 16, even,
// so the frame's 16-bit word grid is the granules' grid), loaded whole (a granule never crosses a page, so reading
// its bytes outside the frame cannot fault; they are masked or subtracted out of every sum). Odd addresses take the
// byte path.
struct Chunk {
    RegAcc R;       // frame bytes [0, 64) (bytes past the frame end are not defined)
    uint32_t fsum;  // big frames: LE-half sum from the frame start to the end of the last granule
    uint32_t nblk;  // big frames: 16-byte granules covering [a, f + len)
    uint32_t sh;    // f - a, even
    bool inb, vec, big;  // descriptor in bounds; even address (vector path); streamed by a quarter-wave
};

// R.w <- bytes [sh, sh + 64) of the 80 bytes {w[0..15], x[0..3]}, sh even: two dword-shift stages (8, 4 bytes) as
// masked blends, then a 2-byte funnel shift. Written as bit blends so the compiler keeps the 20 words in registers
// (a ternary between array elements became a dynamically indexed scratch array).
__device__ __forceinline__ void realign(uint32_t (&w)[16], const uint32_t (&x)[4], uint32_t sh) {
    uint32_t u[20];
#pragma unroll
    for (int k = 0; k < 16; k++) u[k] = w[k];
#pragma unroll
    for (int k = 0; k < 4; k++) u[16 + k] = x[k];
    const uint32_t m8 = 0u - ((sh >> 3) & 1u), m4 = 0u - ((sh >> 2) & 1u);
#pragma unroll
    for (int k = 0; k < 18; k++) u[k] = (u[k + 2] & m8) | (u[k] & ~m8);
#pragma unroll
    for (int k = 0; k < 17; k++) u[k] = (u[k + 1] & m4) | (u[k] & ~m4);
    const uint32_t b = sh & 2u;  // funnel-shift byte count: 0 or 2
#pragma unroll
    for (int k = 0; k < 16; k++) w[k] = __builtin_amdgcn_alignbyte(u[k + 1], u[k], b);
}

// Phase A facts of one lane's frame, from its descriptor. kShift = false: only 16-byte aligned frames take the vector
// path (others the byte path); the receive kernel's instantiation for batches the caller flags DK_RX_BATCH_ALIGNED16,
// which then needs no realignment code and fewer registers.
template <bool kShift>
struct FrameDesc {
    bool inb, vec, big;  // descriptor in bounds; even address (vector path); streamed by a quarter-wave
    uint32_t sh;         // f - a, even (a = granule base)
    uint32_t span;       // bytes from a to the frame end
    uint32_t nblk;       // big frames: granules covering [a, f + len)
    __device__ __forceinline__ FrameDesc(const uint8_t* frames, uint64_t frames_bytes, bool live, uint32_t off,
                                         uint32_t len) {
        inb = live && (uint64_t)off + len <= frames_bytes;
        const uint32_t fmod = (uint32_t)reinterpret_cast<uintptr_t>(frames + off) & 15u;
        sh = kShift ? fmod : 0u;
        vec = inb && (kShift ? (fmod & 1u) == 0 : fmod == 0);
        span = sh + len;
        big = vec && span > 64;
        nblk = big ? (span + 15) >> 4 : 0;
    }
};

// Phase A, small frames (<= 64 bytes from the granule base): straight into the register window. Granules the frame
// does not reach (and every granule of other frames) load at kOob, i.e. zeros from the buffer range check: no branch
// around a load (an exec-masked load per granule made the compiler drain vmcnt after each frame's first load).
template <bool kShift>
__device__ __forceinline__ void small_load(const FrameDesc<kShift>& F, const Blob& B, uint32_t off, RegAcc& R) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const bool use = F.vec && !F.big && (uint32_t)(16 * k) < F.span;
#ifndef DK_SMALL_LOAD_NT
#define DK_SMALL_LOAD_NT 0
#endif
        const uint4 q = B.template ld<DK_SMALL_LOAD_NT != 0>(use ? off - F.sh + 16 * k : kOob);
        R.w[4 * k + 0] = q.x;
        R.w[4 * k + 1] = q.y;
        R.w[4 * k + 2] = q.z;
        R.w[4 * k + 3] = q.w;
    }
}

// ---------------- Phase B: whole-frame quarter-wave streams ----------------
// Every frame of > 64 bytes is streamed once, whole, by 16 lanes. Lane l16 of a quarter-wave loads granules
// b = 96 it + 16 u + l16 (u < kCoopU) of its frame, in address order; slots past the frame load at kOob (zeros): no
// exec masking, no branch around a load. The header window (granules 0..4) is lanes 0..4's first load; the last
// granule (nb - 1) is stored by the lane that loads it; both go to LDS for the owner lane, with the quarter's sum
// (DPP row scan). A step = kRoundsPerStep rounds of 4 frames, all loads in flight together.
struct CoopPlan {  // wave-uniform
    uint32_t ncoop;  // big frames in the chunk
    uint32_t nmed;   // of which medium (<= kMedGran granules): ranks [0, nmed), streamed by the medium step shape
    uint32_t maxit;  // iterations per round of the large shape (1 unless a frame exceeds kCoopSpan granules)
};
// Step shapes: kCoopU = 6 slots per lane (a 1536-byte quarter-wave span) for large frames, kRoundsPerStep (the
// staged kernel: kRoundsStaged) rounds of 4 frames per step; medium frames (<= kMedGran granules, IMIX 576 B) ranked
// first and streamed with a DK_COOP_MED_U-load span, (kRoundsPerStep * kCoopU) / DK_COOP_MED_U rounds per step, i.e.
// 12 medium frames in flight per wave step instead of 4 (a 590-byte frame fills 37 of the large shape's 96 slots).
#ifndef DK_COOP_MED_U
#define DK_COOP_MED_U 5  // medium frames (<= 1,280 B) take a 5-load span, 8 of them per step (round 3, with 9 staged
                         // chunks: IMIX -2.5 % over a 6-load span; 4 loads: -1.1 %, 3: -0.8 % at 8 chunks; C2 ±0)
#endif
constexpr uint32_t kMedU = DK_COOP_MED_U > 0 ? DK_COOP_MED_U : 1;
[[maybe_unused]] constexpr uint32_t kMedR = (kRoundsPerStep * kCoopU) / kMedU;
constexpr uint32_t kMedGran = DK_COOP_MED_U > 0 ? 16 * kMedU : 0;
template <uint32_t U, uint32_t R>
struct CoopStep {
    CoopSlot sl[R];
    uint4 d[R][U];
};

// Per-rank records of the chunk's big frames in W.rec (medium frames first); wave-uniform plan. Ends with a wave
// barrier.
template <bool kShift>
__device__ __forceinline__ CoopPlan coop_plan(const FrameDesc<kShift>& F, uint32_t lane, uint32_t off, WaveLds& W) {
    CoopPlan pl;
    const uint64_t cm = __ballot(F.big);
    pl.ncoop = (uint32_t)__popcll(cm);
    pl.nmed = 0;
    pl.maxit = 1;
    if (pl.ncoop == 0) return pl;
    const bool med = F.big && F.nblk <= kMedGran;
    const uint64_t mm = __ballot(med), lm = cm & ~mm;
    pl.nmed = (uint32_t)__popcll(mm);
    if (F.big) {
        const uint64_t m = med ? mm : lm;
        const uint32_t rank = (med ? 0u : pl.nmed) +
                              __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        W.rec[rank] = make_uint2(lane | (F.nblk << 8), off - F.sh);  // one ds_read_b64 per round
    }
    if (__ballot(F.nblk > kCoopSpan)) {
        uint32_t mx = F.nblk;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, o));
        pl.maxit = __builtin_amdgcn_readfirstlane((mx - 1) / kCoopSpan + 1);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return pl;
}

// Slots of step r (ranks k0 + 4 (r .. r + R - 1) + quarter, below k1) and the loads of its iteration 0.
template <uint32_t U, uint32_t R, bool kHdrT = false>
__device__ __forceinline__ void coop_issue(uint32_t k0, uint32_t k1, uint32_t r, uint32_t lane, const WaveLds& W,
                                           const Blob& B, CoopStep<U, R>& S, uint32_t it) {
    const uint32_t q = lane >> 4, l16 = lane & 15;
    if (it == 0) {
#pragma unroll
        for (uint32_t h = 0; h < R; h++) {
            const uint32_t k = k0 + (r + h) * 4 + q;
            S.sl[h].has = k < k1;
            const uint2 rec = S.sl[h].has ? W.rec[k] : make_uint2(0, 0);
            S.sl[h].j = rec.x & 0xFFu;
            S.sl[h].nb = rec.x >> 8;  // 0 for an empty slot: every load is then out of range
            S.sl[h].boff = rec.y;
            S.sl[h].acc = 0;
        }
    }
    const uint32_t b0 = it * 16 * U + l16;
#pragma unroll
    for (uint32_t h = 0; h < R; h++)
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t b = b0 + 16 * u;
            // kHdrT (the TX kernels): each frame's first 16 granules (its first 256 bytes, u = 0) with the default
            // policy instead of nontemporal, so the header-window rewrite finds its line in L2 (TX C2 -3 %; the
            // receive kernels measured +1.4 % with it)
            const uint32_t a = b < S.sl[h].nb ? S.sl[h].boff + 16 * b : kOob;
            S.d[h][u] = ((kHdrT || DK_HDR_TEMPORAL) && u < DK_HDR_TEMPORAL_U && it == 0)
                            ? B.template ld<false>(a)
                            : B.template ld<DK_NT_LOADS != 0>(a);
        }
}

template <bool kShift, uint32_t U, uint32_t R>
__device__ __forceinline__ void coop_consume(CoopStep<U, R>& S, WaveLds& W, uint32_t lane, uint32_t it) {
    constexpr uint32_t kHdrGran = kShift ? 5u : 4u;  // header granules the owner lane needs
    const uint32_t l16 = lane & 15, b0 = it * 16 * U + l16;
#pragma unroll
    for (uint32_t h = 0; h < R; h++) {
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            S.sl[h].acc = block_sum(S.d[h][u], S.sl[h].acc);
            if (b0 + 16 * u + 1 == S.sl[h].nb) W.tail[S.sl[h].j] = S.d[h][u];  // nb == 0: never
        }
        if (S.sl[h].has && it == 0 && l16 < kHdrGran) W.hdr[S.sl[h].j][l16] = S.d[h][0];
    }
}

// Finish step r whose iteration-0 loads are in flight in S: consume them, run the remaining iterations, reduce.
template <bool kShift, uint32_t U, uint32_t R, bool kHdrT = false>
__device__ __forceinline__ void coop_finish(uint32_t k0, uint32_t k1, uint32_t maxit, uint32_t r, uint32_t lane,
                                            WaveLds& W, const Blob& B, CoopStep<U, R>& S) {
    coop_consume<kShift>(S, W, lane, 0);
    for (uint32_t it = 1; it < maxit; it++) {
        coop_issue<U, R, kHdrT>(k0, k1, r, lane, W, B, S, it);
        coop_consume<kShift>(S, W, lane, it);
    }
#pragma unroll
    for (uint32_t h = 0; h < R; h++) {
        // Quarter = DPP row of 16 lanes: inclusive row scan by row_shr 1/2/4/8; lane 15 holds the sum.
        uint32_t acc = S.sl[h].acc;
        acc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)acc, 0x111, 0xF, 0xF, false);
        acc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)acc, 0x112, 0xF, 0xF, false);
        acc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)acc, 0x114, 0xF, 0xF, false);
        acc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)acc, 0x118, 0xF, 0xF, false);
        if (S.sl[h].has && (lane & 15) == 15) W.csum[S.sl[h].j] = acc;
    }
}

// Phase B of one chunk: the medium frames' steps (kMR rounds each), then the large frames' steps (kR rounds each).
template <bool kShift, bool kHdrT = false, uint32_t kR = kRoundsPerStep, uint32_t kMR = kMedR>
__device__ __forceinline__ void coop_stream(const CoopPlan& pl, uint32_t lane, WaveLds& W, const Blob& B) {
#if DK_COOP_MED_U > 0
    for (uint32_t r = 0; r * 4 < pl.nmed; r += kMR) {
        DK_MARK(med_step);
        CoopStep<kMedU, kMR> S;
        coop_issue<kMedU, kMR, kHdrT>(0, pl.nmed, r, lane, W, B, S, 0);
        coop_finish<kShift, kMedU, kMR, kHdrT>(0, pl.nmed, 1, r, lane, W, B, S);
    }
#endif
    for (uint32_t r = 0; r * 4 < pl.ncoop - pl.nmed; r += kR) {
        DK_MARK(large_step);
        CoopStep<kCoopU, kR> S;
        coop_issue<kCoopU, kR, kHdrT>(pl.nmed, pl.ncoop, r, lane, W, B, S, 0);
        coop_finish<kShift, kCoopU, kR, kHdrT>(pl.nmed, pl.ncoop, pl.maxit, r, lane, W, B, S);
    }
}

// After the last step: the owner lane's whole-frame sum and header window (big frames), then frames not on a 16-byte
// boundary drop the granule bytes before the frame from the sum and shift the window into frame coordinates.
template <bool kShift>
__device__ __forceinline__ void coop_gather(const FrameDesc<kShift>& F, const CoopPlan& pl, uint32_t lane,
                                            const WaveLds& W, Chunk& C) {
    RegAcc& R = C.R;
    C.fsum = 0;
    if (pl.ncoop) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (F.big) {
            C.fsum = W.csum[lane];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint4 h = W.hdr[lane][k];
                R.w[4 * k + 0] = h.x;
                R.w[4 * k + 1] = h.y;
                R.w[4 * k + 2] = h.z;
                R.w[4 * k + 3] = h.w;
            }
        }
    }
    if (kShift && __ballot(F.vec && F.sh != 0)) {
        uint32_t x[4] = {0, 0, 0, 0};
        if (F.big && F.sh != 0) {
            const uint4 h = W.hdr[lane][4];
            x[0] = h.x; x[1] = h.y; x[2] = h.z; x[3] = h.w;
            C.fsum -= block_sum_masked(R.w[0], R.w[1], R.w[2], R.w[3], 0, (int)F.sh, 0);
        }
        if (F.vec && F.sh != 0) realign(R.w, x, F.sh);
    }
    C.sh = F.sh;
    C.inb = F.inb;
    C.vec = F.vec;
    C.big = F.big;
    C.nblk = F.nblk;
}

// Phases A and B of one 64-frame chunk, shared by the RX and TX kernels; every lane of the wave calls it.
// On return the owner lane holds frame bytes [0, 64) in C.R (realigned when sh != 0) and, for big frames, the LE-half
// sum of frame bytes [0, 16 * nblk - sh) in C.fsum and the last granule in W.tail[lane].
template <bool kShift, bool kHdrT = false, uint32_t kR = kRoundsPerStep>
__device__ __forceinline__ void stream_chunk(const uint8_t* frames, uint64_t frames_bytes, bool live, uint32_t lane,
                                             WaveLds& W, uint32_t off, uint32_t len, Chunk& C) {
    DK_MARK(phaseA);
    const FrameDesc<kShift> F(frames, frames_bytes, live, off, len);
    const Blob B(frames, frames_bytes);
    small_load(F, B, off, C.R);
    DK_MARK(plan);
    const CoopPlan pl = coop_plan(F, lane, off, W);
    coop_stream<kShift, kHdrT, kR>(pl, lane, W, B);
    DK_MARK(gather);
    coop_gather(F, pl, lane, W, C);
}

// LE-half sum of frame bytes [34, E) on the fast path (IHL == 5), from what stream_chunk left: the register window
// for small frames; for big frames sum(all granules) - sum[0, 34) - sum[E, 16 * nblk), the last granule being in
// LDS; a direct byte sum when IPv4 total_length ends more than 32 bytes before the last block (rare; sets resum).
template <class WL>
__device__ __forceinline__ uint32_t seg_sum_fast(const Chunk& C, const WL& W, uint32_t lane, const uint8_t* f,
                                                 int E, bool& resum) {
    const RegAcc& R = C.R;
    if (!__ballot(C.big || E != 64)) {  // every active lane: [34, 64) is the window's dwords 8 (upper half) .. 15
        uint32_t acc = hsum2(R.w[8] & 0xFFFF0000u, 0);
#pragma unroll
        for (int k = 9; k < 16; k++) acc = hsum2(R.w[k], acc);
        return acc;
    }
    if (!C.big) {
        // [34, E) inside the register window, E even in [34, 64]: dword k keeps its bytes below E, i.e. the low
        // 32 - sh bits with sh = clamp(32 - 8 (E - 4k), 0, 32) — one 64-bit shift per dword instead of two clamped
        // byte-mask computations (C3: -30 VALU per frame).
        const int t = 32 - 8 * E;
        uint32_t acc = 0;
#pragma unroll
        for (int k = 8; k < 16; k++) {
            const uint32_t sh = (uint32_t)min(max(t + 32 * k, 0), 32);
            uint32_t m = (uint32_t)(0xFFFFFFFFull >> sh);
            if (k == 8) m &= 0xFFFF0000u;  // bytes 32, 33 are the IPv4 header's
            acc = hsum2(R.w[k] & m, acc);
        }
        return acc;
    }
    if ((int)(16 * C.nblk - C.sh) - E <= 16) {
        uint32_t pre = block_sum(make_uint4(R.w[0], R.w[1], R.w[2], R.w[3]), 0);
        pre = block_sum(make_uint4(R.w[4], R.w[5], R.w[6], R.w[7]), pre);
        pre += R.w[8] & 0xFFFFu;
        const int t0 = (int)(16 * C.nblk - C.sh) - 16;  // frame offset of the last granule's first byte
        const uint4 a = W.tail[lane];
        const uint32_t post = block_sum_masked(a.x, a.y, a.z, a.w, E - t0, 16, 0);
        return C.fsum - pre - post;
    }
    resum = true;
    return MemAcc{f}.sum_le16(34, (uint32_t)E);
}

#ifndef DK_RES_STORE
#define DK_RES_STORE 0  // result stores: 0 plain (nontemporal in the small-frame kernel), 1 nontemporal everywhere
#endif
// Result stores. The small-frame kernel stores nontemporal (C3 -3.7 %: its 20-24 B of results per 64-byte frame are
// 28 % of its traffic); the other kernels measured ±0 either way (round 1) and keep plain stores.
template <bool kNt = false>
__device__ __forceinline__ void st_res(uint32_t* p, uint32_t v) {
    if (kNt || DK_RES_STORE == 1)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

// One frame per lane, 64 frames per wave chunk. Returns the verdict and the flow id (DK_FLOW_NONE if none).
//   Phases A, B: stream_chunk.
//   Phase C (lane): parse from registers, checksum = sum(all blocks) - sum[0, S) - sum[E, 16 * nblk) (exact integer
//     arithmetic), T4/U3, options, demux, results.
// The six required result words of one frame (dk_rx.h), held in registers when the kernel stages its stores.
struct Rec {
    uint32_t meta, src, dst, ports, pay, fid;
    uint32_t seq, ack, win;  // the optional TCP fields (staged only by the split kernel's kTcp instantiation)
};
// What a staging slot holds: the six required words, or (kTcp) nine.
template <bool kTcp>
struct StgRec {
    uint32_t meta, src, dst, ports, pay, fid;
    __device__ __forceinline__ StgRec& operator=(const Rec& r) {
        meta = r.meta; src = r.src; dst = r.dst; ports = r.ports; pay = r.pay; fid = r.fid;
        return *this;
    }
};
template <>
struct StgRec<true> {
    uint32_t meta, src, dst, ports, pay, fid, seq, ack, win;
    __device__ __forceinline__ StgRec& operator=(const Rec& r) {
        meta = r.meta; src = r.src; dst = r.dst; ports = r.ports; pay = r.pay; fid = r.fid;
        seq = r.seq; ack = r.ack; win = r.win;
        return *this;
    }
};
// Result staging: result stores interleaved with the frame stream cost ~11 % at C2 (every wave's
// 6 x 256 B of results per chunk reach HBM as scattered write bursts between the reads; ablation: storing them in an
// L2-resident window instead recovers it all). The staged kernels hold the last kStageK chunks' results in registers
// and store them together, so a wave's writes leave in one burst per kStageK chunks (at exit for C2 at 3 WG/CU).
#ifndef DK_STAGE_K
#define DK_STAGE_K 9
#endif
#ifndef DK_MIN_WAVES_STAGED
#define DK_MIN_WAVES_STAGED 3  // 9 x 6 staged words and one round of loads fit in 168 VGPRs without spills
#endif
constexpr int kStageK = DK_STAGE_K;
static_assert(kStageK <= 16, "WaveLds::cb holds the staged chunks' bases");

// Phase C of one chunk (lane per frame) from what the streaming left in C and W: parse, checksum, options, demux,
// results (stored, or handed back in rec for staging). Two halves so a kernel can interleave two chunks: rx_front
// (parse, the first table probe issued, the L4 sum) and rx_back (verdicts, demux, results); rx_finish runs both.
struct FinState {
    Lane L;
    ProbeKey k1;
    uint32_t h1;
    uint4 s1;
    bool fast, resum, big, inb;
};
template <bool kShift, class WL, bool kUb = false>
__device__ __forceinline__ void rx_front(const RxParams& P, bool live, uint32_t lane, WL& W, uint32_t off,
                                         uint32_t len, const Chunk& C, FinState& St, uint32_t stamp_base = ~0u) {
    Lane& L = St.L;
    bool& resum = St.resum;
    const RegAcc& R = C.R;
    const bool inb = C.inb, vec = C.vec, big = C.big;
    const uint8_t* f = P.frames + off;

    // ---------------- Phase C: parse, checksum, options, demux, results ----------------
    // Fast parse: 16-byte aligned, whole Ethernet + IPv4 fixed header present, IHL == 5 (S == 34).
    // ARP (ethertype bytes 08 06) is parsed by the byte path (low volume).
    St.big = big;
    St.inb = inb;
    const bool fast = vec && len >= 34 && ((R.w[3] >> 16) & 0x0Fu) == 5u && (R.w[3] & 0xFFFFu) != 0x0608u;
    resum = false;  // path-stats: streamed frame whose segment is re-summed in-lane
    L.v = kNone; L.src = L.dst = L.ports = L.mhi = L.seq = L.ack = L.winurg = 0;
    L.S = L.E = L.hlen = L.stored = L.need = L.lsum = 0;
    DK_MARK(parse);
    if (!live) {
        L.v = kNone;
    } else if (!inb) {
        L.v = DK_V_BAD_DESC;
    } else if (fast) {
        parse_fast(R, len, P, L);
    } else {
        DK_MARK(parse_slow);
        parse_headers(MemAcc{f}, len, P, L);
    }
    DK_SUB_STAMP(0);
    DK_MARK(probe_l4sum);
    // First demux probe, issued before the checksum work (speculative: used only if the frame passes T4/U3/T5).
    // TCP: the Active slot (hashed); UDP: the flow bound to (local_ip, port), one load of the port table.
    St.fast = fast;
    const ProbeKey k1{DK_FLOW_TCP_ACTIVE, P.local_ip, L.src, (L.ports >> 16) | (L.ports << 16)};
    St.k1 = k1;
    St.s1 = make_uint4(0, 0, 0, 0);
    uint32_t h1 = 0;
    if (L.v == kPendTcp && P.lt_words) {  // the LDS table: no global load
        St.s1 = lt_lookup(P, k1.rip, k1.lport_rport);
    } else if (L.v == kPendTcp) {  // the hash only for TCP lanes (a wave of UDP frames skips it)
        h1 = probe_slot(P, k1);
        St.s1 = reinterpret_cast<const uint4*>(P.table)[h1];
    }
    if (L.v == kPendUdp) udp_local_issue<kUb>(P, L.ports >> 16, St.s1);
    St.h1 = h1;
    if (L.need) L.lsum = fast ? seg_sum_fast(C, W, lane, f, (int)L.E, resum) : MemAcc{f}.sum_le16(L.S, L.E);
    DK_SUB_STAMP(1);
}

template <bool kStage, bool kOpt = true, bool kNtRes = false, bool kTcpStaged = false, bool kUb = false>
__device__ __forceinline__ void rx_back(const RxParams& P, uint32_t i, bool live, uint32_t lane, uint32_t off,
                                        FinState& St, uint32_t& v_out, uint32_t& fid_out, Rec& rec,
                                        uint32_t stamp_base = ~0u) {
    Lane& L = St.L;
    const ProbeKey& k1 = St.k1;
    const uint32_t h1 = St.h1;
    const uint4 s1 = St.s1;
    const bool fast = St.fast, resum = St.resum, big = St.big, inb = St.inb;
    const uint8_t* f = P.frames + off;

    DK_MARK(verdict_demux);
    uint32_t fid = DK_FLOW_NONE;
    if (L.v == kPendIcmp) {
        // compute_checksum over header + body must fold to 0, i.e. the BE word sum is 0 mod 0xFFFF; the LE-half sum
        // is 0 mod 0xFFFF exactly then (sum_BE == 256 * sum_LE, 256 invertible mod 0xFFFF) (icmpv4/header.rs:55-57)
        const uint32_t type = (L.mhi >> 8) & 0xFFu;
        L.v = mod_ffff(L.lsum) != 0 ? (uint32_t)DK_V_ICMP_CSUM
              : (type < 15 && ((kIcmpTypes >> type) & 1u)) ? (uint32_t)DK_V_ICMP : (uint32_t)DK_V_ICMP_TYPE;
    } else if (L.v == kPendTcp || L.v == kPendUdp) {
        const bool tcp = L.v == kPendTcp;
        if (L.need) {
            const uint32_t s = L.lsum - bswap16(L.stored);  // the reference sums the stored field as zero
            const uint32_t seg = L.E - L.S;
            const uint32_t lip = P.local_ip;
            // pseudo-header: src, local (tcp/peer.rs:223-228, udp/peer.rs:134), protocol, segment length (BE words)
            const uint32_t pseudo = bswap16(L.src & 0xFFFFu) + bswap16(L.src >> 16) + bswap16(lip & 0xFFFFu) +
                                    bswap16(lip >> 16) + (tcp ? 6u : 17u) + seg;
            const uint32_t c = csum_from_residue(mod_ffff(be_residue(s) + pseudo));
            if (c != L.stored) L.v = tcp ? DK_V_TCP_CSUM : DK_V_UDP_CSUM;
        }
        if (L.v == kPendTcp && L.hlen > 20) {
            DK_MARK(tcp_options);
            const uint32_t e = tcp_options(f + L.S + 20, L.hlen - 20,
                                           kOpt && live && P.res.tcp_opts ? P.res.tcp_opts + i : nullptr);
            if (e) L.v = e;
        }
        const uint32_t dport = L.ports >> 16;
        if (L.v == kPendTcp) {
            // SocketId::Active(local=(local_ip, dport), remote=(src, sport)), then Passive(local) (tcp/peer.rs:241-251)
            // Active(local, remote): the LDS table's answer is exact (a hit or an empty slot), the global table's
            // first slot may need the rest of the probe walk
            fid = P.lt_words ? (s1.x ? s1.x & 0xFFFFFFu : DK_FLOW_NONE) : probe_finish(P, k1, h1, s1);
            if (fid == DK_FLOW_NONE) fid = port_lookup(P, kPortTcpPassive, dport);
            L.v = fid == DK_FLOW_NONE ? DK_V_TCP_NOSOCK : DK_V_OK_TCP;
        } else if (L.v == kPendUdp) {
            // (local_ip, dport), then (0.0.0.0, dport) (udp/peer.rs:147-165)
            fid = udp_local_finish<kUb>(dport, s1);  // (local_ip, port)
            if (fid == DK_FLOW_NONE) fid = port_lookup(P, kPortUdpAny, dport);
            L.v = fid == DK_FLOW_NONE ? DK_V_UDP_NOSOCK : DK_V_OK_UDP;
        }
    }

    DK_SUB_STAMP(2);
    DK_MARK(results);
    const uint32_t v = L.v;
    if (live) {
        // fields for delivered / no-socket TCP and UDP and for parsed ARP and ICMPv4 (codes 0..3, dk_rx.h)
        const bool full = v <= DK_V_ICMP || v == DK_V_TCP_NOSOCK || v == DK_V_UDP_NOSOCK;
        const bool is_tcp = v == DK_V_OK_TCP || v == DK_V_TCP_NOSOCK;
        uint32_t meta = v, src = 0, dst = 0, ports = 0, pay = 0, seq = 0, ack = 0, win = 0;
        if (full) {
            meta |= L.mhi << 8;
            src = L.src;
            dst = L.dst;
            ports = L.ports;
            const uint32_t poff = L.S + L.hlen;
            pay = poff | ((L.E - poff) << 16);
            if (is_tcp) { seq = L.seq; ack = L.ack; win = L.winurg; }
        }
        rec = Rec{meta, src, dst, ports, pay, fid, seq, ack, win};
        if (!kStage) {
            st_res<kNtRes>(P.res.meta + i, meta);
            st_res<kNtRes>(P.res.src_ip + i, src);
            if (P.res.dst_ip) st_res<kNtRes>(P.res.dst_ip + i, dst);
            st_res<kNtRes>(P.res.ports + i, ports);
            st_res<kNtRes>(P.res.payload + i, pay);
            st_res<kNtRes>(P.res.flow_id + i, fid);
        }
        if (kOpt && !kTcpStaged) {  // optional outputs (kOpt = false: the caller asked for none; fewer live SGPRs)
            if (P.res.tcp_seq) P.res.tcp_seq[i] = seq;
            if (P.res.tcp_ack) P.res.tcp_ack[i] = ack;
            if (P.res.tcp_win) P.res.tcp_win[i] = win;
        }
    }
    DK_SUB_STAMP(3);
    if (kPathStatsOn && kOpt && P.path_stats) {  // diagnostics (dk_diag.h): one atomic per path per wave
        const uint32_t path = !fast ? 3u : resum ? 2u : big ? 1u : 0u;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint64_t m = __ballot(live && inb && path == k);
            if (m && lane == 0) atomicAdd(P.path_stats + k, (unsigned long long)__popcll(m));
        }
    }
    v_out = v;
    fid_out = fid;
}

template <bool kShift, bool kStage, class WL, bool kOpt = true, bool kNtRes = false, bool kTcpStaged = false,
          bool kUb = false>
__device__ __forceinline__ void rx_finish(const RxParams& P, uint32_t i, bool live, uint32_t lane, WL& W,
                                          uint32_t off, uint32_t len, const Chunk& C, uint32_t& v_out,
                                          uint32_t& fid_out, Rec& rec, uint32_t stamp_base = ~0u) {
    FinState St;
    rx_front<kShift, WL, kUb>(P, live, lane, W, off, len, C, St, stamp_base);
    rx_back<kStage, kOpt, kNtRes, kTcpStaged, kUb>(P, i, live, lane, off, St, v_out, fid_out, rec, stamp_base);
}

// Schedule of one wave (host-chosen per launch, measured in DESIGN.md "Tuning log"). Chunk k of a wave holds the
// frames i = c_k + lane with i < lim_k:
//   sched 0: round-robin 256-frame tiles, wave wv of workgroup b takes frames [t * 256 + 64 wv, +64) of tiles
//            t = b, b + G, ... (the grid sweeps one contiguous window of the blob);
//   sched 1: each wave owns one contiguous, equal share of the batch (+-1 frame), walked in 64-frame chunks.
// (Two more schedules — a phase-B-step interleave and an evenly split last round — measured +1 .. +5 % and were
// removed in round 3.)
struct WaveRange {
    uint32_t f0, f1, step, lane_off;
    // Chunk k: false when the wave has no chunk k.
    __device__ __forceinline__ bool chunk(uint32_t k, uint32_t& c, uint32_t& lim) const {
        c = f0 + k * step;
        lim = f1;
        return c < f1;
    }
};
template <uint32_t kW = kWaves>  // waves per workgroup
__device__ __forceinline__ WaveRange wave_range(uint32_t sched, uint32_t n, uint32_t wv, uint32_t lane) {
    WaveRange r;
    const uint32_t nw = gridDim.x * kW, gw = blockIdx.x * kW + wv;
    r.lane_off = lane;
    if (sched == 1) {
        r.f0 = (uint32_t)(((uint64_t)n * gw) / nw);
        r.f1 = (uint32_t)(((uint64_t)n * (gw + 1)) / nw);
        r.step = 64;
    } else {
        r.f0 = gw * 64;  // == blockIdx.x * kBlock + wv * 64
        r.f1 = n;
        r.step = 64 * nw;
    }
    return r;
}

// The staged results are a shift register: stg[q] holds chunk k_last - q (a fixed slot per chunk of a burst, selected
// by the burst position, made the compiler index the array dynamically: scratch memory).
template <class T, int kN>
__device__ __forceinline__ void stage_put(T (&stg)[kN], const Rec& rec) {
#pragma unroll
    for (int q = kN - 1; q > 0; q--) stg[q] = stg[q - 1];
    stg[0] = rec;
}
// Store the nst most recent staged chunks: stg[q] holds the results of the (nst - 1 - q)-th chunk staged since the last
// flush, whose first frame is cb[nst - 1 - q] (the wave's chunk bases in LDS, written by lane 0 as each chunk is
// staged: with the dynamic tail a chunk's position is not a function of its round). kNoRec marks idle lanes.
constexpr uint32_t kNoRec = 0xFFFFFFFFu;  // never a meta word (verdicts < 64)
__device__ __forceinline__ void flush_staged(const RxParams& P, const StgRec<false> (&stg)[kStageK], uint32_t nst,
                                             const uint32_t* cb, uint32_t lane) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int q = kStageK - 1; q >= 0; q--) {
        if ((uint32_t)q >= nst) continue;
        const uint32_t c = __builtin_amdgcn_readfirstlane(cb[nst - 1 - (uint32_t)q]);  // uniform: SGPR addressing
        if (stg[q].meta == kNoRec) continue;
        const uint32_t i = c + lane;
        st_res(P.res.meta + i, stg[q].meta);
        st_res(P.res.src_ip + i, stg[q].src);
        if (P.res.dst_ip) st_res(P.res.dst_ip + i, stg[q].dst);
        st_res(P.res.ports + i, stg[q].ports);
        st_res(P.res.payload + i, stg[q].pay);
        st_res(P.res.flow_id + i, stg[q].fid);
    }
}

// Per-chunk counters: the delivered frame's flow (packed-u16 LDS histogram, or a u64 global atomic for tables too
// large for LDS) and one LDS add per distinct verdict per wave.
// Flow counts are wave-aggregated while that pays: the first undone lane's flow takes every lane of the same flow in
// one add of the popcount, and the rounds go on while a round gathers >= kFlowAggMin lanes; the lanes left over add
// one each. One elephant flow (the tcp-echo shape, C1) is then one LDS add per chunk instead of 64 serialised adds on
// one LDS word; many flows (C2, C5) pay one extra round.
constexpr uint32_t kFlowAggMin = 4;
// A value the compiler must treat as lane-varying. Atomics whose address it can prove uniform get the LLVM atomic
// optimizer's expansion (exec save, mbcnt, a one-lane re-issue: ~10 instructions each) even where a single lane already
// issues them, as the leader-lane adds below do.
__device__ __forceinline__ uint32_t opaque_v(uint32_t x) {
    asm volatile("" : "+v"(x));
    return x;
}
// An LDS add the compiler does not see as an LDS access: issued while the wave's LDS-DMA window is in flight (the
// pipelined small-frame loop), a compiler-visible LDS atomic waits for the DMA first (it may alias the DMA's target);
// these never do (the counters are not in any wave's window). No return value, so no wait of its own.
__device__ __forceinline__ void lds_add_asm(uint32_t* p, uint32_t v) {
    const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)p;
    asm volatile("ds_add_u32 %0, %1" ::"v"(a), "v"(v));
}
template <bool kAsm = false>
__device__ __forceinline__ void flow_add(const RxParams& P, bool lds_flows, uint32_t* s_flow, uint32_t fid,
                                         uint32_t cnt) {
    if (kAsm && lds_flows) lds_add_asm(&s_flow[fid >> 1], cnt << ((fid & 1u) * 16));
    else if (lds_flows) atomicAdd(&s_flow[fid >> 1], cnt << ((fid & 1u) * 16));
    else if (P.flow_mode == kFlowGlobal)
        atomicAdd(reinterpret_cast<unsigned long long*>(P.res.flow_counts + fid), (unsigned long long)cnt);
}
template <bool kAsm = false>
__device__ __forceinline__ void count_chunk(const RxParams& P, bool live, uint32_t lane, uint32_t v, uint32_t fid,
                                            bool lds_flows, uint32_t* s_flow, uint32_t* s_vh) {
    const bool dl = live && (v == DK_V_OK_TCP || v == DK_V_OK_UDP);
    uint64_t todo = __ballot(dl);
    while (todo) {
        const uint32_t leader = (uint32_t)__builtin_ctzll(todo);
        const uint32_t f0 = __builtin_amdgcn_readlane(fid, leader);
        const uint64_t m = __ballot(fid == f0) & todo;
        if (lane == leader) flow_add<kAsm>(P, lds_flows, s_flow, opaque_v(f0), opaque_v((uint32_t)__popcll(m)));
        todo &= ~m;
        if (__popcll(m) < kFlowAggMin) break;
    }
    if ((todo >> lane) & 1u) flow_add<kAsm>(P, lds_flows, s_flow, fid, 1u);
    if (P.res.verdict_counts) {
        uint64_t todo = __ballot(live);
        while (todo) {
            const uint32_t leader = (uint32_t)__builtin_ctzll(todo);
            const uint32_t v0 = __builtin_amdgcn_readlane(v, leader);
            const uint64_t m = __ballot(live && v == v0);
            if (kAsm && lane == leader) lds_add_asm(&s_vh[v0], (uint32_t)__popcll(m));
            else if (lane == leader) atomicAdd(&s_vh[opaque_v(v0)], opaque_v((uint32_t)__popcll(m)));
            todo &= ~m;
        }
    }
}

// Workgroup exit: the LDS histograms (flow words in kFlowLds mode, then the verdict words) become this workgroup's row
// of the launch scratch (plain stores), and dk_flow_reduce_kernel, a second launch on the same stream, adds the rows to
// the caller's u64 counters — or, with DK_RX_BATCH_DEFER_COUNTS, the stream's next receive launch does inside its own
// kernel (combine_pending). Round 3 measured every in-launch combine of a launch's OWN rows against the second launch on
// two boxes: a two-level
// tree of arrival tickets (write-through rows, drained, the last arriver of each group summing its group) was slower on
// every workload (C2 +0.8 %, IMIX +2.3 %, C5 +3.3 %, C3 +23 %) and on small batches too, and replica rows filled by
// memory-side atomics tied with the second launch; the kernels hold no inter-workgroup hand-off at all.
// The kernels' by-value RxParams sits at the start of the kernel-argument segment. Fields used only at a kernel's end
// (counter rows, the pending-rows combine) are read from there at the point of use: read through the by-value
// parameter, the compiler loads them at the entry and keeps them in SGPRs across the chunk loop, where they spill to
// VGPR lanes and cost v_readlane in the loop.
__device__ __forceinline__ const RxParams& kargs(const RxParams& P) {
    (void)P;
    return *(const RxParams*)__builtin_amdgcn_kernarg_segment_ptr();  // (a C cast: it leaves the constant space)
}
__device__ __forceinline__ void flush_counters(const RxParams& P, uint32_t tid, uint32_t nthreads, bool lds_flows,
                                               const uint32_t* s_flow, const uint32_t* s_vh) {
    const RxParams& K = kargs(P);
    if (!K.row_words) return;
    uint32_t* row = K.flow_scratch + (size_t)blockIdx.x * K.row_stride;
    const uint32_t fw = K.flow_words;
    if (lds_flows)
        for (uint32_t k = tid; k < fw; k += nthreads) row[k] = s_flow[k];
    if (K.res.verdict_counts && tid < kVerdictWords) row[fw + tid] = tid < DK_V_COUNT ? s_vh[tid] : 0u;
}

// Sum of one 64-column x rpb-row block of counter rows into the destination counters (the column sums of the
// packed-u16 flow pairs, or a u32 verdict column), lane = column: kCombRows loads per lane in flight together per
// batch, then one device-scope u64 atomic per nonzero counter.
__device__ __forceinline__ void comb_block(const RowCombine& Q, uint32_t t, uint32_t lane) {
    const uint32_t w = (t % Q.ncolblk) * kCombCols + lane;
    const uint32_t r0 = (t / Q.ncolblk) * Q.rpb;
    if (w >= Q.row_words) return;
    const uint32_t r1 = min(Q.nrows, r0 + Q.rpb);
    uint64_t lo = 0, hi = 0;
    for (uint32_t rb = r0; rb < r1; rb += kCombRows) {
        uint32_t x[kCombRows];
#pragma unroll
        for (uint32_t k = 0; k < kCombRows; k++) {
            const uint32_t r = rb + k;
            x[k] = r < r1 ? Q.rows[(size_t)r * Q.row_stride + w] : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < kCombRows; k++) {
            lo += x[k] & 0xFFFFu;
            hi += x[k] >> 16;
        }
    }
    if (w >= Q.flow_words) {  // verdict column: a plain u32 count
        const uint32_t v = w - Q.flow_words;
        const uint64_t s = lo + (hi << 16);
        if (s && v < DK_V_COUNT && Q.verdicts)
            atomicAdd(reinterpret_cast<unsigned long long*>(Q.verdicts + v), (unsigned long long)s);
        return;
    }
    if (!Q.counts) return;
    if (lo) atomicAdd(reinterpret_cast<unsigned long long*>(Q.counts + 2 * w), (unsigned long long)lo);
    if (hi && 2 * w + 1 < Q.nflows)
        atomicAdd(reinterpret_cast<unsigned long long*>(Q.counts + 2 * w + 1), (unsigned long long)hi);
}

// The previous launch's pending counter rows (RowCombine, rx_common.h): the calling wave, the w-th of nw combining
// waves, adds blocks w, w + nw, ... (wave-uniform).
__device__ __forceinline__ void combine_pending(const RxParams& P, uint32_t lane, uint32_t w, uint32_t nw) {
    const RowCombine& Q = kargs(P).comb;
    if (!Q.rows) return;
    for (uint32_t t = w; t < Q.nblk; t += nw) comb_block(Q, t, lane);
}
// Tail form: the waves of a round-robin grid with the fewest chunks are the highest-numbered ones, so block j goes to
// wave nwaves - 1 - j (mod nwaves).
__device__ __forceinline__ void combine_pending_tail(const RxParams& P, uint32_t lane, uint32_t waves_per_group) {
    const uint32_t nw = gridDim.x * waves_per_group, gw = blockIdx.x * waves_per_group + (threadIdx.x >> 6);
    combine_pending(P, lane, nw - 1 - gw, nw);
}

// The staged kernel's dynamic tail (rx_common.h kTailXcds): chunks j in [lo, lo + T) after the round-robin rounds, in
// kTailXcds pools [lo + T x / 8, lo + T (x + 1) / 8), pool x handed out by counter x. Wave-uniform state; lane 0 issues
// the grabs (one returning device-scope atomic each) and readfirstlane broadcasts the old counter value.
constexpr uint32_t kNoChunk = 0xFFFFFFFFu;
// Pools are keyed by blockIdx.x mod tail_pools (the host takes the largest of 8, 4, 2, 1 that divides the grid, so every
// pool has the same number of waves): workgroups b and b + 8 share an XCD (MI355X_MICROARCH.md: dispatch deals blocks
// round-robin over the 8 XCDs), so with 8 pools each pool's counter is grabbed from one XCD — a speed property only;
// correctness needs just that every pool's waves drain it. A wave grabs only from its own pool (stealing from the
// other pools once the own one was empty cost every wave up to seven dependent atomic round trips at its very end,
// where nothing hides them: IMIX 141.8 -> 160.8 us, session r05b). The grab that finds the pool empty was issued a
// chunk earlier, so ending costs nothing. Live state: gv, lane 0's pending grab; the pool, the counter set and the
// tail range are re-read where used (the kernel is at its VGPR budget).
struct TailQ {
    uint32_t gv;  // lane 0: the pending grab's counter value
    __device__ __forceinline__ void issue(const RxParams& P, uint32_t lane) {
        const RxParams& K = kargs(P);
        uint32_t g = 0;
        if (lane == 0) g = atomicAdd(K.tail_ctr + (blockIdx.x & (K.tail_pools - 1)) * kTailStride, 1u);
        gv = g;
    }
    // The chunk the pending grab got, or kNoChunk once the pool is empty.
    __device__ __forceinline__ uint32_t resolve(const RxParams& P) const {
        const RxParams& K = kargs(P);
        const uint32_t lo = K.tail_ks * gridDim.x * kWaves, nchunk = (K.n + 63) / 64;
        const uint32_t T = nchunk > lo ? nchunk - lo : 0u, x = blockIdx.x & (K.tail_pools - 1);
        const uint32_t sh = 31u - (uint32_t)__builtin_clz(K.tail_pools);  // pools: a power of two
        const uint32_t g = __builtin_amdgcn_readfirstlane(gv);
        const uint32_t plo = lo + ((T * x) >> sh), phi = lo + ((T * (x + 1)) >> sh);
        return g < phi - plo ? plo + g : kNoChunk;
    }
};

// Persistent kernel: G resident workgroups (host-chosen); each wave walks its 64-frame chunks (wave_range), so
// per-workgroup state lives across chunks: the verdict histogram and, in kFlowLds mode, a packed-u16 per-flow
// histogram in LDS (flow f -> half f & 1 of word f >> 1; the host caps tiles per workgroup at 255 so a half never
// wraps). At exit both histograms reach the caller's u64 counters through flush_counters and dk_flow_reduce_kernel.
// kFlowGlobal (tables too large for LDS): one u64 atomic per delivered frame.
#ifndef DK_MIN_WAVES_ALIGNED
#define DK_MIN_WAVES_ALIGNED DK_MIN_WAVES
#endif
#ifndef DK_STAGED_PRIO
#define DK_STAGED_PRIO 0  // > 0: a wave streaming its chunk's frames issues at this priority, phase C at 0
#endif
#ifndef DK_STAGED_LATE_INIT
#define DK_STAGED_LATE_INIT 0  // 1: the LDS init, table copy and barrier after a wave's first frame stream
#endif
#ifndef DK_TAIL_LATE
#define DK_TAIL_LATE 0  // 1: a tail grab is for the next round (issued after this round's stream, resolved after its
                        // phase C, the descriptors loaded then): committed half a round ahead instead of 1.5
#endif
template <bool kShift, bool kStage>
__global__ __launch_bounds__(kBlock, kStage ? DK_MIN_WAVES_STAGED : kShift ? DK_MIN_WAVES : DK_MIN_WAVES_ALIGNED)
void dk_rx_kernel(RxParams P) {
    __shared__ WaveLds s_wave[kWaves];        // per-wave phase B/C exchange
    __shared__ uint32_t s_vh[DK_V_COUNT];     // verdict histogram
    extern __shared__ __attribute__((aligned(16))) uint32_t s_flow[];  // kFlowLds: packed u16 flow counters

    const uint32_t tid = threadIdx.x;
    const uint32_t lane = lane_id();
    const uint32_t wv = tid >> 6;
    // the dynamic tail (staged kernel, round-robin schedule): zero the counters the stream's next tail launch uses
    const bool dyn = kStage && P.tail_ctr != nullptr;
    if (dyn && blockIdx.x == 0 && tid < kTailXcds)
        __hip_atomic_store(P.tail_next + tid * kTailStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    DK_STAMPW_RT(12);
    DK_STAMPW(0);
    const bool lds_flows = P.flow_mode == kFlowLds;
    // the histograms' zeroing, the Active table's copy and the workgroup barrier: before the first chunk, or
    // (DK_STAGED_LATE_INIT) after a wave's first frame stream, which needs none of them (a wave without a chunk at its
    // end): the copy then overlaps the first stream
    const auto init = [&]() {
        for (uint32_t k = tid; k < DK_V_COUNT; k += kBlock) s_vh[k] = 0;
        if (lds_flows)
            for (uint32_t k = tid; k < P.flow_words; k += kBlock) s_flow[k] = 0;
        lt_load(P, tid, kBlock);
        __syncthreads();
    };
    constexpr bool kLateInit = DK_STAGED_LATE_INIT != 0 && kStage;
    if (!kLateInit) init();
    DK_STAMPW(1);

    const WaveRange r = wave_range(P.sched, P.n, wv, lane);
    StgRec<false> stg[kStage ? kStageK : 1];
    uint32_t nstg = 0;  // wave-uniform
    TailQ Q{0};
    const uint32_t ks = dyn ? P.tail_ks : ~0u;  // chunks from round ks on come from the tail (host: ks >= 2)
    uint32_t c, lim, nc, nlim;
    bool have = r.chunk(0, c, lim);
    const bool had = have;
    uint32_t noff = 0, nlen = 0;  // descriptors of this wave's next chunk
    if (have && c + r.lane_off < lim) {
        noff = P.off[c + r.lane_off];
        nlen = P.len[c + r.lane_off];
    }
    WaveLds& W = s_wave[wv];
    DK_ACC_DECL;
    for (uint32_t k = 0; have; k++, c = nc, lim = nlim) {
        DK_ACC_BEGIN();
        DK_MARK(loop_top);
        // The lane id re-materialised per chunk: without this the compiler keeps ~20 lane-derived address constants
        // of phases A-C in VGPRs across the whole loop, and this kernel sits at its 168-VGPR budget (3 waves/SIMD).
        uint32_t lane = lane_id();
        asm volatile("" : "+v"(lane));
        const uint32_t i = c + lane;
        const bool live = i < lim;
        const uint32_t off = noff, len = nlen;
        constexpr bool kLate = DK_TAIL_LATE != 0;
        const bool late = kLate && k + 1 >= ks;  // wave-uniform: the next chunk comes from a grab issued this round
        if (k + 1 < ks) {
            have = r.chunk(k + 1, nc, nlim);
        } else if (!kLate) {  // the tail: the chunk grabbed a round ago
            const uint32_t j = Q.resolve(P);
            have = j != kNoChunk;
            nc = 64 * j;
            nlim = P.n;
        }
        if (!late && have && nc + lane < nlim) {  // prefetch the next chunk's descriptors
            noff = P.off[nc + lane];
            nlen = P.len[nc + lane];
        }
        uint32_t v, fid;
        Rec rec;
        rec.meta = kNoRec;
        Chunk C;
        if (k < 3) DK_STAMPW(2 + 3 * k);
        DK_MARK(stream);
        if (DK_STAGED_PRIO) __builtin_amdgcn_s_setprio(DK_STAGED_PRIO);  // the frame stream issues ahead of phase C
        stream_chunk<kShift, false, kStage ? kRoundsStaged : kRoundsPerStep>(P.frames, P.frames_bytes, live, lane, W, off,
                                                                              len, C);
        // the grab for chunk k + 2, resolved at the top of the next round: issued after the frame stream (its return
        // register would be live through the stream's load registers, the kernel's register peak); phase C covers
        // its latency
        if (kLate ? late : have && k + 2 >= ks) Q.issue(P, lane);
        if (kLateInit && k == 0) init();
        if (k < 3) DK_STAMPW(3 + 3 * k);
        DK_ACC_SPLIT(0);
        if (DK_STAGED_PRIO) __builtin_amdgcn_s_setprio(0);
        DK_MARK(phaseC);
        rx_finish<kShift, kStage>(P, i, live, lane, W, off, len, C, v, fid, rec);
        if (k < 3) DK_STAMPW(4 + 3 * k);
        DK_ACC_SPLIT(1);
        // The next chunk's descriptors (loaded a chunk ago) are waited for here, before this chunk's stores: used first
        // at the top of the next chunk, after a staged flush, their wait also waited for every store's write ack.
        if (late) {  // DK_TAIL_LATE: resolve this round's grab; staging and counting cover the descriptors' latency
            const uint32_t j = Q.resolve(P);
            have = j != kNoChunk;
            nc = 64 * j;
            nlim = P.n;
            if (have && nc + lane < nlim) {
                noff = P.off[nc + lane];
                nlen = P.len[nc + lane];
            }
        } else {
            asm volatile("" ::"v"(noff), "v"(nlen));
        }
        DK_MARK(stage);
        if (kStage) {  // the last kStageK chunks' results; stored when full and at exit
            stage_put(stg, rec);
            if (lane == 0) W.cb[nstg] = c;
            if (++nstg == kStageK) {
                flush_staged(P, reinterpret_cast<const StgRec<false>(&)[kStageK]>(stg), nstg, W.cb, lane);
                nstg = 0;
            }
        }
        DK_ACC_SPLIT(2);
        DK_MARK(count);
        count_chunk(P, live, lane, v, fid, lds_flows, s_flow, s_vh);
        DK_ACC_SPLIT(3);
        DK_ACC_CHUNK();
        DK_MARK(loop_tail);
    }

    if (kLateInit && !had) init();  // a wave without a chunk: its share of the copy and the barrier
    DK_STAMPW(11);
    DK_MARK(epilogue);
    DK_ACC_BEGIN();
    if (kStage && nstg) flush_staged(P, reinterpret_cast<const StgRec<false>(&)[kStageK]>(stg), nstg, W.cb, lane);
    DK_ACC_SPLIT(4);
    combine_pending_tail(P, lane, kWaves);  // a previous launch's deferred counter rows, in this wave's tail
    DK_ACC_SPLIT(5);
    DK_STAMPW(14);
    __syncthreads();
    flush_counters(P, tid, kBlock, lds_flows, s_flow, s_vh);
    DK_STAMPW(15);
    DK_STAMPW_RT(13);
    DK_ACC_WRITE(kWaves);
}

// Small-frame kernel (batches of minimum-size frames, C3): the per-chunk chain descriptor -> frame -> parse -> socket
// probe -> stores is latency-bound at 64 bytes a frame, so this kernel drops the quarter-wave streaming machinery
// (its 48 load registers and 27 KB of LDS per workgroup) for more resident waves; descriptors are loaded two chunks
// ahead. The rare frame whose span exceeds the 64-byte register window is summed by the whole wave, one frame at a
// time, and hands the owner lane exactly what stream_chunk would (header window, whole-granule sum, last granule in
// LDS), so phase C is shared code. Measured and not kept: the next chunk's window or registers in
// flight during this chunk (no gain at 5 waves/SIMD, spills at 6), one generation of waves each taking 2-8 chunks
// at once (+35-120 %: every wave then loads, computes and stores in lockstep).
// Packed small frames are read as one contiguous window per chunk. Each lane reading its own 64-byte frame (4
// dwordx4 loads at a 64-byte lane stride, every load touching 32 lines) caps at ~3.8 TB/s on gfx950 whatever the
// occupancy, while the same bytes read lane-contiguously stream at ~7 TB/s (dk_diag_read_probe modes 9-11). So when
// the chunk's frames lie in one window of <= kWinGran granules, ceil(G / 64) LDS-DMA loads
// (buffer_load_dwordx4 ... lds, 1 KiB each, lane-contiguous) bring the window into the wave's LDS slot and every lane
// reads its frame's 64 bytes back; scattered frames (e.g. one per 2 KiB mbuf) keep the per-lane loads.
#ifndef DK_WIN_GRAN
#define DK_WIN_GRAN 288
#endif
constexpr uint32_t kWinGran = DK_WIN_GRAN;            // 4.5 KiB: 64 packed 64-byte frames at any even offset
constexpr uint32_t kWinLoads = (kWinGran + 63) / 64;  // DMA loads for a full window
// kUb: the last granules share the window's LDS (the general pass runs after the main loop's last window), leaving
// room for the LDS bind table at three workgroups per CU; measured 3 % slower at C3 with the port table, so the
// instantiation without the table keeps them apart (session r05zo).
#ifndef DK_SMALL_LDS_UNION
#define DK_SMALL_LDS_UNION 0  // 1: the general pass's last granules share the window's LDS in every instantiation
#endif
template <bool kUb>
struct SmallLds {
    uint4 tail[64];             // the general pass: the last granule of each big frame (seg_sum_fast)
    uint4 win[kWinLoads * 64];  // the main loop: the chunk's frame window (whole 1 KiB DMA pieces)
};
#if DK_SMALL_LDS_UNION
template <>
struct SmallLds<false> {
    union {
        uint4 win[kWinLoads * 64];
        uint4 tail[64];
    };
};
#endif
template <>
struct SmallLds<true> {
    union {
        uint4 win[kWinLoads * 64];
        uint4 tail[64];
    };
};
#ifndef DK_MIN_WAVES_SMALL
#define DK_MIN_WAVES_SMALL 6  // 80 VGPRs, no spills since round 5 (lane id re-materialised per chunk, uniform wave
                              // index): C3 -3.9 % vs 5 waves, random ports +0.8 % (session r05f). Before, 6 waves
                              // spilled 16-22 VGPRs to scratch (C3 +11 %, round 3).
#endif
#ifndef DK_SMALL_WAVES
#define DK_SMALL_WAVES 8  // waves per workgroup of the small-frame kernel: 8 since round 5 (at 6 waves/SIMD, half the
                          // counter rows: C3 -2.7 %, random ports -2 %, session r05v; 4 was ahead at 5 waves/SIMD)
#endif
#ifndef DK_SMALL_WAVES_PORT
#define DK_SMALL_WAVES_PORT DK_SMALL_WAVES  // the instantiation that looks UDP binds up in the port table
#endif
#ifndef DK_SMALL_WAVES_UB
#define DK_SMALL_WAVES_UB DK_SMALL_WAVES  // the instantiation with the LDS bind table (binds on scattered ports)
#endif
// Waves per workgroup of one small-kernel instantiation (the host asks dk_rx_small_block_waves(ub)).
template <bool kUb>
struct SmallShape {
    static constexpr uint32_t kWaves = kUb ? DK_SMALL_WAVES_UB : DK_SMALL_WAVES_PORT;
    static constexpr int kBlock = 64 * (int)kWaves;
};
// The window lives in LDS swizzled: slot s holds window granule s ^ ((s >> 4) & 3) (an involution: it swaps granules
// within aligned groups of 4 by bits 4-5 of the index, so each DMA piece still reads the same 64-byte pieces of the
// blob). Unswizzled, 64 packed 64-byte frames read back as 4 ds_read_b128 at a 64-byte lane stride put lanes
// {0, 12, 20, 24} of every lane group on the same 4 banks (MI355X_MICROARCH.md §LDS: 4-way, 3 extra cycles per group);
// swizzled, the 16 lanes of a group cover the 64 banks once.
#ifndef DK_WIN_SWIZZLE
#define DK_WIN_SWIZZLE 1
#endif
__device__ __forceinline__ uint32_t win_slot(uint32_t g) { return DK_WIN_SWIZZLE ? g ^ ((g >> 4) & 3u) : g; }
// Window plan of one chunk (wave-uniform): DMA'd into the wave's LDS slot, or per-lane loads.
struct WinPlan {
    bool win;
    uint32_t lo;  // blob offset of the window's first granule
};
// Issue the chunk's window DMA if its frames lie in one window (the wave's window slot must no longer be read).
template <bool kShift, class WL, uint32_t kGran = kWinGran>
__device__ __forceinline__ WinPlan small_window_issue(const FrameDesc<kShift>& F, const Blob& B, uint32_t off,
                                                      uint32_t len, bool live, uint32_t lane, WL& W) {
    WinPlan pl{false, 0};
    const bool use = F.vec && !F.big;
    const uint32_t a = off - F.sh;  // the frame's first granule
    const uint64_t lm = __ballot(live);
    if (!(lm & 1u)) return pl;  // lane 0 starts every chunk
    const uint32_t lo = __builtin_amdgcn_readfirstlane(a);
    const uint32_t last = 63u - (uint32_t)__builtin_clzll(lm);
    const uint32_t hi = __builtin_amdgcn_readlane(off + len, last);
    const bool inwin = !use || (a >= lo && off + len <= hi);
    if (hi > lo && hi - lo <= kGran * 16 && !__ballot(live && !inwin)) {
        const uint32_t G = (hi - lo + 15) >> 4;  // wave-uniform
        const uint32_t sl = win_slot(lane);  // the granule this lane's slot holds (slots 64 k + lane)
#pragma unroll
        for (uint32_t k = 0; k < kWinLoads; k++) {  // unrolled: no loop counters, uniform branches per piece
            if (k * 64 >= G) break;
            const uint32_t g = 64 * k + sl;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(B.rs, (lds_void*)&W.win[64 * k], 16, g < G ? lo + 16 * g : kOob,
                                                     0, 0, DK_NT_LOADS ? 2 : 0);
        }
        pl.win = true;
        pl.lo = lo;
    }
    return pl;
}
// The chunk's register windows: from the DMA'd window in LDS, or by per-lane loads (scattered frames).
template <bool kShift, class WL>
__device__ __forceinline__ void small_window_read(const WinPlan& pl, const FrameDesc<kShift>& F, const Blob& B,
                                                  uint32_t off, WL& W, RegAcc& R) {
    if (pl.win) {
        // The DMA pieces must have landed: wait for them explicitly (the compiler's own LDS-DMA tracking dropped
        // this wait once the read addresses were computed, round 3).
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t b = F.vec && !F.big ? (off - F.sh - pl.lo) >> 4 : 0u;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint4 q = W.win[win_slot(b + k)];
            R.w[4 * k + 0] = q.x;
            R.w[4 * k + 1] = q.y;
            R.w[4 * k + 2] = q.z;
            R.w[4 * k + 3] = q.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read out before the next chunk's DMA reuses the slot
        return;
    }
    small_load(F, B, off, R);
}

template <bool kShift, class WL>
__device__ __forceinline__ void small_big_frames(const FrameDesc<kShift>& F, uint32_t lane, uint32_t off, const Blob& B,
                                                 WL& W, Chunk& C) {
    RegAcc& R = C.R;
    uint32_t x[4] = {0, 0, 0, 0};
    C.fsum = 0;
    uint64_t bm = __ballot(F.big);
    if (bm) {
        while (bm) {
            const uint32_t j = (uint32_t)__builtin_ctzll(bm);
            bm &= bm - 1;
            const uint32_t base = __builtin_amdgcn_readlane(off - F.sh, j);
            const uint32_t nb = __builtin_amdgcn_readlane(F.nblk, j);
            uint32_t acc = 0;
            uint4 g0 = make_uint4(0, 0, 0, 0);  // granule `lane`: the header window is granules 0..4
            for (uint32_t b0 = 0; b0 < nb; b0 += 128) {
                const uint32_t b1 = b0 + lane, b2 = b1 + 64;
                const uint4 q1 = B.template ld<DK_NT_LOADS != 0>(b1 < nb ? base + 16 * b1 : kOob);
                const uint4 q2 = B.template ld<DK_NT_LOADS != 0>(b2 < nb ? base + 16 * b2 : kOob);
                acc = block_sum(q2, block_sum(q1, acc));
                if (b0 == 0) g0 = q1;
                if (b1 + 1 == nb) W.tail[j] = q1;
                if (b2 + 1 == nb) W.tail[j] = q2;
            }
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) acc += (uint32_t)__shfl_xor((int)acc, o);
            uint32_t h[20];
#pragma unroll
            for (int k = 0; k < 5; k++) {
                h[4 * k + 0] = (uint32_t)__shfl((int)g0.x, k);
                h[4 * k + 1] = (uint32_t)__shfl((int)g0.y, k);
                h[4 * k + 2] = (uint32_t)__shfl((int)g0.z, k);
                h[4 * k + 3] = (uint32_t)__shfl((int)g0.w, k);
            }
            if (lane == j) {
                C.fsum = acc;
#pragma unroll
                for (int k = 0; k < 16; k++) R.w[k] = h[k];
#pragma unroll
                for (int k = 0; k < 4; k++) x[k] = h[16 + k];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (kShift && __ballot(F.vec && F.sh != 0)) {
        if (F.big && F.sh != 0) C.fsum -= block_sum_masked(R.w[0], R.w[1], R.w[2], R.w[3], 0, (int)F.sh, 0);
        if (F.vec && F.sh != 0) realign(R.w, x, F.sh);
    }
    C.sh = F.sh;
    C.inb = F.inb;
    C.vec = F.vec;
    C.big = F.big;
    C.nblk = F.nblk;
}

// The small-frame kernel's main loop takes a frame only when it lies in its 64-byte register window (vector path, not
// streamed), has the whole Ethernet + 20-byte IPv4 header, is not ARP and, for TCP, carries no options: then phase C
// is the Appendix A chain from registers (parse_fast), one socket-table load, the segment sum from the window, the
// verdict, demux and result stores — no byte path, no wave-wide big-frame sum, no option walk (a call) in the loop.
// Every other frame is left to a second pass after the loop (per-chunk masks in the launch scratch, P.defer), which
// runs the general phase C (rx_finish) on them; results and counts are the same either way. Keeping the general path
// out of the loop took the loop's code from 95 VGPRs and 71 spilled SGPRs to the fast path's own.
#ifndef DK_SMALL_PRIO
#define DK_SMALL_PRIO 1
#endif
#ifndef DK_SMALL_LATE_BARRIER
#define DK_SMALL_LATE_BARRIER 0
#endif
#ifndef DK_SMALL_PIPE
#define DK_SMALL_PIPE 0  // 1: the next window's DMA in flight through a chunk's stores and counts (round 6: +5 % on C3)
#endif
// A workgroup barrier that orders LDS only (no wait for the wave's outstanding global loads and stores).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
template <bool kShift>
__device__ __forceinline__ bool small_fast_eligible(const FrameDesc<kShift>& F, uint32_t len, const RegAcc& R) {
    const bool ihl5 = ((R.w[3] >> 16) & 0x0Fu) == 5u;
    const bool arp = (R.w[3] & 0xFFFFu) == 0x0608u;
    const bool topt = R.b8(23) == 6u && (R.b8(46) >> 4) > 5u;
    return F.vec && !F.big && len >= 34 && ihl5 && !arp && !topt;
}
struct NoMid {
    __device__ __forceinline__ void operator()() const {}
};
// mid(): called between the verdicts (every socket-table load waited for) and the result stores: the pipelined loop
// issues the next window's DMA there. (Issued right after the table load, the compiler waited for the DMA with it:
// it counts LDS-DMA and loads as events that may complete out of order, so only vmcnt(0) covers the table load.)
template <bool kOpt, bool kUb, class Mid = NoMid>
__device__ __forceinline__ void small_fast(const RxParams& P, uint32_t i, bool live, uint32_t lane, const RegAcc& R,
                                           uint32_t len, uint32_t& v_out, uint32_t& fid_out, const Mid& mid = Mid()) {
    Lane L;
    parse_fast(R, len, P, L);
    if (!live) {
        L.v = kNone;
        L.need = 0;
    }
    // first socket-table load before the checksum arithmetic (as rx_front)
    const ProbeKey k1{DK_FLOW_TCP_ACTIVE, P.local_ip, L.src, (L.ports >> 16) | (L.ports << 16)};
    uint32_t h1 = 0;
    uint4 s1 = make_uint4(0, 0, 0, 0);
    if (L.v == kPendTcp) {
        h1 = probe_slot(P, k1);
        s1 = reinterpret_cast<const uint4*>(P.table)[h1];
    }
    if (L.v == kPendUdp) udp_local_issue<kUb>(P, L.ports >> 16, s1);
    uint32_t lsum = 0;
    if (L.need) {  // LE-half sum of frame bytes [34, E), E <= 64: the window (seg_sum_fast's small-frame forms)
        if (!__ballot(L.E != 64u)) {
            lsum = hsum2(R.w[8] & 0xFFFF0000u, 0);
#pragma unroll
            for (int k = 9; k < 16; k++) lsum = hsum2(R.w[k], lsum);
        } else {
            const int t = 32 - 8 * (int)L.E;
#pragma unroll
            for (int k = 8; k < 16; k++) {
                const uint32_t sh = (uint32_t)min(max(t + 32 * k, 0), 32);
                uint32_t m = (uint32_t)(0xFFFFFFFFull >> sh);
                if (k == 8) m &= 0xFFFF0000u;
                lsum = hsum2(R.w[k] & m, lsum);
            }
        }
    }
    uint32_t fid = DK_FLOW_NONE;
    if (L.v == kPendIcmp) {  // as rx_back (icmpv4/header.rs:55-57, protocol.rs:37-56)
        const uint32_t type = (L.mhi >> 8) & 0xFFu;
        L.v = mod_ffff(lsum) != 0 ? (uint32_t)DK_V_ICMP_CSUM
              : (type < 15 && ((kIcmpTypes >> type) & 1u)) ? (uint32_t)DK_V_ICMP : (uint32_t)DK_V_ICMP_TYPE;
    } else if (L.v == kPendTcp || L.v == kPendUdp) {
        const bool tcp = L.v == kPendTcp;
        if (L.need) {  // T4 / U3 (tcp/header.rs:203-207, udp/header.rs:78-88)
            const uint32_t sm = lsum - bswap16(L.stored);
            const uint32_t lip = P.local_ip;
            const uint32_t pseudo = bswap16(L.src & 0xFFFFu) + bswap16(L.src >> 16) + bswap16(lip & 0xFFFFu) +
                                    bswap16(lip >> 16) + (tcp ? 6u : 17u) + (L.E - L.S);
            if (csum_from_residue(mod_ffff(be_residue(sm) + pseudo)) != L.stored)
                L.v = tcp ? DK_V_TCP_CSUM : DK_V_UDP_CSUM;
        }
        const uint32_t dport = L.ports >> 16;
        if (L.v == kPendTcp) {  // Active(local, remote), then Passive(local) (tcp/peer.rs:241-251)
            fid = probe_finish(P, k1, h1, s1);
            if (fid == DK_FLOW_NONE) fid = port_lookup(P, kPortTcpPassive, dport);
            L.v = fid == DK_FLOW_NONE ? DK_V_TCP_NOSOCK : DK_V_OK_TCP;
        } else if (L.v == kPendUdp) {  // (local_ip, dport), then (0.0.0.0, dport) (udp/peer.rs:147-165)
            fid = udp_local_finish<kUb>(dport, s1);
            if (fid == DK_FLOW_NONE) fid = port_lookup(P, kPortUdpAny, dport);
            L.v = fid == DK_FLOW_NONE ? DK_V_UDP_NOSOCK : DK_V_OK_UDP;
        }
    }
    const uint32_t v = L.v;
    mid();
    if (live) {
        const bool full = v <= DK_V_ICMP || v == DK_V_TCP_NOSOCK || v == DK_V_UDP_NOSOCK;
        const bool is_tcp = v == DK_V_OK_TCP || v == DK_V_TCP_NOSOCK;
        const uint32_t poff = L.S + L.hlen;
        st_res<true>(P.res.meta + i, full ? v | L.mhi << 8 : v);
        st_res<true>(P.res.src_ip + i, full ? L.src : 0u);
        if (P.res.dst_ip) st_res<true>(P.res.dst_ip + i, full ? L.dst : 0u);
        st_res<true>(P.res.ports + i, full ? L.ports : 0u);
        st_res<true>(P.res.payload + i, full ? poff | ((L.E - poff) << 16) : 0u);
        st_res<true>(P.res.flow_id + i, fid);
        if (kOpt) {
            const bool t = full && is_tcp;
            if (P.res.tcp_seq) P.res.tcp_seq[i] = t ? L.seq : 0u;
            if (P.res.tcp_ack) P.res.tcp_ack[i] = t ? L.ack : 0u;
            if (P.res.tcp_win) P.res.tcp_win[i] = t ? L.winurg : 0u;
        }
    }
    if (kPathStatsOn && kOpt && P.path_stats) {  // diagnostics (dk_diag.h): every frame taken here is a register-window
        const uint64_t m = __ballot(live);           // frame (path 0)
        if (m && lane == 0) atomicAdd(P.path_stats + 0, (unsigned long long)__popcll(m));
    }
    v_out = v;
    fid_out = fid;
}

template <bool kShift, bool kOpt, bool kUb = false>
__global__ __launch_bounds__(SmallShape<kUb>::kBlock, DK_MIN_WAVES_SMALL) void dk_rx_small_kernel(RxParams P) {
    constexpr uint32_t kSmallWaves = SmallShape<kUb>::kWaves;
    constexpr int kSmallBlock = SmallShape<kUb>::kBlock;
    __shared__ SmallLds<kUb> s_wave[kSmallWaves];
    __shared__ uint32_t s_vh[DK_V_COUNT];  // verdict histogram
    extern __shared__ __attribute__((aligned(16))) uint32_t s_flow[];  // kFlowLds: packed u16 flow counters

    const uint32_t tid = threadIdx.x;
    const uint32_t lane = lane_id();
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: LDS bases (DMA m0) in SGPRs
    DK_STAMP_RT(12);
    DK_STAMP(0);
    const bool lds_flows = P.flow_mode == kFlowLds;
    const WaveRange r = wave_range<kSmallWaves>(P.sched, P.n, wv, lane);
    uint32_t c, lim, c1 = 0, lim1 = 0, c2 = 0, lim2 = 0;
    bool have = r.chunk(0, c, lim);
    bool have1 = have && r.chunk(1, c1, lim1);
    uint32_t off = 0, len = 0, off1 = 0, len1 = 0;
    // the first two chunks' descriptors in flight during the LDS init and the barrier
    if (have && c + r.lane_off < lim) {
        off = P.off[c + r.lane_off];
        len = P.len[c + r.lane_off];
    }
    if (have1 && c1 + r.lane_off < lim1) {
        off1 = P.off[c1 + r.lane_off];
        len1 = P.len[c1 + r.lane_off];
    }
    for (uint32_t k = tid; k < DK_V_COUNT; k += kSmallBlock) s_vh[k] = 0;
    if (lds_flows)
        for (uint32_t k = tid; k < P.flow_words; k += kSmallBlock) s_flow[k] = 0;
    if (kUb) ub_load(P, tid, kSmallBlock);
    // Without the LDS bind table the counters are the only shared LDS state: the barrier that orders their zeroing
    // before any count can wait until the first chunk's counts (kLateBarrier), off the first window's path.
    constexpr bool kLateBarrier = DK_SMALL_LATE_BARRIER && !kUb;
    const bool have0 = have;
    if (!kLateBarrier) __syncthreads();
    DK_STAMP(11);
    // The grid is one generation of waves and the chunks do not divide evenly: the waves with one chunk more than the
    // rest (the last round's) set the launch's length, so they issue first on their SIMD (s_setprio; round 4: C3
    // -2.1 % together with the first descriptors loaded before the barrier).
    if (DK_SMALL_PRIO) {
        uint32_t cc, ll;
        if (r.chunk(P.small_kmin, cc, ll)) __builtin_amdgcn_s_setprio(DK_SMALL_PRIO);  // (host: chunks / waves)
    }
    const Blob B(P.frames, P.frames_bytes);
    SmallLds<kUb>& W = s_wave[wv];
    // Pipeline: descriptors are loaded two chunks ahead. Chunk k + 2's descriptor loads are issued before chunk k's
    // window DMA, so the window's wait covers them, and chunk k's deferral mask is stored after its result stores and
    // only when the chunk left frames (`had`), so it sits behind the next window's wait. (Issued after the window,
    // rounds 2-3, the descriptor loads and the mask store were caught by the compiler's wait for the window registers of
    // the per-lane-load path: one more memory round trip per chunk.)
    Chunk C;
    FrameDesc<kShift> F(P.frames, P.frames_bytes, have && c + r.lane_off < lim, off, len);
    const uint32_t nw = gridDim.x * kSmallWaves, gw = blockIdx.x * kSmallWaves + wv;  // deferral mask index k nw + gw
    bool deferred = false;  // wave-uniform: a chunk left frames to the general pass
    // wave-uniform: bit k set = chunk k (< 64) stored its deferral mask; chunks from 64 on always store theirs
    uint64_t had = 0;
    DK_ACC_DECL;
    // kPipe (no LDS bind table; its general-pass granules share the window's LDS): chunk k + 1's window DMA is issued
    // inside chunk k, once k's verdicts are decided (its socket-table loads waited for), and is in flight through k's
    // result stores, counts and the loop's turn; chunk k + 3's descriptors come by LDS-DMA into
    // the wave's general-pass granule slots with it (registers holding a load in flight would be waited for at the
    // loop's turn) and are read out at the top of chunk k + 1. The counts' LDS adds are inline asm: a compiler-visible
    // LDS atomic would first wait for the pending DMA.
    constexpr bool kPipe = DK_SMALL_PIPE != 0 && !kUb;
    WinPlan pl{false, 0};
    uint32_t* const dsc = reinterpret_cast<uint32_t*>(&W.tail[0]);  // [0, 64): offsets; [64, 97): length dwords
    // Chunk j's descriptors into dsc: 64 offsets, and the 33 dwords covering its 64 lengths from the 4-byte boundary
    // below &len[j] (the length array is only 2-byte aligned); every load stays inside a dword that holds an element.
    const auto desc_dma = [&](uint32_t cj, uint32_t limj, uint32_t ln) {
        const uint32_t o = min(cj + ln, limj - 1);
        __builtin_amdgcn_global_load_lds(P.off + o, (lds_void*)dsc, 4, 0, 0);
        if (ln < 33) {
            const uintptr_t lb = reinterpret_cast<uintptr_t>(P.len + cj) & ~(uintptr_t)3;
            const uintptr_t hi = (reinterpret_cast<uintptr_t>(P.len + limj) - 1) & ~(uintptr_t)3;
            const uintptr_t la = min(lb + 4 * (uintptr_t)ln, hi);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(la), (lds_void*)(dsc + 64), 4, 0, 0);
        }
    };
    if (kPipe && have) {
        const uint32_t ln = lane_id();
        pl = small_window_issue(F, B, off, len, c + ln < lim, ln, W);
        uint32_t c2p, lim2p;
        if (have1 && r.chunk(2, c2p, lim2p)) desc_dma(c2p, lim2p, ln);
    }
    for (uint32_t k = 0; have; k++) {
        DK_ACC_BEGIN();
        // the lane id re-materialised per chunk (as in dk_rx_kernel): lane-derived constants are not held in VGPRs
        // across the loop
        DK_MARK(s_loop_top);
        uint32_t lane = lane_id();
        asm volatile("" : "+v"(lane));
        const uint32_t i = c + lane;
        const bool live = i < lim;
        const bool have2 = have1 && r.chunk(k + 2, c2, lim2);
        uint32_t off2 = 0, len2 = 0;
        if (!kPipe && have2 && c2 + lane < lim2) {  // descriptors two chunks ahead, before this chunk's window DMA
            off2 = P.off[c2 + lane];
            len2 = P.len[c2 + lane];
        }
        const FrameDesc<kShift> F1(P.frames, P.frames_bytes, have1 && c1 + lane < lim1, off1, len1);
        uint32_t v, fid;
        if (k == 0) DK_STAMP(1);
        DK_MARK(s_window);
        if (!kPipe) pl = small_window_issue(F, B, off, len, live, lane, W);
        small_window_read(pl, F, B, off, W, C.R);  // waits for every load and store in flight (vmcnt 0)
        if (kPipe && have2) {  // chunk k + 2's descriptors, DMA'd during chunk k - 1 (or before the loop)
            const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(P.len + c2) & 3u) + 2 * lane;
            const uint32_t o2 = dsc[lane], l2 = (dsc[64 + (sh >> 2)] >> ((sh & 3u) * 8)) & 0xFFFFu;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read out before chunk k + 3's DMA reuses the slots
            if (c2 + lane < lim2) {
                off2 = o2;
                len2 = l2;
            }
        }
        if (k < 3) DK_STAMP(2 + 3 * k);
        DK_MARK(s_eligible);
        DK_ACC_SPLIT(0);
        if (kShift && __ballot(live && F.vec && !F.big && F.sh != 0)) {  // realign the windows of shifted frames
            uint32_t x[4] = {0, 0, 0, 0};
            if (F.vec && !F.big && F.sh != 0) realign(C.R.w, x, F.sh);
        }
        const bool take = live && small_fast_eligible(F, len, C.R);
        const uint64_t dm = __ballot(live && !take);
        deferred = deferred || dm != 0;
        DK_MARK(s_fast);
        if (kPipe) {
            const auto mid = [&]() {
                uint32_t c3, lim3;
                if (have2 && r.chunk(k + 3, c3, lim3)) desc_dma(c3, lim3, lane);
                if (have1) pl = small_window_issue(F1, B, off1, len1, c1 + lane < lim1, lane, W);
                asm volatile("" ::: "memory");  // issued here, not sunk to the loop's end (the compiler did)
            };
            small_fast<kOpt, kUb>(P, i, take, lane, C.R, len, v, fid, mid);
        } else {
            small_fast<kOpt, kUb>(P, i, take, lane, C.R, len, v, fid);
        }
        if (k < 3) DK_STAMP(3 + 3 * k);
        DK_ACC_SPLIT(1);
        if (kLateBarrier && k == 0) lds_barrier();  // every wave of the workgroup arrives once (below if no chunk)
        DK_MARK(s_count);
        count_chunk<kPipe>(P, take, lane, v, fid, lds_flows, s_flow, s_vh);
        DK_MARK(s_loop_tail);
        if (dm != 0 || k >= 64) {  // read back by this wave after the loop
            if (lane == 0) P.defer[k * nw + gw] = dm;
            if (k < 64) had |= 1ull << k;
        }
        if (k < 3) DK_STAMP(4 + 3 * k);
        DK_ACC_SPLIT(2);
        DK_ACC_CHUNK();
        // rotate the pipeline
        have = have1;
        c = c1;
        lim = lim1;
        off = off1;
        len = len1;
        F = F1;
        have1 = have2;
        c1 = c2;
        lim1 = lim2;
        off1 = off2;
        len1 = len2;
    }
    DK_MARK(s_epilogue);
    if (kLateBarrier && !have0) lds_barrier();
    DK_ACC_BEGIN();
    if (deferred) {  // the general pass over the frames the loop left (byte path, streamed frames, options, ARP)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's mask stores
        uint32_t cd, limd;
        for (uint32_t k = 0; r.chunk(k, cd, limd); k++) {
            if (k < 64 && !((had >> k) & 1u)) continue;  // chunk k left no frame (no mask stored)
            const uint64_t m = P.defer[k * nw + gw];  // wave-uniform
            if (!m) continue;
            const uint32_t i = cd + r.lane_off;
            const bool mine = (m >> lane) & 1u;
            const uint32_t o = mine ? P.off[i] : 0u, ln = mine ? P.len[i] : 0u;
            const FrameDesc<kShift> Fd(P.frames, P.frames_bytes, mine, o, ln);
            small_load(Fd, B, o, C.R);
            small_big_frames(Fd, lane, o, B, W, C);
            uint32_t v, fid;
            Rec rec;
            rec.meta = kNoRec;
            rx_finish<kShift, false, SmallLds<kUb>, kOpt, true, false, kUb>(P, i, mine, lane, W, o, ln, C, v, fid, rec);
            count_chunk(P, mine, lane, v, fid, lds_flows, s_flow, s_vh);
        }
    }
    DK_ACC_SPLIT(3);
    combine_pending_tail(P, lane, kSmallWaves);  // a previous launch's deferred counter rows, in this wave's tail
    DK_ACC_SPLIT(4);
    DK_STAMP(14);
    __syncthreads();
    flush_counters(P, tid, kSmallBlock, lds_flows, s_flow, s_vh);
    DK_STAMP(15);
    DK_STAMP_RT(13);
    DK_ACC_SPLIT(5);
    DK_ACC_WRITE(kSmallWaves);
}

// A wave's chunks with their descriptors loaded one chunk ahead: D.off / D.len belong to chunk D.c (0 outside the
// batch); next() starts the loads of the following chunk.
// A global pointer in address space 1: where the compiler cannot prove a parameter's pointer global (TxParams in the
// split TX kernel) it emits flat loads and stores, which count in lgkmcnt too, so every LDS wait after them (the split
// kernels' hand-off spins and releases) also waits for the memory access: a descriptor prefetch or a window rewrite
// then stalls the hand-off for a full memory round trip.
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gptr(T* p) {
    return (__attribute__((address_space(1))) T*)(p);
}

struct DescAhead {
    uint32_t c, lim, off, len;
    bool have;
    template <class PT>  // RxParams or TxParams: off, len
    __device__ __forceinline__ DescAhead(const PT& P, const WaveRange& r, uint32_t p0) {
        have = r.chunk(p0, c, lim);
        off = len = 0;
        if (have && c + r.lane_off < lim) {
            off = gptr(P.off)[c + r.lane_off];
            len = gptr(P.len)[c + r.lane_off];
        }
    }
    template <class PT>
    __device__ __forceinline__ void next(const PT& P, const WaveRange& r, uint32_t p) {
        have = r.chunk(p, c, lim);
        off = len = 0;
        if (have && c + r.lane_off < lim) {
            off = gptr(P.off)[c + r.lane_off];
            len = gptr(P.len)[c + r.lane_off];
        }
    }
};

// LDS flag words between the waves of a workgroup (the split kernels' hand-off): acquire spin, release publish.
typedef __attribute__((address_space(3))) uint32_t lu32;
__device__ __forceinline__ void lds_wait_eq(uint32_t* w, uint32_t want) {
    while (__hip_atomic_load((lu32*)w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != want)
        __builtin_amdgcn_s_sleep(1);
}
__device__ __forceinline__ void lds_publish(uint32_t* w, uint32_t v) {
    __hip_atomic_store((lu32*)w, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}


// Split kernel: one workgroup per CU, two roles. Stream waves 0..3 run phases A+B of their chunks (sched 0 over the 4
// stream waves of each workgroup) into LDS buffers (header windows, last granules, whole-frame sums; frames of <= 64
// bytes ride along as their register window), and kFin finish waves per stream wave run phase C (parse, checksum,
// options, demux, counters, results) from those buffers: finisher f of stream wave w takes w's chunks p with
// p % kFin == f. The streaming waves never stop for parse, demux, counters or result stores — 4 streaming waves per CU
// is also the count at which the read probe peaks — and the finish waves stage their results in registers for one
// burst per kStg chunks.
//   kFin = 1 (512 threads, 2 waves/SIMD, 256 VGPRs, 16 staged chunks): large frames (C2, C5), where phase C is a small
//     share of a chunk's time. (kFin = 2, 768 threads for mixed sizes, measured slower than the staged kernel on IMIX
//     and was removed in round 3)
#ifndef DK_SPLIT_NT_RES
#define DK_SPLIT_NT_RES true  // split kernels: result bursts nontemporal (C2 -0.3 %, C5 -1.4 %, steadier)
#endif
template <int kFin>
struct SplitShape {
    static_assert(kFin == 1, "one finish wave per stream wave");
    static constexpr int kThreads = 64 * kWaves * (1 + kFin);
#ifndef DK_SPLIT_BUFS
#define DK_SPLIT_BUFS 3
#endif
#ifndef DK_SPLIT_STG
#define DK_SPLIT_STG 16
#endif
    static constexpr int kBufs = DK_SPLIT_BUFS;  // LDS buffers per stream wave
    static constexpr int kStg = DK_SPLIT_STG;    // chunks of results a finish wave stages
#ifndef DK_SPLIT_STG_TCP
#define DK_SPLIT_STG_TCP 10
#endif
    static constexpr int kStgTcp = DK_SPLIT_STG_TCP;  // ... with the TCP fields (9 words a frame)
};
constexpr int kSplitBlock = SplitShape<1>::kThreads;  // the TX split kernel's shape
// Rounds of 4 frames a split-kernel stream wave keeps in flight per step (large frames; medium frames: as many 5-load
// rounds as fit the same load registers). A stream wave's chunks are a chain of dependent steps, so a batch with few
// chunks per stream wave (C1: 2) is bound by the chain length, not by bandwidth; the finish waves' register budget
// (256 VGPRs) leaves the stream role room for deeper steps.
#ifndef DK_SPLIT_ROUNDS
#define DK_SPLIT_ROUNDS 2
#endif
constexpr uint32_t kSplitRounds = DK_SPLIT_ROUNDS;
constexpr uint32_t kSplitMedRounds = (kSplitRounds * kCoopU) / kMedU;
template <int kStgK>
__device__ __forceinline__ void store_tcp_fields(const RxParams& P, const StgRec<false>&, uint32_t) {}
template <int kStgK>
__device__ __forceinline__ void store_tcp_fields(const RxParams& P, const StgRec<true>& x, uint32_t i) {
    if (P.res.tcp_seq) st_res<DK_SPLIT_NT_RES>(P.res.tcp_seq + i, x.seq);
    if (P.res.tcp_ack) st_res<DK_SPLIT_NT_RES>(P.res.tcp_ack + i, x.ack);
    if (P.res.tcp_win) st_res<DK_SPLIT_NT_RES>(P.res.tcp_win + i, x.win);
}
template <int kStgK, bool kTcp>
__device__ __forceinline__ void flush_split(const RxParams& P, const StgRec<kTcp> (&stg)[kStgK], uint32_t nst,
                                            const WaveRange& r, uint32_t k_last, uint32_t stride) {
#pragma unroll
    for (int q = kStgK - 1; q >= 0; q--) {
        if ((uint32_t)q >= nst) continue;
        uint32_t c, lim;
        (void)r.chunk(k_last - (uint32_t)q * stride, c, lim);
        if (stg[q].meta == kNoRec) continue;
        const uint32_t i = c + r.lane_off;
        st_res<DK_SPLIT_NT_RES>(P.res.meta + i, stg[q].meta);
        st_res<DK_SPLIT_NT_RES>(P.res.src_ip + i, stg[q].src);
        if (P.res.dst_ip) st_res<DK_SPLIT_NT_RES>(P.res.dst_ip + i, stg[q].dst);
        st_res<DK_SPLIT_NT_RES>(P.res.ports + i, stg[q].ports);
        st_res<DK_SPLIT_NT_RES>(P.res.payload + i, stg[q].pay);
        st_res<DK_SPLIT_NT_RES>(P.res.flow_id + i, stg[q].fid);
        store_tcp_fields<kStgK>(P, stg[q], i);
    }
}

// Hand-off through kBufs LDS buffers per stream wave (chunk p in buffer p % kBufs), each with a ready word (p + 1:
// written, set by the stream wave) and a free word (p + 1: read out, set by the finish wave that took p). A stream wave
// runs up to kBufs - 1 chunks ahead of the slowest finisher and no wave waits at a workgroup barrier.

// kTcp: the LibOS record (tcp_seq / tcp_ack / tcp_win requested) — the finish waves stage those too (9 words per
// frame, 16 chunks in 256 VGPRs) instead of storing them between the frame reads.
template <bool kShift, int kFin, bool kTcp = false>
__global__ __launch_bounds__(SplitShape<kFin>::kThreads, 1) void dk_rx_split_kernel(RxParams P) {
    using S = SplitShape<kFin>;
    constexpr int kBufs = S::kBufs;
    constexpr int kStg = kTcp ? S::kStgTcp : S::kStg;
    __shared__ WaveLds s_buf[kBufs][kWaves];  // [chunk % kBufs][stream wave]
    __shared__ uint32_t s_ready[kWaves][kBufs], s_free[kWaves][kBufs];
    __shared__ uint32_t s_vh[DK_V_COUNT];  // verdict histogram
    extern __shared__ __attribute__((aligned(16))) uint32_t s_flow[];  // kFlowLds: packed u16 flow counters

    const uint32_t tid = threadIdx.x;
    const uint32_t lane = lane_id();
    const uint32_t wv = tid >> 6, sw = wv & (kWaves - 1);
    const bool finisher = wv >= (uint32_t)kWaves;
    const uint32_t fin = finisher ? (wv - kWaves) / kWaves : 0u;  // which of the stream wave's finishers
    const bool lds_flows = P.flow_mode == kFlowLds;
    for (uint32_t k = tid; k < DK_V_COUNT; k += S::kThreads) s_vh[k] = 0;
    if (lds_flows)
        for (uint32_t k = tid; k < P.flow_words; k += S::kThreads) s_flow[k] = 0;
    if (tid < kWaves * kBufs) {
        (&s_ready[0][0])[tid] = 0;
        (&s_free[0][0])[tid] = 0;
    }
    lt_load(P, tid, S::kThreads);
    __syncthreads();

    const WaveRange r = wave_range(0, P.n, sw, lane);  // sched 0 over the 4 stream waves of each workgroup
    const Blob B(P.frames, P.frames_bytes);
    // The two roles run separate loops, so neither carries the other's registers (the finish waves' 16 staged chunks
    // are not live in the stream loop, which may then keep deeper steps in flight: DK_SPLIT_ROUNDS). Both read their
    // descriptors one chunk ahead (round 4: loaded at the top of chunk p, a stream wave opened every chunk with a
    // dependent descriptor round trip before its first frame load; C5 -1.3 %).
    DescAhead D(P, r, finisher ? fin : 0u);
    if (!finisher) {
        for (uint32_t p = 0; D.have; p++) {
            const uint32_t b = p % kBufs;
            WaveLds& W = s_buf[b][sw];
            const bool live = D.c + r.lane_off < D.lim;
            const uint32_t off = D.off, len = D.len;
            D.next(P, r, p + 1);
            const FrameDesc<kShift> F(P.frames, P.frames_bytes, live, off, len);
            // frames of <= 64 bytes: their granules ride along with the big frames' stream and reach the finisher
            // through the LDS header slot too, so the finish wave never waits on frame memory (IMIX: 7 of 12 frames)
            RegAcc Rs;
            small_load(F, B, off, Rs);
            if (p >= (uint32_t)kBufs) lds_wait_eq(&s_free[sw][b], p - kBufs + 1);  // buffer read out
            const CoopPlan pl = coop_plan(F, lane, off, W);
            coop_stream<kShift, false, kSplitRounds, kSplitMedRounds>(pl, lane, W, B);
            if (F.vec && !F.big)
#pragma unroll
                for (int k = 0; k < 4; k++)
                    W.hdr[lane][k] = make_uint4(Rs.w[4 * k], Rs.w[4 * k + 1], Rs.w[4 * k + 2], Rs.w[4 * k + 3]);
            if (lane == 0) lds_publish(&s_ready[sw][b], p + 1);
        }
    } else {
        // a previous launch's deferred counter rows: the finish waves have nothing to do until their stream wave's
        // first chunk has landed
        combine_pending(P, lane, blockIdx.x * kWaves + sw, gridDim.x * kWaves);
        StgRec<kTcp> stg[kStg];
        uint32_t nstg = 0, klast = 0;
        for (uint32_t p = fin; D.have; p += (uint32_t)kFin) {
            const uint32_t b = p % kBufs;
            WaveLds& W = s_buf[b][sw];
            const uint32_t i = D.c + r.lane_off;
            const bool live = i < D.lim;
            const uint32_t off = D.off, len = D.len;
            D.next(P, r, p + (uint32_t)kFin);
            const FrameDesc<kShift> F(P.frames, P.frames_bytes, live, off, len);
            Chunk C;
            lds_wait_eq(&s_ready[sw][b], p + 1);
            if (F.vec && !F.big)
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint4 h = W.hdr[lane][k];
                    C.R.w[4 * k] = h.x;
                    C.R.w[4 * k + 1] = h.y;
                    C.R.w[4 * k + 2] = h.z;
                    C.R.w[4 * k + 3] = h.w;
                }
            const CoopPlan pl{(uint32_t)__popcll(__ballot(F.big)), 0, 1};
            coop_gather(F, pl, lane, W, C);
            uint32_t v, fid;
            Rec rec;
            rec.meta = kNoRec;
            rx_finish<kShift, true, WaveLds, true, false, kTcp>(P, i, live, lane, W, off, len, C, v, fid, rec);
            asm volatile("" ::"v"(D.off), "v"(D.len));  // waited for before the stores (as dk_rx_kernel)
            if (lane == 0) lds_publish(&s_free[sw][b], p + 1);  // after this wave's last read of W (release)
            stage_put(stg, rec);
            klast = p;
            if (++nstg == (uint32_t)kStg) {
                flush_split<kStg, kTcp>(P, stg, nstg, r, klast, (uint32_t)kFin);
                nstg = 0;
            }
            count_chunk(P, live, lane, v, fid, lds_flows, s_flow, s_vh);
        }
        if (nstg) flush_split<kStg, kTcp>(P, stg, nstg, r, klast, (uint32_t)kFin);
    }
    __syncthreads();
    flush_counters(P, tid, S::kThreads, lds_flows, s_flow, s_vh);
}

// Adds the per-workgroup rows of flow_scratch[rows][row_words] into the caller's u64 counters: columns
// [0, flow_words) are packed-u16 flow pairs (flow_counts), the next DK_V_COUNT are u32 verdict counts
// (verdict_counts). Block (x, y) = 64 columns x kReduceRows rows: wave w sums every 4th row of the block's rows (lane =
// column: 256-byte row pieces, 8 independent loads in flight per lane), the 4 waves combine in LDS and the block adds
// its 64-bit partials with device-scope atomics: rows / kReduceRows adds per counter.
#ifndef DK_REDUCE_ROWS
#define DK_REDUCE_ROWS 64
#endif
constexpr uint32_t kReduceRows = DK_REDUCE_ROWS;
constexpr uint32_t kReduceCols = 64;
__global__ __launch_bounds__(kBlock) void dk_flow_reduce_kernel(const uint32_t* scratch, uint32_t rows,
                                                                uint32_t row_words, uint32_t row_stride, uint32_t flow_words,
                                                                uint32_t nflows, uint64_t* counts,
                                                                uint64_t* verdicts) {
    __shared__ uint64_t s_part[kWaves][2][kReduceCols];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t w = blockIdx.x * kReduceCols + lane;
    const uint32_t r0 = blockIdx.y * kReduceRows, r1 = min(rows, r0 + kReduceRows);
    uint64_t lo = 0, hi = 0;
    if (w < row_words) {
        uint32_t x[kReduceRows / kWaves];  // all of this lane's loads in flight at once: one memory round trip
#pragma unroll
        for (uint32_t k = 0; k < kReduceRows / kWaves; k++) {
            const uint32_t r = r0 + wv + k * kWaves;
            x[k] = r < r1 ? scratch[(size_t)r * row_stride + w] : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < kReduceRows / kWaves; k++) {
            lo += x[k] & 0xFFFFu;
            hi += x[k] >> 16;
        }
    }
    s_part[wv][0][lane] = lo;
    s_part[wv][1][lane] = hi;
    __syncthreads();
    if (wv != 0 || w >= row_words) return;
#pragma unroll
    for (int k = 1; k < kWaves; k++) {
        lo += s_part[k][0][lane];
        hi += s_part[k][1][lane];
    }
    if (w >= flow_words) {  // verdict column: a plain u32 count
        const uint32_t v = w - flow_words;
        const uint64_t t = lo + (hi << 16);
        if (t && v < DK_V_COUNT) atomicAdd(reinterpret_cast<unsigned long long*>(verdicts + v), (unsigned long long)t);
        return;
    }
    if (lo) atomicAdd(reinterpret_cast<unsigned long long*>(counts + 2 * w), (unsigned long long)lo);
    if (hi && 2 * w + 1 < nflows) atomicAdd(reinterpret_cast<unsigned long long*>(counts + 2 * w + 1), (unsigned long long)hi);
}


// ---------------------------------------------------------------------------------------------------------------------
// TX checksum fill: Ipv4Header::serialize_and_attach (ipv4/header.rs:229-266),
// TcpHeader::serialize_and_attach (tcp/header.rs:397-404) and UdpHeader::serialize_and_attach (udp/header.rs:119-124)
// with offload off, over already-built frames: the IPv4 header checksum (first 20 bytes) and the TCP/UDP checksum
// with the frame's own src/dst in the pseudo-header are written in place. Frames that are not Ethernet/IPv4 with a
// consistent total_length are left untouched; TCP with a bad data offset / UDP shorter than 8 keep only the IPv4 fill
// (oracle dko_tx_fill_checksums). Frames must not overlap.
// ---------------------------------------------------------------------------------------------------------------------
// A 16-bit field write (frames shorter than 64 bytes or not 16-byte aligned; p is 2-byte aligned on the fast path).
// Frames of >= 64 bytes rewrite their whole 64-byte header window instead (tx_finish): full-line writes need no
// partial-write merge below L2 (16-bit stores, nontemporal 16-bit stores and 16-byte block rewrites measured slower,
// round 1-2, profiles/HISTORY.md).
__device__ __forceinline__ void store_be16(uint8_t* p, uint32_t v) {
    *gptr(reinterpret_cast<uint16_t*>(p)) = (uint16_t)bswap16(v);
}

// The checksum pair of dk_tx_checksum_fields (dk_rx.h): IPv4 | L4 << 16, DK_TX_NOT_WRITTEN for a half not filled.
constexpr uint32_t kTxNone = DK_TX_NOT_WRITTEN | (DK_TX_NOT_WRITTEN << 16);
__device__ __forceinline__ uint32_t tx_pair(uint32_t ipc, bool l4, uint32_t c) {
    return ipc | ((l4 ? c : DK_TX_NOT_WRITTEN) << 16);
}

// Byte path (misaligned frames, IHL != 5): lane per frame. Writes the fields in place unless kFields; returns the pair.
template <bool kFields>
__device__ __noinline__ uint32_t tx_slow(uint8_t* f, uint32_t len) {
    if (len < 34) return kTxNone;
    const MemAcc M{f};
    if (M.be16(12) != 0x0800u) return kTxNone;
    const uint32_t hs = (f[14] & 15u) * 4;
    const uint32_t tot = M.be16(16);
    if (hs < 20 || 14 + tot > len || tot < hs) return kTxNone;
    const uint32_t hsum = M.le16(14) + M.le16(16) + M.le16(18) + M.le16(20) + M.le16(22) + M.le16(26) + M.le16(28) +
                          M.le16(30) + M.le16(32);
    const uint32_t ipc = csum_from_residue(be_residue(hsum));
    if (!kFields) {
        f[24] = (uint8_t)(ipc >> 8);
        f[25] = (uint8_t)ipc;
    }
    const uint32_t proto = f[23];
    const uint32_t S = 14 + hs, E = 14 + tot, seg = tot - hs;
    uint32_t cs_at;
    if (proto == 6u) {
        if (seg < 20) return tx_pair(ipc, false, 0);
        const uint32_t doff = (f[S + 12] >> 4) * 4u;
        if (doff < 20 || doff > seg) return tx_pair(ipc, false, 0);
        cs_at = S + 16;
    } else if (proto == 17u) {
        if (seg < 8) return tx_pair(ipc, false, 0);
        cs_at = S + 6;
    } else {
        return tx_pair(ipc, false, 0);
    }
    const uint32_t s = M.sum_le16(S, E) - M.le16(cs_at);  // the field is summed as zero
    const uint32_t src = M.u32(26), dst = M.u32(30);
    const uint32_t pseudo = bswap16(src & 0xFFFFu) + bswap16(src >> 16) + bswap16(dst & 0xFFFFu) + bswap16(dst >> 16) +
                            proto + seg;
    const uint32_t c = csum_from_residue(mod_ffff(be_residue(s) + pseudo));
    if (!kFields) {
        f[cs_at] = (uint8_t)(c >> 8);
        f[cs_at + 1] = (uint8_t)c;
    }
    return tx_pair(ipc, true, c);
}

#ifndef DK_TX_LINE128
#define DK_TX_LINE128 0  // 1: frames of >= 128 bytes on a 128-byte boundary rewrite their whole first 128-byte line
#endif
// A frame's rewritten 64-byte header window, held in registers by the split TX kernel's finish waves until a burst.
constexpr uint32_t kNoWin = 0xFFFFFFFFu;
struct TxWin {
    uint32_t d[16];
    uint32_t off;  // frame offset in the blob; kNoWin: nothing staged
};
// Checksum computation and field writes of one lane's frame from what the streaming left in C and W. kStage: the
// full-window rewrite is handed back in win instead of stored (other writes are stored at once). kFields
// (dk_tx_checksum_fields): nothing is written to the frame; frame i's checksum pair goes to P.fields[i].
template <bool kStage, bool kFields = false>
__device__ __forceinline__ void tx_finish(const TxParams& P, uint32_t lane, const WaveLds& W, uint32_t off,
                                          uint32_t len, const Chunk& C, TxWin& win, uint32_t i = 0, bool live = false) {
    win.off = kNoWin;
    if (!C.inb) {
        if (kFields && live) __builtin_nontemporal_store(kTxNone, gptr(P.fields) + i);
        return;
    }
    uint8_t* f = P.frames + off;
    const RegAcc& R = C.R;
    if (!(C.vec && len >= 34 && ((R.w[3] >> 16) & 0x0Fu) == 5u)) {
        const uint32_t pr = tx_slow<kFields>(f, len);
        if (kFields) __builtin_nontemporal_store(pr, gptr(P.fields) + i);
        return;
    }
    const uint32_t tot = R.be16(16);
    if (R.be16(12) != 0x0800u || 14 + tot > len || tot < 20) {
        if (kFields) __builtin_nontemporal_store(kTxNone, gptr(P.fields) + i);
        return;
    }
    const uint32_t hsum = R.le16(14) + R.le16(16) + R.le16(18) + R.le16(20) + R.le16(22) + R.le16(26) + R.le16(28) +
                          R.le16(30) + R.le16(32);
    const uint32_t ipc = csum_from_residue(be_residue(hsum));
    const uint32_t proto = R.b8(23), seg = tot - 20;
    const bool tcp = proto == 6u;
    const uint32_t doff = (R.b8(46) >> 4) * 4u;
    const bool l4 = tcp ? (seg >= 20 && doff >= 20 && doff <= seg) : (proto == 17u && seg >= 8);
    uint32_t c = 0;
    if (l4) {
        bool resum = false;
        const uint32_t s = seg_sum_fast(C, W, lane, f, (int)(14 + tot), resum) - (tcp ? R.le16(50) : R.le16(40));
        const uint32_t src = R.u32(26), dst = R.u32(30);
        const uint32_t pseudo = bswap16(src & 0xFFFFu) + bswap16(src >> 16) + bswap16(dst & 0xFFFFu) +
                                bswap16(dst >> 16) + proto + seg;
        c = csum_from_residue(mod_ffff(be_residue(s) + pseudo));
    }
    if (kFields) {
        __builtin_nontemporal_store(tx_pair(ipc, l4, c), gptr(P.fields) + i);
        return;
    }
    if (len >= 64 && C.sh == 0) {  // rewrite the whole 64-byte header window: full-line writes, no partial-write merge below L2
        uint32_t d[16];
#pragma unroll
        for (int k = 0; k < 16; k++) d[k] = R.w[k];
        d[6] = (d[6] & 0xFFFF0000u) | bswap16(ipc);
        if (l4 && tcp) d[12] = (d[12] & 0xFFFFu) | (bswap16(c) << 16);
        if (l4 && !tcp) d[10] = (d[10] & 0xFFFF0000u) | bswap16(c);
        if (kStage) {
#pragma unroll
            for (int k = 0; k < 16; k++) win.d[k] = d[k];
            win.off = off;
            return;
        }
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const auto q = gptr(reinterpret_cast<u32x4*>(f));
        if (DK_TX_LINE128 && len >= 128 && (reinterpret_cast<uintptr_t>(f) & 127u) == 0) {
            // the frame's whole first 128-byte line (the L2 line): bytes [64, 128) read back (an L2 hit: kHdrT loads
            // them temporally) so the line goes out whole
            u32x4 e[4];
#pragma unroll
            for (int k = 0; k < 4; k++) e[k] = q[4 + k];
#pragma unroll
            for (int k = 0; k < 4; k++) q[k] = u32x4{d[4 * k], d[4 * k + 1], d[4 * k + 2], d[4 * k + 3]};
#pragma unroll
            for (int k = 0; k < 4; k++) q[4 + k] = e[k];
            return;
        }
#pragma unroll
        for (int k = 0; k < 4; k++) q[k] = u32x4{d[4 * k], d[4 * k + 1], d[4 * k + 2], d[4 * k + 3]};
        return;
    }
    store_be16(f + 24, ipc);
    if (l4) store_be16(f + (tcp ? 50 : 40), c);
}

template <bool kFields>
__device__ __forceinline__ void tx_tile(const TxParams& P, bool live, uint32_t lane, WaveLds& W, uint32_t off,
                                        uint32_t len, uint32_t i) {
    Chunk C;
    stream_chunk<true, true>(P.frames, P.frames_bytes, live, lane, W, off, len, C);
    TxWin win;
    tx_finish<false, kFields>(P, lane, W, off, len, C, win, i, live);
}


// Split TX kernel (large frames), the receive split kernel's structure and hand-off: stream waves 0..3 run phases A+B
// of their chunks into 3 LDS buffers each, finish waves 4..7 compute the checksums and rewrite the header windows, with
// ready / free words instead of a per-period workgroup barrier; the streaming waves never wait on the checksum
// arithmetic or the writes.
template <bool kFields>
__global__ __launch_bounds__(kSplitBlock, 1) void dk_tx_split_kernel(TxParams P) {
    constexpr int kBufs = SplitShape<1>::kBufs;
    __shared__ WaveLds s_buf[kBufs][kWaves];  // [chunk % kBufs][stream wave]
    __shared__ uint32_t s_ready[kWaves][kBufs], s_free[kWaves][kBufs];
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = lane_id();
    const uint32_t wv = tid >> 6, sw = wv & (kWaves - 1);
    const bool finisher = wv >= (uint32_t)kWaves;
    if (tid < kWaves * kBufs) {
        (&s_ready[0][0])[tid] = 0;
        (&s_free[0][0])[tid] = 0;
    }
    __syncthreads();
    const WaveRange r = wave_range(0, P.n, sw, lane);
    const Blob B(P.frames, P.frames_bytes);
    // separate role loops, descriptors one chunk ahead (as dk_rx_split_kernel)
    DescAhead D(P, r, 0);
    if (!finisher) {
        for (uint32_t p = 0; D.have; p++) {
            const uint32_t b = p % kBufs;
            WaveLds& W = s_buf[b][sw];
            const bool live = D.c + r.lane_off < D.lim;
            const uint32_t off = D.off, len = D.len;
            D.next(P, r, p + 1);
            const FrameDesc<true> F(P.frames, P.frames_bytes, live, off, len);
            if (p >= (uint32_t)kBufs) lds_wait_eq(&s_free[sw][b], p - kBufs + 1);  // buffer read out
            const CoopPlan pl = coop_plan(F, lane, off, W);
            coop_stream<true, true>(pl, lane, W, B);
            if (lane == 0) lds_publish(&s_ready[sw][b], p + 1);
        }
    } else {
        for (uint32_t p = 0; D.have; p++) {
            const uint32_t b = p % kBufs;
            WaveLds& W = s_buf[b][sw];
            const uint32_t i = D.c + r.lane_off;
            const bool live = i < D.lim;
            const uint32_t off = D.off, len = D.len;
            D.next(P, r, p + 1);
            const FrameDesc<true> F(P.frames, P.frames_bytes, live, off, len);
            Chunk C;
            small_load(F, B, off, C.R);
            lds_wait_eq(&s_ready[sw][b], p + 1);
            const CoopPlan pl{(uint32_t)__popcll(__ballot(F.big)), 0, 1};
            coop_gather(F, pl, lane, W, C);
            TxWin win;
            tx_finish<false, kFields>(P, lane, W, off, len, C, win, i, live);
            asm volatile("" ::"v"(D.off), "v"(D.len));  // the next descriptors waited for before this chunk's writes
            if (lane == 0) lds_publish(&s_free[sw][b], p + 1);  // after this wave's last read of W (release)
        }
    }
}

// Persistent, same schedule as dk_rx_kernel.
template <bool kFields>
__global__ __launch_bounds__(kBlock, DK_MIN_WAVES) void dk_tx_kernel(TxParams P) {
    __shared__ WaveLds s_wave[kWaves];
    const uint32_t lane = lane_id();
    const uint32_t wv = threadIdx.x >> 6;
    const WaveRange r = wave_range(P.sched, P.n, wv, lane);
    uint32_t c, lim, nc, nlim;
    bool have = r.chunk(0, c, lim);
    uint32_t noff = 0, nlen = 0;
    if (have && c + r.lane_off < lim) {
        noff = P.off[c + r.lane_off];
        nlen = P.len[c + r.lane_off];
    }
    for (uint32_t k = 0; have; k++, c = nc, lim = nlim) {
        const uint32_t i = c + r.lane_off;
        const uint32_t off = noff, len = nlen;
        have = r.chunk(k + 1, nc, nlim);
        if (have && nc + r.lane_off < nlim) {
            noff = P.off[nc + r.lane_off];
            nlen = P.len[nc + r.lane_off];
        }
        tx_tile<kFields>(P, i < lim, lane, s_wave[wv], off, len, i);
    }
}

}  // namespace
}  // namespace dk

int dk_rx_resident_blocks(uint32_t dyn_lds_bytes, uint32_t family) {
    int blocks = 0;
    hipError_t e;
    if (family == dk::kFamilySplit)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, dk::dk_rx_split_kernel<true, 1>, dk::kSplitBlock,
                                                          dyn_lds_bytes);
    else if (family == dk::kFamilySmall)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, dk::dk_rx_small_kernel<true, true>,
                                                          dk::SmallShape<false>::kBlock,
                                                          dyn_lds_bytes);
    else if (family == dk::kFamilySmallUb)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, dk::dk_rx_small_kernel<true, true, true>,
                                                          dk::SmallShape<true>::kBlock, dyn_lds_bytes);
    else
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &blocks, family == dk::kFamilyStaged ? dk::dk_rx_kernel<true, true> : dk::dk_rx_kernel<true, false>,
            dk::kBlock, dyn_lds_bytes);
    return e == hipSuccess ? blocks : 0;
}

uint32_t dk_rx_small_block_waves(bool ub) { return ub ? dk::SmallShape<true>::kWaves : dk::SmallShape<false>::kWaves; }

int dk_launch_rx(const dk::RxParams& p, uint32_t grid, void* stream) {
    if (p.n == 0 || grid == 0) return 0;
    size_t dyn = p.lt_words ? (size_t)(p.lt_off + p.lt_words) * 4
                 : p.flow_mode == dk::kFlowLds ? (size_t)p.flow_words * 4 : 0;
    if (p.ub) dyn = std::max(dyn, (size_t)(p.ub_off + p.ub_words) * 4);
    const hipStream_t s = (hipStream_t)stream;
    const bool opt = p.res.tcp_seq || p.res.tcp_ack || p.res.tcp_win || p.res.tcp_opts || p.path_stats;
    const bool tcp = p.res.tcp_seq || p.res.tcp_ack || p.res.tcp_win;  // the split kernel stages the TCP fields
    const int SMALL_BLOCK = p.ub ? dk::SmallShape<true>::kBlock : dk::SmallShape<false>::kBlock;
    if (p.small && p.ub && p.aligned16 && opt)
        hipLaunchKernelGGL((dk::dk_rx_small_kernel<false, true, true>), dim3(grid), dim3(SMALL_BLOCK), dyn, s, p);
    else if (p.small && p.ub && p.aligned16)
        hipLaunchKernelGGL((dk::dk_rx_small_kernel<false, false, true>), dim3(grid), dim3(SMALL_BLOCK), dyn, s, p);
    else if (p.small && p.ub && opt)
        hipLaunchKernelGGL((dk::dk_rx_small_kernel<true, true, true>), dim3(grid), dim3(SMALL_BLOCK), dyn, s, p);
    else if (p.small && p.ub)
        hipLaunchKernelGGL((dk::dk_rx_small_kernel<true, false, true>), dim3(grid), dim3(SMALL_BLOCK), dyn, s, p);
    else if (p.small && p.aligned16 && opt)
        hipLaunchKernelGGL((dk::dk_rx_small_kernel<false, true>), dim3(grid), dim3(SMALL_BLOCK), dyn, s, p);
    else if (p.small && p.aligned16)
        hipLaunchKernelGGL((dk::dk_rx_small_kernel<false, false>), dim3(grid), dim3(SMALL_BLOCK), dyn, s, p);
    else if (p.small && opt)
        hipLaunchKernelGGL((dk::dk_rx_small_kernel<true, true>), dim3(grid), dim3(SMALL_BLOCK), dyn, s, p);
    else if (p.small)
        hipLaunchKernelGGL((dk::dk_rx_small_kernel<true, false>), dim3(grid), dim3(SMALL_BLOCK), dyn, s, p);
    else if (p.split && p.aligned16 && tcp)
        hipLaunchKernelGGL((dk::dk_rx_split_kernel<false, 1, true>), dim3(grid), dim3(dk::kSplitBlock), dyn, s, p);
    else if (p.split && tcp)
        hipLaunchKernelGGL((dk::dk_rx_split_kernel<true, 1, true>), dim3(grid), dim3(dk::kSplitBlock), dyn, s, p);
    else if (p.split && p.aligned16)
        hipLaunchKernelGGL((dk::dk_rx_split_kernel<false, 1>), dim3(grid), dim3(dk::kSplitBlock), dyn, s, p);
    else if (p.split)
        hipLaunchKernelGGL((dk::dk_rx_split_kernel<true, 1>), dim3(grid), dim3(dk::kSplitBlock), dyn, s, p);
    else if (p.aligned16 && p.stage)
        hipLaunchKernelGGL((dk::dk_rx_kernel<false, true>), dim3(grid), dim3(dk::kBlock), dyn, s, p);
    else if (p.aligned16)
        hipLaunchKernelGGL((dk::dk_rx_kernel<false, false>), dim3(grid), dim3(dk::kBlock), dyn, s, p);
    else if (p.stage)
        hipLaunchKernelGGL((dk::dk_rx_kernel<true, true>), dim3(grid), dim3(dk::kBlock), dyn, s, p);
    else
        hipLaunchKernelGGL((dk::dk_rx_kernel<true, false>), dim3(grid), dim3(dk::kBlock), dyn, s, p);
    if (hipGetLastError() != hipSuccess) return 5;
    if (p.row_words && !p.defer_rows) {
        const dim3 g2((p.row_words + dk::kReduceCols - 1) / dk::kReduceCols,
                      (grid + dk::kReduceRows - 1) / dk::kReduceRows);
        hipLaunchKernelGGL(dk::dk_flow_reduce_kernel, g2, dim3(dk::kBlock), 0, s, p.flow_scratch, grid, p.row_words,
                           p.row_stride, p.flow_words, p.nflows, p.res.flow_counts, p.res.verdict_counts);
        if (hipGetLastError() != hipSuccess) return 5;
    }
    return 0;
}

int dk_launch_reduce(const dk::RowCombine& q, void* stream) {
    if (!q.rows || !q.nrows || !q.row_words) return 0;
    const dim3 g2((q.row_words + dk::kReduceCols - 1) / dk::kReduceCols, (q.nrows + dk::kReduceRows - 1) / dk::kReduceRows);
    hipLaunchKernelGGL(dk::dk_flow_reduce_kernel, g2, dim3(dk::kBlock), 0, (hipStream_t)stream, q.rows, q.nrows,
                       q.row_words, q.row_stride, q.flow_words, q.nflows, q.counts, q.verdicts);
    return hipGetLastError() == hipSuccess ? 0 : 5;
}

int dk_tx_resident_blocks() {
    int blocks = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, dk::dk_tx_kernel<false>, dk::kBlock, 0) != hipSuccess)
        return 0;
    return blocks;
}

int dk_launch_tx(const dk::TxParams& p, uint32_t grid, void* stream) {
    if (p.n == 0 || grid == 0) return 0;
    const hipStream_t s = (hipStream_t)stream;
    if (p.split && p.fields)
        hipLaunchKernelGGL(dk::dk_tx_split_kernel<true>, dim3(grid), dim3(dk::kSplitBlock), 0, s, p);
    else if (p.split)
        hipLaunchKernelGGL(dk::dk_tx_split_kernel<false>, dim3(grid), dim3(dk::kSplitBlock), 0, s, p);
    else if (p.fields)
        hipLaunchKernelGGL(dk::dk_tx_kernel<true>, dim3(grid), dim3(dk::kBlock), 0, s, p);
    else
        hipLaunchKernelGGL(dk::dk_tx_kernel<false>, dim3(grid), dim3(dk::kBlock), 0, s, p);
    return hipGetLastError() == hipSuccess ? 0 : 5;
}
