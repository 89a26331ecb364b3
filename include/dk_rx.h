/*
 * dk_rx.h — C ABI of the MI355X receive-path engine (batch checksum + parse + 4-tuple demux).
 *
 * One call of dk_rx_process() replaces, for a whole batch of received Ethernet frames, the per-frame chain the
 * Demikernel inetstack runs between the physical layer and the socket queues (reference @ /root/reference,
 * paths relative to src/rust/):
 *
 *   PhysicalLayer::receive            inetstack/protocols/layer1/mod.rs:27-33        (input side of the boundary)
 *   SharedLayer2Endpoint::receive     inetstack/protocols/layer2/mod.rs:56-79
 *     Ethernet2Header::parse_and_strip  layer2/ethernet2/header.rs:50-65, protocol.rs:35-41
 *   SharedLayer3Endpoint::receive     inetstack/protocols/layer3/mod.rs:71-120
 *     Ipv4Header::parse_and_strip       layer3/ipv4/header.rs:111-225 (+ compute_checksum :280-301)
 *   Peer::receive_batch               inetstack/protocols/layer4/mod.rs:97-107
 *     TcpPeer::receive                  layer4/tcp/peer.rs:220-255 (TcpHeader::parse_and_strip tcp/header.rs:162-327,
 *                                       tcp_checksum :433-509, SocketId demux)
 *     UdpPeer::receive                  layer4/udp/peer.rs:129-168 (UdpHeader::parse_and_strip udp/header.rs:57-94,
 *                                       UdpHeader::checksum :140-193, SocketAddrV4 demux)
 *   socket.receive(...)               tcp/peer.rs:254, udp/peer.rs:167                (output side of the boundary)
 *
 * Instead of stripping a DemiBuffer in place, the engine writes one result record per frame (struct-of-arrays,
 * below): the verdict (Appendix A of SURVEY.md, first failing check wins, in the reference's order), the parsed
 * 4-tuple, the payload window (what DemiBuffer::adjust/trim leave, runtime/memory/demibuffer.rs:515-590) and the
 * socket the frame demuxes to. Frame memory stays owned by the caller and is never written.
 *
 * Conventions:
 *   - Return values: 0 or a positive errno (demikernel/bindings.rs:314-341 convention). Per-frame failures are not
 *     call failures: they are verdict codes; dk_rx_verdict_errno() maps them back to the reference's errno.
 *   - IPv4 addresses are uint32_t whose in-memory bytes are the address octets (s_addr / Ipv4Addr::octets order).
 *     Ports are host-order uint16_t values (the reference's u16 port).
 *   - Not re-entrant per context; one host thread per context (demikernel/bindings.rs:33-35). GPU work is
 *     ordered on the caller's stream. A context keeps its launch scratch per stream (up to 8 streams; past that the
 *     least recently used stream's scratch is taken over behind that stream's last launch), so batches issued on
 *     different streams of one context may run concurrently; counters they share are added atomically. A stream
 *     handed to dk_rx_process must stay valid while the context lives, or be released with dk_rx_stream_forget
 *     before it is destroyed (a later stream may reuse its handle value).
 *   - Tuning: the engine's choices (kernel family, grid) follow the batch; overrides are diagnostics set only by an
 *     explicit dk_diag_rx_set_tuning call (dk_diag.h). The process environment is never read.
 *   - No torch / HIP types in signatures: streams are passed as void* (a hipStream_t, NULL = default stream).
 */
#ifndef DK_RX_H
#define DK_RX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DK_RX_ABI_VERSION 4u

/* Frames at an address that is a multiple of this take the vectorised path (16-byte aligned frames directly, other
 * even addresses — e.g. NIC buffers with the Ethernet header at 2 mod 16 — through a realigned header window); any
 * other address is still processed (bit-exact), by a per-lane byte-load path. */
#define DK_RX_FAST_ALIGN 2u

/* dk_rx_batch.flags */
#define DK_RX_BATCH_ALIGNED16 1u /* hint: frames are (mostly) at 16-byte aligned addresses; the engine launches its
                                    instantiation without the realignment path (other frames then take the byte path,
                                    still bit-exact) */

#define DK_RX_BATCH_DEFER_COUNTS 2u /* leave this batch's flow / verdict counter contributions pending on `stream`
                                       (per-workgroup partial rows in the context's scratch): the next dk_rx_process on
                                       the same context and stream adds them to THIS batch's counters inside its own
                                       kernel, or dk_rx_counts_flush does. Saves the dependent second launch
                                       (dk_flow_reduce_kernel) per batch when batches follow each other; the counters
                                       are current once a later launch on the stream, or a flush, has run. Ignored by
                                       dk_rx_process_host (synchronous, counters current at return).
                                       Scope: verdict_counts are always deferred; flow_counts only while the flow
                                       table has <= DK_RX_MAX_DEFERRED_FLOWS entries. Larger tables count flows with
                                       device atomics inside the launch itself, so a caller that double-buffers the
                                       counters (reads one set while launches add to the other) must treat such a
                                       launch as writing its flow_counts immediately.
                                       Lifetime: the pending contributions keep raw pointers to this call's
                                       flow_counts / verdict_counts arrays; they must stay allocated until the next
                                       launch on the stream, a flush, dk_rx_stream_forget or dk_rx_ctx_destroy. */
#define DK_RX_MAX_DEFERRED_FLOWS 32768u /* flow tables up to this size keep per-workgroup flow rows (deferrable) */

/* Largest frame blob of one batch (bytes): offsets are u32 and the engine keeps 256 bytes of the 32-bit range for its
 * out-of-range loads. */
#define DK_RX_MAX_BLOB 0xFFFFFF00ull

/* flow_id value for frames that do not demux to a socket. */
#define DK_FLOW_NONE 0xFFFFFFFFu

/* ---------------------------------------------------------------------------------------------------------------
 * Verdicts: one per frame. Order and errno follow SURVEY.md Appendix A / the reference lines cited.
 * ------------------------------------------------------------------------------------------------------------- */
enum dk_verdict {
    DK_V_OK_TCP = 0,          /* delivered: socket.receive (tcp/peer.rs:254)                                  */
    DK_V_OK_UDP = 1,          /* delivered: socket.receive (udp/peer.rs:167)                                  */
    DK_V_ARP = 2,             /* diverted to ARP peer (layer3/mod.rs:75-78); its PDU parses (arp/header.rs:80-111) */
    DK_V_ICMP = 3,            /* diverted to ICMPv4 peer (layer3/mod.rs:109-112); header parses
                                 (icmpv4/header.rs:47-66)                                                       */
    DK_V_IPV6 = 4,            /* dropped, IPv6 unsupported (layer3/mod.rs:116)                                */
    DK_V_ETH_SHORT = 5,       /* E1  len < 14 (ethernet2/header.rs:51-53)                        EBADMSG      */
    DK_V_ETH_TYPE = 6,        /* E2  unknown ethertype (ethernet2/protocol.rs:35-41)             ENOTSUP      */
    DK_V_IP_SHORT = 7,        /* I1  datagram < 20 B (ipv4/header.rs:113-115)                    EBADMSG      */
    DK_V_IP_VERSION = 8,      /* I2  version != 4 (:117-120)                                     ENOTSUP      */
    DK_V_IP_IHL_SMALL = 9,    /* I3  IHL*4 < 20 (:123-127)                                       EBADMSG      */
    DK_V_IP_HDR_TRUNC = 10,   /* I4  datagram < IHL*4 (:128-130)                                 EBADMSG      */
    DK_V_IP_TOTLEN_SMALL = 11,/* I5  total_length < IHL*4 (:145-148)                             EBADMSG      */
    DK_V_IP_TOTLEN_BIG = 12,  /* I6  total_length > datagram (:150-152)                          EBADMSG      */
    DK_V_IP_EVIL = 13,        /* I7  RFC 3514 evil bit (:168-172)                                EBADMSG      */
    DK_V_IP_MF = 14,          /* I8  more-fragments (:175-178)                                   ENOTSUP      */
    DK_V_IP_FRAGOFF = 15,     /* I9  fragment offset != 0 (:180-185)                             ENOTSUP      */
    DK_V_IP_TTL = 16,         /* I10 TTL == 0 (:187-190)                                         EBADMSG      */
    DK_V_IP_PROTO = 17,       /* I11 protocol not in {1,6,17} (:192, ip/protocol.rs:34-41)       ENOTSUP      */
    DK_V_IP_CSUM_FFFF = 18,   /* I12 stored header checksum 0xFFFF (:194-197)                    EBADMSG      */
    DK_V_IP_CSUM = 19,        /* I13 header checksum mismatch (:198-200)                         EBADMSG      */
    DK_V_IP_DST = 20,         /* F1  dst not local and not broadcast (layer3/mod.rs:91-95)       dropped      */
    DK_V_IP_SRC = 21,         /* F2  src broadcast/multicast/unspecified (layer3/mod.rs:98-105)  dropped      */
    DK_V_TCP_SHORT = 22,      /* T1  segment < 20 B (tcp/header.rs:168-170)                      EBADMSG      */
    DK_V_TCP_DOFF_TRUNC = 23, /* T2  segment < data offset (:171-174)                            EBADMSG      */
    DK_V_TCP_DOFF_SMALL = 24, /* T3  data offset < 20 (:175-177)                                 EBADMSG      */
    DK_V_TCP_CSUM = 25,       /* T4  checksum mismatch (:203-207)                                EBADMSG      */
    DK_V_TCP_OPT = 26,        /* T5  malformed option / > 5 options (:215-302)                   EBADMSG      */
    DK_V_TCP_OPT_EIO = 27,    /* T5  truncated option read, io::Error -> Fail (runtime/fail.rs:61-67) EIO     */
    DK_V_TCP_NOSOCK = 28,     /* no Active(local,remote) and no Passive(local) (tcp/peer.rs:241-251) dropped  */
    DK_V_UDP_SHORT = 29,      /* U1  segment < 8 B (udp/header.rs:64-66)                         EBADMSG      */
    DK_V_UDP_LEN = 30,        /* U2  length field != segment length (:72-75)                     EBADMSG      */
    DK_V_UDP_CSUM = 31,       /* U3  checksum mismatch (:78-88)                                  EBADMSG      */
    DK_V_UDP_NOSOCK = 32,     /* no (local_ip,port) and no (0.0.0.0,port) (udp/peer.rs:147-165) dropped       */
    DK_V_BAD_DESC = 33,       /* descriptor outside the frame blob (this ABI, not the reference)  EINVAL       */
    /* Diverted frames whose control-plane parse fails. The reference hands these to the ARP /
     * ICMPv4 peer, whose background loop drops them with a warning (arp/peer.rs:140-147, icmpv4/peer.rs:114-121). */
    DK_V_ARP_SHORT = 34,      /* ARP PDU < 28 B (arp/header.rs:81-83)                            EBADMSG      */
    DK_V_ARP_UNSUP = 35,      /* HTYPE/PTYPE/HLEN/PLEN/operation unsupported (:85-100, :161-166) ENOTSUP      */
    DK_V_ICMP_SHORT = 36,     /* ICMPv4 message < 8 B (icmpv4/header.rs:48-50)                   EBADMSG      */
    DK_V_ICMP_CSUM = 37,      /* ICMPv4 checksum mismatch (:55-57, protocols/mod.rs:47-71)       EBADMSG      */
    DK_V_ICMP_TYPE = 38,      /* type byte not a known Icmpv4Type2 (icmpv4/protocol.rs:35-58)    EBADMSG      */
    DK_V_COUNT = 39
};

/* ---------------------------------------------------------------------------------------------------------------
 * Configuration: the hot-path-relevant subset of the reference's YAML config (demikernel/config.rs:115, :340-346).
 * ------------------------------------------------------------------------------------------------------------- */
typedef struct dk_rx_cfg {
    uint32_t local_ipv4;              /* demikernel.local_ipv4_addr (octet order, see conventions)         */
    uint8_t tcp_rx_checksum_offload;  /* inetstack_config.tcp_checksum_offload (config/tcp.rs:48-51)       */
    uint8_t udp_rx_checksum_offload;  /* inetstack_config.udp_checksum_offload (config/udp.rs:26-30)       */
    uint16_t reserved;
    int32_t device;                   /* HIP device ordinal the context lives on                          */
} dk_rx_cfg;

/* Socket table entry. Mirrors SocketId::{Active(local, remote), Passive(local)} (runtime/network/socket/mod.rs:22-26)
 * for TCP, and the UdpPeer `addresses` key SocketAddrV4 (udp/peer.rs:38) for UDP. flow_id = index in the array. */
enum dk_flow_kind { DK_FLOW_TCP_ACTIVE = 1, DK_FLOW_TCP_PASSIVE = 2, DK_FLOW_UDP = 3 };

typedef struct dk_flow {
    uint32_t kind;         /* enum dk_flow_kind                                                    */
    uint32_t local_ip;     /* local address (UDP: may be 0.0.0.0 = wildcard bind)                  */
    uint32_t remote_ip;    /* Active only, else 0                                                  */
    uint16_t local_port;   /* host order                                                           */
    uint16_t remote_port;  /* Active only, else 0                                                  */
} dk_flow;                 /* 16 bytes */

/* A batch of received frames: the data the reference receives as ArrayVec<DemiBuffer, RECEIVE_BATCH_SIZE>
 * (runtime/network/consts.rs:42), widened to any n. Frame i occupies frames[off[i] .. off[i]+len[i]).
 * For dk_rx_process all pointers are device pointers (HBM-resident batch). */
typedef struct dk_rx_batch {
    const uint8_t* frames;    /* frame blob base                                                       */
    uint64_t frames_bytes;    /* blob size in bytes (<= DK_RX_MAX_BLOB); frames outside it: DK_V_BAD_DESC */
    const uint32_t* off;      /* [n] byte offset of each frame in the blob                             */
    const uint16_t* len;      /* [n] frame length: Ethernet header included, FCS excluded              */
    uint32_t n;
    uint32_t flags;           /* DK_RX_BATCH_* hints, 0 = none                                         */
} dk_rx_batch;

/* TCP options of one segment: the reference's option list [TcpOptions2; 5] (tcp/header.rs:26-41, filled in header
 * order by parse_and_strip :215-302; NoOperation and EndOfOptionsList are not entries). */
enum dk_tcp_opt_kind {
    DK_TCPOPT_MSS = 2,      /* MaximumSegmentSize(u16)                                   */
    DK_TCPOPT_WS = 3,       /* WindowScale(u8)                                           */
    DK_TCPOPT_SACK_OK = 4,  /* SelectiveAcknowlegementPermitted                          */
    DK_TCPOPT_SACK = 5,     /* SelectiveAcknowlegement { num_sacks, sacks: [_; 4] }       */
    DK_TCPOPT_TS = 8        /* Timestamp { sender_timestamp, echo_timestamp }             */
};
typedef struct dk_tcp_opt {
    uint8_t kind;   /* enum dk_tcp_opt_kind                                                              */
    uint8_t u8;     /* WS: the shift count; SACK: num_sacks (1..4)                                         */
    uint16_t u16;   /* MSS: the segment size; SACK: index of its first block in dk_tcp_opts.sack            */
    uint32_t v0;    /* TS: sender_timestamp                                                                */
    uint32_t v1;    /* TS: echo_timestamp                                                                  */
} dk_tcp_opt;       /* 12 bytes */
typedef struct dk_tcp_opts {
    uint32_t num;          /* entries in opt[] (0..5)                                                       */
    dk_tcp_opt opt[5];
    uint32_t sack[4][2];   /* SACK blocks (begin, end) of every SACK entry, in order (40 option bytes hold <= 4) */
} dk_tcp_opts;             /* 96 bytes; unused entries and blocks are zero */

/* Per-frame results, struct-of-arrays, one element per frame. Required arrays: meta, src_ip, ports, payload, flow_id
 * (20 bytes per frame). Optional (NULL = not written): dst_ip, tcp_seq, tcp_ack, tcp_win, flow_counts,
 * verdict_counts, tcp_opts. (ABI 3: dst_ip became optional. What a delivered frame goes on to, socket.receive, never sees the
 * destination address — tcp/peer.rs:254 passes (src_ip, header, payload), udp/peer.rs:167 (remote, payload) — and
 * it is the configured local address or 255.255.255.255 for every delivered frame, layer3/mod.rs:91-95.)
 *
 *  TCP / UDP (DK_V_OK_*, DK_V_*_NOSOCK):
 *  meta     = verdict | ip_protocol << 8 | tcp byte 13 (CWR..FIN) << 16 | tcp byte 12 (data offset, NS) << 24
 *  ports    = src_port | dst_port << 16
 *  payload  = payload_off | payload_len << 16     (payload_off counted from the frame start)
 *  tcp_win  = window | urgent_pointer << 16
 *  ICMPv4 (DK_V_ICMP): meta = verdict | 1 << 8 | type << 16 | code << 24; src_ip / dst_ip from the IPv4 header;
 *           ports = rest-of-header words: id | seq_num << 16 (echo request / reply); payload = the message after
 *           the 8-byte header (what Icmpv4Header::parse_and_strip leaves).
 *  ARP (DK_V_ARP): meta = verdict | operation << 16; src_ip = sender protocol address, dst_ip = target protocol
 *           address; payload = 14 | (len - 14) << 16 (the buffer ArpPeer::receive takes). The sender / target
 *           hardware addresses are frame bytes [22, 28) and [32, 38).
 * For every other verdict the fields are 0 (flow_id DK_FLOW_NONE).
 * flow_counts[flow_id] and verdict_counts[verdict] are incremented (they accumulate across calls); with
 * DK_RX_BATCH_DEFER_COUNTS the increments land one launch later (see the flag). */
typedef struct dk_rx_results {
    uint32_t* meta;
    uint32_t* src_ip;
    uint32_t* dst_ip;
    uint32_t* ports;
    uint32_t* payload;
    uint32_t* flow_id;
    uint32_t* tcp_seq;
    uint32_t* tcp_ack;
    uint32_t* tcp_win;
    uint64_t* flow_counts;     /* [number of flows in the table] */
    uint64_t* verdict_counts;  /* [DK_V_COUNT]                   */
    dk_tcp_opts* tcp_opts;     /* [n], optional: written only for frames whose TCP segment carries options (data
                                  offset > 5) and parses (verdict DK_V_OK_TCP or DK_V_TCP_NOSOCK); every other
                                  frame's record is left untouched (dk_rx_process_host: zeroed). Saves the LibOS a
                                  CPU re-parse of SYN / SYN-ACK option lists (active_open.rs / passive_open.rs
                                  consume them). */
} dk_rx_results;

typedef struct dk_rx_ctx dk_rx_ctx;

/* Create / destroy a receive context on cfg->device. Replaces the receive-side state SharedInetStack::new builds
 * (inetstack/mod.rs:69-93): local address, offload flags, socket tables. Returns 0, EINVAL, ENOMEM or EIO. */
int dk_rx_ctx_create(const dk_rx_cfg* cfg, dk_rx_ctx** out);
void dk_rx_ctx_destroy(dk_rx_ctx* ctx);

/* Install the socket table (host array of n entries; copied to HBM: Active connections as an open-addressing hash
 * table, UDP binds and TCP listeners as a port-indexed table for the configured local address and 0.0.0.0 — the only
 * addresses the reference looks them up with). Plays the role of TcpPeer::addresses / UdpPeer::addresses (tcp/peer.rs,
 * udp/peer.rs:38). Duplicate keys: the last entry wins, as with HashMap::insert. Returns 0, EINVAL (bad kind) or
 * ENOMEM. Synchronous. */
int dk_rx_flow_table_set(dk_rx_ctx* ctx, const dk_flow* flows, uint32_t n);
uint32_t dk_rx_flow_table_size(const dk_rx_ctx* ctx);

/* Process one HBM-resident batch on `stream` (hipStream_t or NULL). Asynchronous: returns after the launch.
 * Returns 0, EINVAL (null required pointer, frames_bytes > DK_RX_MAX_BLOB) or EIO (launch failure). */
int dk_rx_process(dk_rx_ctx* ctx, const dk_rx_batch* batch, const dk_rx_results* res, void* stream);

/* Add the counter contributions a DK_RX_BATCH_DEFER_COUNTS launch left pending on `stream` to that launch's
 * flow_counts / verdict_counts: one small launch on `stream` (nothing when nothing is pending). Asynchronous; the counters
 * are current for work ordered after it on `stream`. Also done implicitly by the next dk_rx_process on the stream (in its
 * kernel), dk_rx_stream_forget and dk_rx_ctx_destroy. Returns 0 or EIO. */
int dk_rx_counts_flush(dk_rx_ctx* ctx, void* stream);

/* Release the context's launch scratch of `stream` before the caller destroys that stream: flushes pending counters,
 * waits for the stream's work, then frees the slot for another stream. Returns 0 (also when the context never saw the
 * stream) or EIO. */
int dk_rx_stream_forget(dk_rx_ctx* ctx, void* stream);

/* Process a batch that lives in host memory (a NIC ring / raw-socket buffer / DPDK mempool): the kernel, with
 * descriptors copied in and results copied back to host arrays, over the context's own streams. Synchronous.
 * batch/res pointers are host pointers. Frames in page-locked, GPU-mapped memory (hipHostMalloc, hipHostRegister)
 * are read by the kernel in place over PCIe, one launch for the batch (zero-copy; DK_RX_HOST_ZC=0 at context creation
 * turns it off); other memory is staged through chunked H2D copies pipelined over 3 streams. flow/verdict counts are
 * host arrays too. chunk_frames = frames per pipeline stage (0 = default: 65,536 staged, the whole batch zero-copy).
 * Returns 0, EINVAL, ENOMEM or EIO.
 * (dk_rx_process itself also accepts a batch whose frames pointer is the device alias of mapped host memory: the
 * DPDK-mbuf path of INTEGRATION.md.) */
int dk_rx_process_host(dk_rx_ctx* ctx, const dk_rx_batch* batch, const dk_rx_results* res, uint32_t chunk_frames);

/* Multi-GPU packet shards: sum res->flow_counts[0 .. flow table size) and
 * res->verdict_counts[0 .. DK_V_COUNT) (device arrays; either may be NULL) over every rank of `nccl_comm` (an
 * ncclComm_t, e.g. from dk_comm.h), in place, as one grouped ncclAllReduce(ncclUint64, ncclSum) on `stream` — the only
 * collective of the receive path (RCCL over xGMI; per-frame results stay on their GPU). Every rank must call it with
 * the same flow table size. Asynchronous. Returns 0, EINVAL or EIO. */
int dk_rx_flow_counts_allreduce(dk_rx_ctx* ctx, const dk_rx_results* res, void* nccl_comm, void* stream);
/* The same into separate device arrays (flow_out[flow table size], verdict_out[DK_V_COUNT]; required where the
 * corresponding res array is set): each rank keeps accumulating its own counters across batches and reads the
 * node-wide totals from the outputs, with no per-batch reset of its counters. */
int dk_rx_flow_counts_allreduce_to(dk_rx_ctx* ctx, const dk_rx_results* res, uint64_t* flow_out,
                                   uint64_t* verdict_out, void* nccl_comm, void* stream);

/* TX side: compute and store the IPv4 header checksum and the TCP/UDP checksum of every
 * frame in place, as Ipv4Header/TcpHeader/UdpHeader::serialize_and_attach do (ipv4/header.rs:229-266,
 * tcp/header.rs:330-405, udp/header.rs:97-130) with tx offload off. The pseudo-header uses the frame's own IPv4
 * src/dst. Frames that are not Ethernet/IPv4 with IHL >= 5 and TCP/UDP are left untouched. Device pointers, async. */
int dk_tx_checksum(uint8_t* frames, uint64_t frames_bytes, const uint32_t* off, const uint16_t* len, uint32_t n,
                   void* stream);

/* The same checksums returned instead of written (for a host that builds the headers itself, as serialize_and_attach
 * does, and patches two u16s per frame): the frames are only read, and fields[i] (u32, device memory) =
 * ipv4 | l4 << 16, each half the value dk_tx_checksum would store big-endian at frame bytes 24..25 (IPv4 header
 * checksum) and at the TCP (S + 16) / UDP (S + 6) checksum, S = 14 + IHL * 4; DK_TX_NOT_WRITTEN (0xFFFF, never a
 * computed checksum: the fold maps a zero residue to 0) for a half the in-place fill leaves untouched. 4 bytes written per
 * frame instead of a 64-byte header line. Device pointers, async. */
#define DK_TX_NOT_WRITTEN 0xFFFFu
int dk_tx_checksum_fields(const uint8_t* frames, uint64_t frames_bytes, const uint32_t* off, const uint16_t* len,
                          uint32_t n, uint32_t* fields, void* stream);

/* Introspection. */
const char* dk_rx_verdict_name(int verdict);
int dk_rx_verdict_errno(int verdict); /* errno the reference returns for this verdict; 0 for deliver/divert/drop */
uint32_t dk_rx_abi_version(void);
/* Content hash of the sources, headers and compiler flags this library was built from (hex; "unversioned" for a build
 * outside __graft_entry__.build()), so a test run can prove which build it loaded. */
const char* dk_rx_build_id(void);
int dk_rx_device_count(void);

#ifdef __cplusplus
}
#endif

#endif /* DK_RX_H */
