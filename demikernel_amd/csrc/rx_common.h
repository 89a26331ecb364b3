// rx_common.h — definitions shared by the host driver (rx_host.cpp) and the HIP kernels (rx_kernels.hip).
#pragma once

#include <stdint.h>

#include "../../include/dk_diag.h"
#include "../../include/dk_rx.h"

#if defined(__HIPCC__)
#define DK_HD __host__ __device__ __forceinline__
#else
#define DK_HD inline
#endif

namespace dk {

// Device socket table: open addressing, linear probing, power-of-two capacity >= 8 * entries (at most 2^26 slots,
// and >= 2 * entries). A wave waits for its worst lane's probe walk (one dependent load per displaced slot): at load
// 0.5 that was 3-6 dependent round trips per 64-frame chunk at 1024 flows, at 0.125 mostly one (C3 -8 %, IMIX -3 %;
// a two-choice cuckoo table, two loads and one round trip always, measured C3 -7 % but IMIX +3 %: DESIGN.md §8).
// Slot = 16 bytes, one dwordx4 load per probe:
//   x = kind << 24 | flow_id   (0 = empty; kind in 1..3, flow_id < 2^24)
//   y = local_ip, z = remote_ip, w = local_port | remote_port << 16
// Keys are normalised exactly as the reference builds them for lookups:
//   TCP Active  (1, local_ip, remote_ip, local_port, remote_port)  SocketId::Active(local, remote)
//   TCP Passive (2, local_ip, 0,         local_port, 0)            SocketId::Passive(local)
//   UDP         (3, ip or 0.0.0.0, 0,    port,       0)            SocketAddrV4 (udp/peer.rs:38)
// UDP binds and TCP listeners are keyed by a port alone once the address is fixed: every lookup asks for the configured
// local address or 0.0.0.0, so they live in a direct-indexed port table (one exact load, no probe walk) after the
// Active slots: words [kPortUdpLocal + port] (UDP bound to local_ipv4), [kPortUdpAny + port] (UDP on 0.0.0.0),
// [kPortTcpPassive + port] (Passive on local_ipv4) hold the flow id or DK_FLOW_NONE. Entries for other local
// addresses can never match a lookup and are not stored. The Active table holds only Active connections.
constexpr uint32_t kPortUdpLocal = 0, kPortUdpAny = 1u << 16, kPortTcpPassive = 2u << 16;
constexpr uint32_t kPortTabWords = 3u << 16;
constexpr uint32_t kMaxFlows = (1u << 24) - 1;
constexpr uint32_t kMinTableSlots = 16;

DK_HD uint32_t flow_hash(uint32_t kind, uint32_t lip, uint32_t rip, uint32_t ports) {
    uint32_t h = kind * 0x9E3779B1u;
    h ^= lip;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h ^= rip;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    h ^= ports;
    h *= 0x27D4EB2Fu;
    h ^= h >> 15;
    return h;
}

// LDS copy of the Active table (round 3). Under a full frame stream a lane's table load waits behind the streaming
// loads in the vector-memory queues (IMIX: 13.6 us of 151 without the load), while LDS latency does not.
// The Active connections a lookup can find (local_ip = the configured address, as every reference lookup asks) are
// placed by a minimal perfect hash (hash and displace): N keys, B = ceil(N / 4) buckets, bucket b = mulhi(h, B) of the
// key's flow_hash h; the bucket's displacement d (chosen on the host, smallest first) puts each key at slot
// mulhi(fmix32(h ^ lt_disp(d)), N). One slot per key, so the table is 12 bytes per connection, laid out as u32 words
// [remote_ip x N][local_port | remote_port << 16 x N][flow_id x N][d x B] (padded to 16 bytes). A lookup is two
// dependent LDS reads (d, then the slot) and one key compare: a key that is not in the table lands on some other key's
// slot and fails the compare. The host uses it when it fits the kernel family's LDS without costing occupancy.
constexpr uint32_t kLtMaxKeys = 4096;
DK_HD uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}
DK_HD uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
DK_HD uint32_t lt_bucket(uint32_t h, uint32_t nb) { return mulhi32(h, nb); }
DK_HD uint32_t lt_slot(uint32_t h, uint32_t d, uint32_t n) { return mulhi32(fmix32(h ^ (d * 0x9E3779B1u + 0x7F4A7C15u)), n); }
DK_HD uint32_t lt_words(uint32_t n, uint32_t nb) { return (3 * n + nb + 3) & ~3u; }

// UDP binds on the configured address as a compact table (round 5). The port table's local-bind words span 256 KB:
// binds on scattered ports put nearly every lane's load on its own line (C3 with its 1,024 binds on random ports:
// that load was 14 % of the launch, against 1.4 % with consecutive ports; ablation, session r05zl). The compact table
// is a two-choice cuckoo table of 2^k buckets of two words (load <= 1/2: 8 KB for 1,024 binds), word = port |
// flow_id << 16 (flow ids < 0xFFFF; kUbEmpty empty); a port's two buckets come from one hash, h & mask and
// (h >> 16) & mask, read together (two 8-byte LDS reads). The small-frame kernel has an instantiation that copies it
// into LDS at the start and looks binds up there; the host launches it when the binds' port-table words span more
// lines than the table and the copy costs no occupancy (C3 on random ports -10 %, session r05zo). Everything else
// reads the port table.
constexpr uint32_t kUbMaxBinds = 1u << 15;  // 2^15 buckets at most: the bucket indices are 16-bit halves of h
constexpr uint32_t kUbEmpty = 0xFFFFFFFFu;
DK_HD uint32_t ub_hash(uint32_t port, uint32_t seed) { return fmix32(port * 0x9E3779B1u + seed); }
DK_HD bool ub_hit(uint32_t e, uint32_t port) { return ((e ^ port) & 0xFFFFu) == 0 && (e >> 16) != 0xFFFFu; }
// The flow bound to `port` from the words of its two buckets (s.x, s.y: the first; s.z, s.w: the second), or
// DK_FLOW_NONE.
DK_HD uint32_t ub_pick(uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1, uint32_t port) {
    return ub_hit(a0, port) ? a0 >> 16 : ub_hit(a1, port) ? a1 >> 16 : ub_hit(b0, port) ? b0 >> 16
         : ub_hit(b1, port) ? b1 >> 16 : DK_FLOW_NONE;
}

// Per-flow counting strategy (chosen per launch by the host).
constexpr uint32_t kFlowNone = 0;    // no flow_counts requested
constexpr uint32_t kFlowLds = 1;     // per-workgroup packed-u16 LDS histogram + scratch rows, combined per launch
constexpr uint32_t kFlowGlobal = 2;  // per-frame u64 global atomics (tables too large for LDS)
constexpr uint32_t kMaxLdsFlowWords = 16384;  // 64 KiB of LDS -> up to 32768 flows on the LDS path
static_assert(2 * kMaxLdsFlowWords == DK_RX_MAX_DEFERRED_FLOWS, "dk_rx.h: flow counts defer on the LDS path only");
constexpr uint32_t kVerdictWords = (DK_V_COUNT + 3) & ~3u;  // verdict histogram columns of a scratch row
constexpr uint32_t kMaxTilesPerBlockLds = 255;  // 255 * 256 frames < 65536: a packed u16 counter never wraps
constexpr uint32_t kRowAlignWords = 32;  // counter rows padded to whole 128-byte lines

// Counter rows a previous launch on the same stream left pending (DK_RX_BATCH_DEFER_COUNTS), added to that launch's
// counters inside this launch by waves with nothing else to do: the split kernel's finish waves before their first
// chunk (their stream waves are filling the pipeline), every other kernel's waves with the fewest chunks after their
// last one (round-robin chunks leave the highest-numbered waves one chunk short). Blocks of 64 columns x rpb rows are
// assigned statically, block j to the j-th of those waves (mod their count): no atomics on a shared word (a ticket word
// taken by every wave measured 3x slower at C3: ~6,000 same-address atomics per launch serialise at the memory side).
// rpb: 16 rows for narrow rows (many small blocks for many waves), 64 for wide ones (C5's 10k flows: 4x fewer u64
// atomics). kCombRows = the loads per lane in flight together.
constexpr uint32_t kCombRows = 16;
constexpr uint32_t kCombCols = 64;
struct RowCombine {
    const uint32_t* rows;  // nullptr: nothing pending
    uint32_t nrows, row_words, row_stride, flow_words, nflows;
    uint64_t* counts;      // the pending launch's flow_counts / verdict_counts (either may be nullptr)
    uint64_t* verdicts;
    uint32_t rpb;          // rows per block
    uint32_t ncolblk, nblk;
};

// Dynamic tail of the staged kernel (round 5). With round-robin chunks a wave's chunk count is fixed and its chunks'
// sizes are random (IMIX), so the waves finish over ~25 us and the launch waits for the slowest. The first tail_ks
// rounds stay round-robin (chunk j = wave + k * nwaves: the grid sweeps the blob in address order); the remaining
// chunks are split into tail_pools (<= kTailXcds) pools, one per group of workgroups that share an XCD, handed out by
// one counter per pool, each on its own 256-byte span (one shared line serialises every grab at one memory channel,
// round 4: +42 %). A wave grabs from its own pool only; each grab is issued a chunk before its descriptors are
// needed, so its latency is hidden. A launch zeroes the counter set the stream's next tail launch will use (two sets
// per stream slot, alternating).
constexpr uint32_t kTailXcds = 8;
constexpr uint32_t kStagedWaves = 4;  // waves per workgroup of the staged kernel (the host's tail boundary uses it too)
constexpr uint32_t kTailStride = 64;  // words between counters
constexpr uint32_t kTailSetWords = kTailXcds * kTailStride;

// Kernel parameters (passed by value).
struct RxParams {
    const uint8_t* frames;
    uint64_t frames_bytes;
    const uint32_t* off;
    const uint16_t* len;
    uint32_t n;
    uint32_t local_ip;
    uint32_t tcp_offload;
    uint32_t udp_offload;
    const uint32_t* table;  // Active slots as 4 x u32
    uint32_t table_mask;
    const uint32_t* port_tab;  // kPortTabWords: UDP / Passive flow ids by port
    const uint32_t* lt;        // the LDS Active table's words in global memory (copied into LDS at the kernel start)
    uint32_t lt_words;         // 0: Active lookups probe the global table instead
    uint32_t lt_off;           // word offset of the LDS copy in dynamic LDS (after the flow histogram)
    uint32_t lt_n, lt_b;       // keys, buckets
    const uint32_t* ub;  // the compact UDP bind table (above) the small-frame kernel copies to dynamic LDS at word
                         // ub_off and reads there; nullptr: the port table
    uint32_t ub_off, ub_words, ub_mask, ub_seed;  // ub_words = 2 (ub_mask + 1)
    uint32_t nflows;
    uint32_t flow_mode;      // kFlow*
    uint32_t flow_words;     // kFlowLds: ceil(nflows / 2), else 0
    uint32_t row_words;      // words per workgroup row of flow_scratch: flow_words + (verdict_counts ? kVerdictWords : 0)
    uint32_t row_stride;     // row_words rounded up to kRowAlignWords
    uint32_t* flow_scratch;  // [grid][row_stride]: the packed-u16 flow histogram (kFlowLds), then the u32 verdict
                             // histogram; nullptr when row_words == 0. dk_flow_reduce_kernel (or, deferred, the
                             // stream's next launch) adds the rows up.
    uint64_t* defer;         // small-frame kernel: [ceil(n / 64)] masks of the frames each 64-frame chunk left to the
                             // general path after its main loop
    unsigned long long* path_stats;  // nullable: [4] frames per path (dk_diag.h)
    uint32_t sched;          // 0: round-robin 256-frame tiles; 1: one contiguous share per wave (tuning)
    uint32_t aligned16;      // DK_RX_BATCH_ALIGNED16 hint: launch the instantiation without the realignment path
    uint32_t stage;          // launch the instantiation that stages result stores in registers (large frames)
    uint32_t split;          // launch the split (stream waves / finish waves) kernel (large frames)
    uint32_t small;          // launch the small-frame kernel (minimum-size frames)
    uint32_t small_kmin;     // small-frame kernel: whole chunks per wave (ceil(n / 64) / waves of the grid)
    uint32_t defer_rows;     // leave this launch's counter rows pending (no dk_flow_reduce_kernel after it)
    uint32_t tail_ks;        // staged kernel: round-robin rounds per wave before the dynamic tail (0: none)
    uint32_t tail_pools;     // pools of the tail (8, 4, 2 or 1: divides the grid); workgroup b grabs from b mod this
    uint32_t* tail_ctr;      // this launch's kTailXcds grab counters (zero at launch), nullptr: no dynamic tail
    uint32_t* tail_next;     // the counter set the stream's next tail launch uses: zeroed by this launch
    RowCombine comb;         // a previous launch's pending rows, combined in this launch
    dk_rx_results res;
};

// TX checksum fill (dk_tx_checksum): the same chunk streaming as the receive kernel, in-place checksum writes.
struct TxParams {
    uint8_t* frames;
    uint64_t frames_bytes;
    const uint32_t* off;
    const uint16_t* len;
    uint32_t n;
    uint32_t sched;  // as RxParams::sched
    uint32_t split;  // launch the split (stream waves / finish waves) kernel: one 512-thread workgroup per CU
    uint32_t* fields;  // nullptr: fill in place (dk_tx_checksum); else dk_tx_checksum_fields' u32 per frame (frames
                       // are only read)
};

}  // namespace dk

// Launchers implemented in rx_kernels.hip (internal symbols, not part of the C ABI).
// Receive kernel families (launch_batch picks one per launch).
namespace dk {
constexpr uint32_t kFamilyUnstaged = 0, kFamilyStaged = 1, kFamilySplit = 2, kFamilySmall = 3;
constexpr uint32_t kFamilySmallUb = 4;  // occupancy queries only: the small-frame kernel with the LDS bind table
}
int dk_rx_resident_blocks(uint32_t dyn_lds_bytes, uint32_t family);  // resident workgroups per CU (0 on error)
int dk_launch_rx(const dk::RxParams& p, uint32_t grid, void* stream);
// dk_flow_reduce_kernel over rows left pending by a deferred launch (dk_rx_counts_flush and the scratch paths).
int dk_launch_reduce(const dk::RowCombine& q, void* stream);
uint32_t dk_rx_small_block_waves(bool ub);  // waves per workgroup of the small-frame kernel (ub: the LDS bind table's)
// The host pipeline under the ring's copy policy (rx_host.cpp; dk_rx_process_tpacket3).
int dk_rx_process_ring_host(struct dk_rx_ctx* c, const dk_rx_batch* b, const dk_rx_results* r);
int dk_tx_resident_blocks();  // occupancy of dk_tx_kernel per CU (0 on error)
int dk_launch_tx(const dk::TxParams& p, uint32_t grid, void* stream);
