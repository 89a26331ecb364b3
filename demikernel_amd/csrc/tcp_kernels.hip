// tcp_kernels.hip — established-state TCP receive processing on the GPU (include/dk_tcp.h).
//
// The reference queues each delivered segment on its socket (tcp/socket.rs:308-314, ctrlblk.rs:345-347) and
// ControlBlock::poll runs process_packet on them one at a time (ctrlblk.rs:350-440). Connections are independent;
// within one, order matters (RCV.NXT, the out-of-order store). For a whole dk_rx batch:
//   1. dk_tcp_key_kernel (one pass over the batch, coalesced): frame -> key (its connection, for delivered TCP segments
//      of a connection in the table; else nconns) and its {seq, ack, meta, payload} record; skipped frames' outputs;
//   2. a stable sort of (key, frame index): one counting pass over the whole key up to 255 table rows
//      (dk_tcp_sort_*_kernel), rocPRIM's onesweep radix sort above: each connection's segments contiguous, in
//      arrival order;
//   3. each connection's range: from the whole-key pass's scan, else dk_tcp_range_kernel (lower_bound of its key);
//   4. dk_tcp_walk_kernel: one lane per connection (its out-of-order store in LDS) runs its segments through the
//      state machine in order, reading each segment's record through the sorted frame index (pipelined: indices two
//      batches of kBatch ahead, records one batch ahead). The walk is the only sequential part
//      (latency-bound, lanes = connections); everything else is a pass over the batch.
//   4'. dk_tcp_wave_walk_kernel instead, at >= kWaveWalkMinSegs segments per connection: one wave per connection,
//      64 segments classified in parallel per step, the state machine only for the segments that need it;
//   4''. the scan walk for few connections with many segments each (dk_tcp_scan_pre_kernel, dk_tcp_scan_kernel,
//      dk_tcp_scan_post_kernel): windows precomputed across the chip, 64 windows resolved per wave scan, the decided
//      windows written in parallel (below); dk_tcp_relay_walk_kernel (dk_diag_tcp_set_walk): 8 waves per connection
//      take its windows in turn and pass its state from window to window through LDS.
// Segments whose outcome cannot depend on their place in the connection's order are classified in step 1 and never
// walked: RCV.NXT only moves forward, from its value at the start of the batch up to the window end (reader_next +
// buffer size, fixed during the batch), so a segment starting past the window end is OUT_OF_WINDOW whenever it is
// processed, and one ending before the starting RCV.NXT is a DUPLICATE (check_segment_in_window, ctrlblk.rs:447-567;
// the bounds below keep every wrapping comparison on the same side). Only the connection's state decides between
// that and UNPROCESSED (queued behind a close): the walks record the first frame index after the close, and
// 5. dk_tcp_fix_kernel turns the classified segments from there on into UNPROCESSED. A connection whose window is
// full (every later segment beyond it) then costs one coalesced pass instead of a serial walk.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/warp/warp_scan.hpp>

#include <algorithm>
#include <climits>
#include <cerrno>
#include <cstdlib>
#include <cstddef>
#include <cstring>

#include "../../include/dk_diag.h"
#include "../../include/dk_tcp.h"

namespace dk_tcp {
namespace {

constexpr uint32_t kBlock = 256;
constexpr uint32_t kBatch = 8;  // segments whose fields a walker lane loads together

// Onesweep for every size above one block: rocPRIM's default switches to a merge sort up to 1M items, 3-4x slower
// here (20 launches for 1M 15-bit keys vs 2 onesweep passes).
using SortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                              rocprim::default_config, 0>;

__device__ __forceinline__ bool lt(uint32_t a, uint32_t b) { return (int32_t)(a - b) < 0; }
__device__ __forceinline__ bool le(uint32_t a, uint32_t b) { return (int32_t)(a - b) <= 0; }
__device__ __forceinline__ bool ge(uint32_t a, uint32_t b) { return (int32_t)(a - b) >= 0; }

struct Params {
    const uint32_t* meta;
    const uint32_t* flow_id;
    const uint32_t* seq;
    const uint32_t* ack;
    const uint32_t* payload;
    uint32_t n;
    dk_tcp_conn* conns;
    uint32_t nconns;
    uint32_t* keys;
    uint32_t* skeys;
    uint32_t* svals;
    uint4* rec;        // [n] {seq, ack, meta, payload} in frame order
    uint32_t* range;   // [2 nconns + 1]: connection c's segments are svals[range[2c] .. range[2c + 2]), of which
                       // [range[2c], range[2c + 1]) are walked and the rest were classified (sort key 2c + 1)
    uint32_t* cls;     // [n]: the connection of a segment classified in the key kernel (never walked), else kNoConn
    uint32_t* open_until;  // [nconns]: frames of the connection from this index on come after its close
    // the scan walk's per-window scratch (window v of connection c at ws = range[2c] / 64 + c + v: disjoint per c)
    uint4* scan_sum;   // [3 ws]: {A, U, window maximum, A2} against the connection's state at the call's start (decided
                       // iff A <= R <= U or R >= A2); {n0, lo, e0, e1}, {e2, e3}: the count summary (pre kernel)
    int* scan_ends;    // [ws][lane]: each lane's candidate end if it delivers at R below it, else INT_MIN
    uint32_t* scan_idx;  // [ws][lane]: the window's frame indices and their records, copied by the pre kernel (the
    uint4* scan_rec;     // slow path and the post kernel read them in one round trip instead of index -> record)
    uint4* scan_post;  // [ws]: {R, deliveries before the window, 1 = decided by the scan (written by the post kernel)}
    uint32_t* scan_head;  // [8 nconns]: the connection's state at the call's start {rn0, wend, snd, nooo, front,
                          // fin_pending, fin_seq}, saved by the scan kernel for the post kernel
    uint32_t* shape;      // device u64: finished blocks << 40 | STORED segments of this call (zero between calls)
    uint32_t* shape_host; // host-mapped [3] {STORED, n, call number}: written by the fix kernel's last block
    uint32_t call;
    dk_tcp_out out;
};
constexpr uint32_t kNoConn = 0xFFFFFFFFu;

__global__ __launch_bounds__(kBlock) void dk_tcp_key_kernel(Params P) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= P.n) return;
    const uint32_t meta = P.meta[i], pay = P.payload[i], seq = P.seq[i];
    uint32_t key = 2 * P.nconns, cls = kNoConn;  // sort key: 2c walked, 2c + 1 classified, 2 nconns not c's
    uint8_t act = DK_TCP_SKIP;
    if ((meta & 0xFFu) == DK_V_OK_TCP) {
        const uint32_t f = P.flow_id[i];
        if (f < P.nconns) {
            // state, receive_next, reader_next, buffer_size: the first 16 bytes of dk_tcp_conn, one load
            static_assert(offsetof(dk_tcp_conn, state) == 0 && offsetof(dk_tcp_conn, receive_next) == 4 &&
                              offsetof(dk_tcp_conn, reader_next) == 8 && offsetof(dk_tcp_conn, buffer_size) == 12,
                          "dk_tcp_conn layout");
            const uint4 h = *reinterpret_cast<const uint4*>(P.conns + f);
            const uint32_t state = h.x;
            if (state != DK_TCP_NONE) key = 2 * f;
            const uint32_t bufsz = h.w, rn0 = h.y, wend = h.z + bufsz;
            // order-independent outcomes (see the top of the file); the bounds keep (seq - RCV.NXT) and
            // (seg_end - RCV.NXT) of every RCV.NXT in [rn0, wend] on one side of the wrap
            if (state == DK_TCP_ESTABLISHED && wend - rn0 <= bufsz && bufsz < 0x40000000u) {
                const uint32_t flags = (meta >> 16) & 0xFFu, len = pay >> 16;
                const uint32_t full = len + ((flags >> 1) & 1u) + (flags & 1u);
                const uint32_t seg_end = full ? seq + (full - 1) : seq;
                const uint32_t lim = 0x7FFFFFFFu - bufsz - 0x20000u;
                if (seq - wend - 1u < lim) act = DK_TCP_OUT_OF_WINDOW;  // seq - wend in [1, lim]
                else if (rn0 - seg_end - 1u < lim) act = DK_TCP_DUPLICATE;  // seg_end - rn0 in [-lim, -1]
                if (act != DK_TCP_SKIP) {
                    cls = f;
                    key = 2 * f + 1;
                }
            }
        }
    }
    P.keys[i] = key;
    P.cls[i] = cls;
    P.rec[i] = make_uint4(seq, P.ack[i], meta, pay);
    if (key == 2 * P.nconns || cls != kNoConn) {  // the walk writes the outputs of every segment it owns
        P.out.action[i] = act;
        P.out.view[i] = dk_tcp_view{i, pay & 0xFFFFu, pay >> 16};
    }
}

// Classified segments after their connection's close are UNPROCESSED (the walks' queued-behind-the-close rule). The
// same pass counts the STORED segments of the first kShapeBlocks blocks (16,384 segments in arrival order, every
// connection's: the stream's shape, the walk choice of the context's next call, below) and the last of those blocks
// writes the count to the context's host-mapped words. (Counting in every block meant thousands of same-address
// atomics: 40-50 us on a 1M-segment call, session r6s4.)
constexpr uint32_t kShapeBlocks = 64;
__global__ __launch_bounds__(kBlock) void dk_tcp_fix_kernel(Params P) {
    __shared__ uint32_t s_cnt[kBlock / 64];
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    bool stored = false;
    if (i < P.n) {
        const uint32_t c = P.cls[i];
        if (c != kNoConn && i >= P.open_until[c]) P.out.action[i] = DK_TCP_UNPROCESSED;
        else stored = blockIdx.x < kShapeBlocks && c == kNoConn && P.out.action[i] == DK_TCP_STORED;
    }
    if (blockIdx.x >= kShapeBlocks) return;  // block-uniform
    const uint64_t m = __ballot(stored);
    if ((threadIdx.x & 63u) == 0) s_cnt[threadIdx.x / 64] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t sum = 0;
        for (uint32_t w = 0; w < kBlock / 64; w++) sum += s_cnt[w];
        // One 64-bit atomic per sampling block carries both its count (low 40 bits) and its arrival (high 24 bits):
        // the block that arrives last holds the total without any fence (a device-scope release here wrote back the
        // L2 in every block). Host-mapped words are visible once the kernel has completed, which is when the host
        // reads them (the call's event).
        const uint32_t nb = min(gridDim.x, kShapeBlocks);
        const unsigned long long old = atomicAdd(reinterpret_cast<unsigned long long*>(P.shape),
                                                 (1ull << 40) | (unsigned long long)sum);
        if ((uint32_t)(old >> 40) == nb - 1) {
            const uint32_t total = (uint32_t)(old & ((1ull << 40) - 1)) + sum;
            atomicExch(reinterpret_cast<unsigned long long*>(P.shape), 0ull);  // zero for the context's next call
            __hip_atomic_store(P.shape_host + 0, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(P.shape_host + 1, min(P.n, nb * kBlock), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(P.shape_host + 2, P.call, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

__global__ __launch_bounds__(kBlock) void dk_tcp_range_kernel(Params P) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;  // a sort key value, 0 .. 2 nconns
    if (c > 2 * P.nconns) return;
    uint32_t lo = 0, hi = P.n;  // first p with skeys[p] >= c
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if (P.skeys[mid] < c)
            lo = mid + 1;
        else
            hi = mid;
    }
    P.range[c] = lo;
}

// ---------------- Up to 255 connections: the batch's stable sort by one counting pass (round 6) ----------------
// Up to kSortMaxRows table rows, a stable counting pass over the whole key instead of the radix sort and the range
// kernel: (1) each block counts its tile's keys in LDS (H[k][b], key-major); (2) one block scans H flat, so H[k][b]
// becomes the position of tile b's first key-k segment and range[k] = H[k][0]; (3) each wave of a block places its
// share of the tile 64 segments a round in arrival order: a gather of each lane's key's next position, then the lanes
// of equal key found by one ballot per key bit (the AND of each bit's ballot or its complement), the rank among them
// by popcount, and the group's lowest lane moves the key's position on. Each wave loads its keys up front (one load
// latency, not one per round), counts by key group when the keys are few (same-address LDS adds serialize), and the
// scan goes through LDS so its global loads and stores coalesce. rocPRIM's onesweep costs ~9 µs per launch at 1M
// segments and ~5 µs per lookback-state fill (5 launches + 5 fills at 16 bits); the counting pass is three short
// launches (sessions r6s24-r6s25: -3 % at 1 connection to -17 % at 127 against the radix sort). Many keys need two
// passes, whose scatter and scan lose to onesweep (session r6s21: +33 % at 16,384 connections).
constexpr uint32_t kSortBlock = 512, kSortWaves = kSortBlock / 64, kSortTile = 8192, kSortSub = kSortTile / kSortWaves;
#ifndef DK_TCP_SORT_ROWS
#define DK_TCP_SORT_ROWS 255
#endif
constexpr uint32_t kSortMaxRows = DK_TCP_SORT_ROWS, kSortMaxBuckets = 2 * kSortMaxRows + 1;
struct SortPass {
    const uint32_t* kin;  // keys in
    const uint32_t* vin;  // values in (nullptr: the element's index)
    uint32_t* kout;       // keys out (nullptr: not kept)
    uint32_t* vout;       // values out
    uint32_t* H;          // [nbuck][ntiles] counts, then positions
    uint32_t shift, mask, nbuck;
};

// A wave's 64-key round grouped by digit: `same` = the live lanes whose digit equals this lane's (one ballot per digit
// bit: the AND of each bit's ballot or its complement); the group's lowest lane is its leader.
__device__ __forceinline__ uint64_t digit_group(uint32_t d, bool live, uint32_t nbits) {
    uint64_t same = __ballot(live);
    for (uint32_t bit = 0; bit < nbits; bit++) {
        const uint64_t ones = __ballot(live && ((d >> bit) & 1u));
        same &= ((d >> bit) & 1u) ? ones : ~ones;
    }
    return same;
}
constexpr uint32_t kSortRounds = kSortSub / 64;  // rounds of 64 a wave takes; its keys are loaded up front
constexpr uint32_t kSortGroupBits = 4;  // up to 16 key values the counts go by digit group (session r6s24)

// Each wave's share of the tile: keys loaded together (one load latency per wave, not one per round), then counted by
// digit group — one LDS add per group and round from its leader, so a tile of one key costs 16 adds per wave instead
// of 1,024 serialized on one address.
__device__ __forceinline__ void sort_load_keys(const SortPass& S, uint32_t s0, uint32_t s1, uint32_t lane,
                                               uint32_t (&kr)[kSortRounds]) {
#pragma unroll
    for (uint32_t r = 0; r < kSortRounds; r++) {
        const uint32_t i = s0 + r * 64 + lane;
        kr[r] = i < s1 ? S.kin[i] : 0u;
    }
}
__device__ __forceinline__ void sort_count_keys(const SortPass& S, uint32_t s0, uint32_t s1, uint32_t lane,
                                                const uint32_t (&kr)[kSortRounds], uint32_t* cnt, uint32_t nbits) {
    const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
    for (uint32_t r = 0; r < kSortRounds; r++) {
        const bool live = s0 + r * 64 + lane < s1;
        const uint32_t d = (kr[r] >> S.shift) & S.mask;
        if (nbits <= kSortGroupBits) {  // few keys: one add per group (same-address adds serialize)
            const uint64_t same = digit_group(d, live, nbits);
            if (live && !(same & lt)) atomicAdd(&cnt[d], (uint32_t)__popcll(same));
        } else if (live) {  // many keys: the adds rarely meet, and the ballots would cost more
            atomicAdd(&cnt[d], 1u);
        }
    }
}

__global__ __launch_bounds__(kSortBlock) void dk_tcp_sort_count_kernel(uint32_t n, SortPass S) {
    __shared__ uint32_t hist[kSortMaxBuckets];
    const uint32_t b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t nbits = 32u - (uint32_t)__builtin_clz(S.mask | 1u);
    uint32_t kr[kSortRounds];
    const uint32_t s0 = b * kSortTile + wv * kSortSub, s1 = min(n, s0 + kSortSub);
    sort_load_keys(S, s0, s1, lane, kr);
    for (uint32_t k = tid; k < S.nbuck; k += kSortBlock) hist[k] = 0;
    __syncthreads();
    sort_count_keys(S, s0, s1, lane, kr, hist, nbits);
    __syncthreads();
    for (uint32_t k = tid; k < S.nbuck; k += kSortBlock) S.H[(size_t)k * nb + b] = hist[k];
}

// One block: exclusive scan of H's m = nbuck * nb entries in place (digit-major); range (non-null: a whole-key pass)
// [k] = H[k][0]. Per iteration 12,288 entries go through LDS: loaded and stored coalesced (a thread's consecutive
// entries straight from global memory put 64 lanes on 64 lines per load and store: 17 µs for 16,768 entries, session
// r6s24), summed per thread over 12 consecutive ones (padded rows: no bank conflicts), one wave scan, one barrier.
constexpr uint32_t kSortScanBlock = 1024, kSortScanPer = 12, kSortScanRow = kSortScanPer + 1;
__global__ __launch_bounds__(kSortScanBlock) void dk_tcp_sort_scan_kernel(uint32_t* H, uint32_t m, uint32_t nb,
                                                                          uint32_t* range) {
    __shared__ uint32_t wsum[kSortScanBlock / 64];
    __shared__ uint32_t buf[kSortScanBlock * kSortScanRow];  // entry e at (e / 12) * 13 + e % 12
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const auto at = [](uint32_t e) { return (e / kSortScanPer) * kSortScanRow + e % kSortScanPer; };
    uint32_t carry = 0;
    for (uint32_t base = 0; base < m; base += kSortScanBlock * kSortScanPer) {
#pragma unroll
        for (uint32_t q = 0; q < kSortScanPer; q++) {
            const uint32_t e = q * kSortScanBlock + tid, j = base + e;
            buf[at(e)] = j < m ? H[j] : 0u;
        }
        __syncthreads();
        uint32_t x[kSortScanPer], t = 0;
#pragma unroll
        for (uint32_t q = 0; q < kSortScanPer; q++) {
            x[q] = buf[tid * kSortScanRow + q];
            t += x[q];
        }
        uint32_t incl = t;  // the thread's total, scanned over the wave
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        uint32_t before = carry, all = 0;
#pragma unroll
        for (uint32_t w = 0; w < kSortScanBlock / 64; w++) {
            const uint32_t ws = wsum[w];
            before += w < wv ? ws : 0u;
            all += ws;
        }
        uint32_t run = before + incl - t;
#pragma unroll
        for (uint32_t q = 0; q < kSortScanPer; q++) {
            buf[tid * kSortScanRow + q] = run;
            run += x[q];
        }
        __syncthreads();
#pragma unroll
        for (uint32_t q = 0; q < kSortScanPer; q++) {
            const uint32_t e = q * kSortScanBlock + tid, j = base + e;
            if (j < m) {
                const uint32_t v = buf[at(e)];
                H[j] = v;
                if (range && j % nb == 0) range[j / nb] = v;
            }
        }
        carry += all;
        __syncthreads();  // buf and wsum reused
    }
}

__global__ __launch_bounds__(kSortBlock) void dk_tcp_sort_scatter_kernel(uint32_t n, SortPass S) {
    __shared__ uint32_t cur[kSortWaves][kSortMaxBuckets];  // per wave: the next position per digit
    const uint32_t b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t nbits = 32u - (uint32_t)__builtin_clz(S.mask | 1u);  // digit bits (mask = 2^bits - 1)
    const uint32_t s0 = b * kSortTile + wv * kSortSub, s1 = min(n, s0 + kSortSub);
    uint32_t kr[kSortRounds];
    sort_load_keys(S, s0, s1, lane, kr);
    for (uint32_t k = tid; k < kSortWaves * kSortMaxBuckets; k += kSortBlock) (&cur[0][0])[k] = 0;
    __syncthreads();
    sort_count_keys(S, s0, s1, lane, kr, cur[wv], nbits);  // this wave's counts
    __syncthreads();
    for (uint32_t k = tid; k < S.nbuck; k += kSortBlock) {  // -> each wave's first position per digit
        uint32_t pos = S.H[(size_t)k * nb + b];
#pragma unroll
        for (uint32_t w = 0; w < kSortWaves; w++) {
            const uint32_t c = cur[w][k];
            cur[w][k] = pos;
            pos += c;
        }
    }
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
    for (uint32_t r = 0; r < kSortRounds; r++) {
        const uint32_t i = s0 + r * 64 + lane;
        const bool live = i < s1;
        const uint32_t key = kr[r], d = (key >> S.shift) & S.mask;
        const uint64_t same = digit_group(d, live, nbits);
        const uint32_t at = cur[wv][d];
        const uint32_t rank = (uint32_t)__popcll(same & lt);
        if (live && rank == 0) cur[wv][d] = at + (uint32_t)__popcll(same);
        if (live) {
            S.vout[at + rank] = S.vin ? S.vin[i] : i;
            if (S.kout) S.kout[at + rank] = key;
        }
    }
}

// One connection's scalar receive state, in registers during the walk.
struct Walk {
    uint32_t state, rn, reader, bufsz, snd, fin_pending, fin_seq, nooo;
};

// The connection's out-of-order store in LDS, one column per lane ([field][entry][lane]: conflict-free, each lane
// touches only its own column). Loaded from the table at the start of the walk and written back at the end, so the
// store's scans and shifts cost LDS latency, not HBM latency.
constexpr uint32_t kWalkBlock = 64;
struct Store {
    uint32_t* lds;  // [4][DK_TCP_OOO_MAX][kWalkBlock] + lane
    __device__ __forceinline__ uint32_t& start(uint32_t k) { return lds[(0 * DK_TCP_OOO_MAX + k) * kWalkBlock]; }
    __device__ __forceinline__ uint32_t& ref(uint32_t k) { return lds[(1 * DK_TCP_OOO_MAX + k) * kWalkBlock]; }
    __device__ __forceinline__ uint32_t& off(uint32_t k) { return lds[(2 * DK_TCP_OOO_MAX + k) * kWalkBlock]; }
    __device__ __forceinline__ uint32_t& len(uint32_t k) { return lds[(3 * DK_TCP_OOO_MAX + k) * kWalkBlock]; }
    __device__ __forceinline__ dk_tcp_view view(uint32_t k) { return dk_tcp_view{ref(k), off(k), len(k)}; }
    __device__ __forceinline__ void set(uint32_t k, uint32_t s, dk_tcp_view v) {
        start(k) = s;
        ref(k) = v.ref;
        off(k) = v.off;
        len(k) = v.len;
    }
    __device__ __forceinline__ void copy(uint32_t to, uint32_t from) { set(to, start(from), view(from)); }
    // VecDeque::remove(at) / insert(at) over the n live entries (insert drops what falls past the cap)
    __device__ __forceinline__ void remove(uint32_t at, uint32_t n) {
        for (uint32_t k = at; k + 1 < n; k++) copy(k, k + 1);
    }
    __device__ __forceinline__ void insert(uint32_t at, uint32_t n, uint32_t st, dk_tcp_view v) {
        for (uint32_t k = min(n, DK_TCP_OOO_MAX - 1); k > at; k--) copy(k, k - 1);
        set(at, st, v);
    }
};

// The wave walk's store: entry k in lane k's registers (lanes >= DK_TCP_OOO_MAX unused). Reads are lane reads of a
// wave-uniform index, remove and insert one cross-lane shift each instead of an entry-by-entry copy loop.
static_assert(DK_TCP_OOO_MAX <= 16, "RegStore keeps the store in row 0 (lanes 0..15)");
struct RegStore {
    uint32_t st, rf, of, ln, lane;
    __device__ __forceinline__ uint32_t start(uint32_t k) const { return __builtin_amdgcn_readlane(st, k); }
    __device__ __forceinline__ uint32_t len(uint32_t k) const { return __builtin_amdgcn_readlane(ln, k); }
    __device__ __forceinline__ dk_tcp_view view(uint32_t k) const {
        return dk_tcp_view{(uint32_t)__builtin_amdgcn_readlane(rf, k), (uint32_t)__builtin_amdgcn_readlane(of, k),
                           (uint32_t)__builtin_amdgcn_readlane(ln, k)};
    }
    // Entries live in lanes 0..DK_TCP_OOO_MAX - 1 = row 0: the shifts are DPP row shifts (a VALU operand
    // modifier) rather than LDS-unit permutes.
    static __device__ __forceinline__ uint32_t from_next(uint32_t x) {  // lane l gets lane l + 1 (row_shl:1)
        return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x101, 0xF, 0xF, false);
    }
    static __device__ __forceinline__ uint32_t from_prev(uint32_t x) {  // lane l gets lane l - 1 (row_shr:1)
        return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x111, 0xF, 0xF, false);
    }
    __device__ __forceinline__ void remove(uint32_t at, uint32_t) {
        const uint32_t a = from_next(st), b = from_next(rf), c = from_next(of), d = from_next(ln);
        if (lane >= at) {
            st = a;
            rf = b;
            of = c;
            ln = d;
        }
    }
    __device__ __forceinline__ void insert(uint32_t at, uint32_t, uint32_t s, dk_tcp_view v) {
        const uint32_t a = from_prev(st), b = from_prev(rf), c = from_prev(of), d = from_prev(ln);
        if (lane > at) {
            st = a;
            rf = b;
            of = c;
            ln = d;
        } else if (lane == at) {
            st = s;
            rf = v.ref;
            of = v.off;
            ln = v.len;
        }
    }
};

struct Out {  // the connection's delivery slots
    dk_tcp_view* d;
    uint32_t n, cap;
    __device__ __forceinline__ void push(dk_tcp_view v, Walk& w) {  // Receiver::push (ctrlblk.rs:131-136)
        if (n < cap) d[n] = v;
        n++;
        w.rn += v.len;
    }
};

template <class S>
__device__ __forceinline__ void ooo_remove(S& s, Walk& w, uint32_t at) {
    s.remove(at, w.nooo);
    w.nooo--;
}

// store_out_of_order_segment (ctrlblk.rs:844-941) on the fixed arrays.
template <class S>
__device__ __forceinline__ uint32_t ooo_store(S& s, Walk& w, uint32_t new_start, uint32_t new_end,
                                              dk_tcp_view buf) {
    uint32_t at = w.nooo;
    bool again = true;
    while (again) {
        again = false;
        at = w.nooo;
        for (uint32_t i = 0; i < w.nooo; i++) {
            const uint32_t ss = s.start(i), se = ss + (s.len(i) - 1);
            if (lt(new_start, ss)) {
                if (lt(new_end, ss)) {
                    at = i;
                    break;
                }
                if (lt(se, new_end)) {  // encompasses entry i: drop it and scan again
                    again = true;
                    at = i;
                    break;
                }
                const uint32_t excess = (new_end - ss) + 1;  // front overlap; inserted at the back (reference)
                new_end -= excess;
                buf.len -= excess;
                break;
            }
            if (le(new_end, se)) return DK_TCP_STORE_DUP;
            if (lt(se, new_start)) continue;
            const uint32_t dup = se - new_start;  // end overlap, one byte short (reference, ctrlblk.rs:916)
            new_start += dup;
            buf.off += dup;
            buf.len -= dup;
        }
        if (again) ooo_remove(s, w, at);
    }
    // VecDeque::insert at `at`, then pop_back while longer than the cap
    if (at >= DK_TCP_OOO_MAX) return DK_TCP_STORED;
    s.insert(at, w.nooo, new_start, buf);
    w.nooo = min(w.nooo + 1, DK_TCP_OOO_MAX);
    return DK_TCP_STORED;
}

// receive_data (ctrlblk.rs:951-1001): true if a stored FIN is now in order.
template <class S>
__device__ __forceinline__ bool receive_data(S& s, Walk& w, dk_tcp_view buf, Out& o) {
    uint32_t recv_next = w.rn + buf.len;
    o.push(buf, w);
    while (w.nooo > 0 && s.start(0) == recv_next) {
        const dk_tcp_view t = s.view(0);
        ooo_remove(s, w, 0);
        recv_next += t.len;
        o.push(t, w);
    }
    return w.fin_pending && w.fin_seq == recv_next;
}

// process_packet (ctrlblk.rs:403-440) for segment g = {seq, ack, meta, payload} of frame i.
template <class S>
__device__ __forceinline__ uint32_t process(S& s, Walk& w, uint4 g, uint32_t i, Out& o, dk_tcp_view& view) {
    const uint32_t flags = (g.z >> 16) & 0xFFu;
    bool syn = flags & 0x02u, fin = flags & 0x01u;
    const bool rst = flags & 0x04u, ack = flags & 0x10u;
    dk_tcp_view data{i, g.w & 0xFFFFu, g.w >> 16};
    uint32_t seg_start = g.x, seg_end = g.x, seg_len = data.len;
    view = data;
    // check_segment_in_window (ctrlblk.rs:447-567); window end = RCV.NXT + buffer - (RCV.NXT - reader_next)
    if (syn) seg_len += 1;
    if (fin) seg_len += 1;
    if (seg_len > 0) seg_end = seg_start + (seg_len - 1);
    const uint32_t after = w.rn + (w.bufsz - (w.rn - w.reader));
    if (seg_start != w.rn) {
        if (lt(seg_start, w.rn)) {
            if (lt(seg_end, w.rn)) return DK_TCP_DUPLICATE;
            uint32_t dup = w.rn - seg_start;
            seg_start += dup;
            seg_len -= dup;
            if (syn) {
                syn = false;
                dup -= 1;
            }
            data.off += dup;
            data.len -= dup;
        } else if (ge(seg_start, after)) {
            return DK_TCP_OUT_OF_WINDOW;
        }
    }
    if (seg_len > 0 && ge(seg_end, after)) {
        uint32_t excess = (seg_end - after) + 1;
        seg_end -= excess;
        seg_len -= excess;
        if (fin) {
            fin = false;
            excess -= 1;
        }
        data.len -= excess;
    }
    view = data;
    if (rst) {
        w.state = DK_TCP_CLOSED;
        return DK_TCP_RST;
    }
    if (syn) return DK_TCP_SYN;
    if (!ack) return DK_TCP_NO_ACK;
    if (!le(g.y, w.snd)) return DK_TCP_ACK_UNSENT;
    uint32_t action = DK_TCP_NO_DATA;
    if (data.len > 0 || fin) {  // process_data (ctrlblk.rs:652-695)
        if (seg_start != w.rn) {
            action = DK_TCP_STORED;
            if (seg_len > 0) {
                if (fin) {
                    seg_len -= 1;
                    w.fin_pending = 1;
                    w.fin_seq = seg_end;
                    seg_end -= 1;
                    fin = false;
                }
                if (seg_len > 0) action = ooo_store(s, w, seg_start, seg_end, data);
            }
        } else {
            action = DK_TCP_DELIVERED;
            if (receive_data(s, w, data, o)) fin = true;
        }
    }
    if (fin) {  // process_remote_close (ctrlblk.rs:1003-1024)
        o.push(dk_tcp_view{DK_TCP_REF_EOF, 0, 0}, w);
        w.rn += 1;
        w.state = DK_TCP_CLOSED;
        return DK_TCP_FIN;
    }
    return action;
}

__global__ __launch_bounds__(kWalkBlock) void dk_tcp_walk_kernel(Params P) {
    __shared__ uint32_t lds[4 * DK_TCP_OOO_MAX * kWalkBlock];
    const uint32_t c = blockIdx.x * kWalkBlock + threadIdx.x;
    if (c >= P.nconns) return;
    dk_tcp_conn* t = P.conns + c;
    const uint32_t k0 = P.range[2 * c], cnt = P.range[2 * c + 1] - k0, all = P.range[2 * c + 2] - k0;
    const uint32_t d0 = k0 + DK_TCP_DELIV_EXTRA * c;
    P.out.deliv_start[c] = d0;
    Walk w{t->state, t->receive_next, t->reader_next, t->buffer_size, t->send_next, t->fin_pending, t->fin_seq,
           min(t->ooo_count, DK_TCP_OOO_MAX)};
    Store s{lds + threadIdx.x};
    for (uint32_t k = 0; k < w.nooo; k++) s.set(k, t->ooo_start[k], t->ooo[k]);
    uint32_t open_until = w.state == DK_TCP_ESTABLISHED ? 0xFFFFFFFFu : 0u;
    Out o{P.out.deliv + d0, 0, all + DK_TCP_DELIV_EXTRA};
    // Software pipeline over batches of kBatch segments: frame indices two batches ahead, their records one batch
    // ahead, so neither load level waits in the loop (the walk is latency-bound: about one wave per SIMD).
    uint32_t ia[kBatch], ib[kBatch], ic[kBatch];
    uint4 gb[kBatch], gc[kBatch];
#pragma unroll
    for (uint32_t j = 0; j < kBatch; j++) {
        ib[j] = j < cnt ? P.svals[k0 + j] : 0u;
        ia[j] = kBatch + j < cnt ? P.svals[k0 + kBatch + j] : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < kBatch; j++)
        if (j < cnt) gb[j] = P.rec[ib[j]];
    for (uint32_t k = 0; k < cnt; k += kBatch) {
#pragma unroll
        for (uint32_t j = 0; j < kBatch; j++) {
            gc[j] = gb[j];
            ic[j] = ib[j];
        }
        if (k + kBatch < cnt) {
#pragma unroll
            for (uint32_t j = 0; j < kBatch; j++) {
                if (k + kBatch + j < cnt) gb[j] = P.rec[ia[j]];
                ib[j] = ia[j];
            }
        }
        if (k + 2 * kBatch < cnt) {
#pragma unroll
            for (uint32_t j = 0; j < kBatch; j++)
                if (k + 2 * kBatch + j < cnt) ia[j] = P.svals[k0 + k + 2 * kBatch + j];
        }
#pragma unroll
        for (uint32_t j = 0; j < kBatch; j++) {
            if (k + j >= cnt) break;
            if (w.state != DK_TCP_ESTABLISHED) {
                P.out.action[ic[j]] = DK_TCP_UNPROCESSED;
                P.out.view[ic[j]] = dk_tcp_view{ic[j], gc[j].w & 0xFFFFu, gc[j].w >> 16};
                continue;
            }
            dk_tcp_view v;
            P.out.action[ic[j]] = (uint8_t)process(s, w, gc[j], ic[j], o, v);
            P.out.view[ic[j]] = v;
            if (w.state != DK_TCP_ESTABLISHED) open_until = ic[j] + 1;  // this segment closed the connection
        }
    }
    P.open_until[c] = open_until;
    t->state = w.state;
    t->receive_next = w.rn;
    t->fin_pending = w.fin_pending;
    t->fin_seq = w.fin_seq;
    t->ooo_count = w.nooo;
    for (uint32_t k = 0; k < DK_TCP_OOO_MAX; k++) {
        const bool live = k < w.nooo;
        t->ooo_start[k] = live ? s.start(k) : 0u;
        t->ooo[k] = live ? s.view(k) : dk_tcp_view{0, 0, 0};
    }
    P.out.deliv_count[c] = o.n;
}

// The same walk with one wave per connection, for batches with many segments per connection (lanes = connections
// leaves the chip idle when there are few). The connection's state stays wave-uniform. Each window of 64 segments is
// classified in parallel (see the loop below): segments whose process_packet outcome needs no state machine are
// taken at once — in-order data with no SYN/FIN/RST that ends inside the window and does not end exactly at the
// out-of-order store's first entry or a pending FIN (NO_ACK / ACK_UNSENT with no state change, else DELIVERED = one
// push and RCV.NXT += length, nothing drained from the store, or NO_DATA), the same for a partial retransmission
// (starts before RCV.NXT, ends after it: its old front trimmed, the rest as in order), entirely old segments
// (DUPLICATE) and segments past the window (OUT_OF_WINDOW). The window end
// RCV.NXT + buffer - (RCV.NXT - reader_next) is reader_next + buffer for the whole batch, since nothing reads during
// it. The first other segment goes through process() with every lane executing it redundantly (same inputs; the
// out-of-order store is a RegStore, entry k in lane k), then the parallel check resumes at the next lane.
constexpr uint32_t kWave = 64;

using WaveScan = rocprim::warp_scan<uint32_t, kWave>;

// kRing = false (many connections, where occupancy hides the latency): each window's records are loaded one window
// ahead into registers. kRing = true (few connections, where one wave's window loop is the whole run): the frame
// indices and records stream into LDS rings by LDS-DMA loads (global_load_lds), kRingH windows ahead, with explicit
// waits (below). Register prefetch does not survive the compiler here: the window loop holds stores and inner loops,
// and the compiler waits for every outstanding load before such a loop (a 1-connection batch ran at 1.2 µs per
// 64-segment window, one load latency each, with records prefetched four windows ahead in registers).
constexpr uint32_t kRingH = 6, kIdxSlots = 16, kRecSlots = 8;
static_assert(2 * kRingH + 1 <= kIdxSlots && kRingH + 1 <= kRecSlots, "ring slots cover the windows in flight");
static_assert(2 * kRingH - 2 == 10, "the s_waitcnt immediate below");
typedef __attribute__((address_space(3))) void lds_void;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
template <class T>
__device__ __forceinline__ uint32_t lds_addr(T* p) {
    return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) T*)p;
}
__device__ __forceinline__ uint32_t lds_read_u32(uint32_t a) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
    return v;
}
// one window's frame indices (a_i), records (a_g) and the frame indices of window + kRingH (a_f)
__device__ __forceinline__ void lds_read_window(uint32_t a_i, uint32_t a_g, uint32_t a_f, uint32_t& i, uint4& g,
                                                uint32_t& f) {
    u32x4 q;
    asm volatile("ds_read_b32 %0, %3\n\tds_read_b128 %1, %4\n\tds_read_b32 %2, %5\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(i), "=&v"(q), "=&v"(f)
                 : "v"(a_i), "v"(a_g), "v"(a_f)
                 : "memory");
    g = make_uint4(q.x, q.y, q.z, q.w);
}

// One segment's fields for the parallel check (lanes = consecutive segments of one connection).
struct Seg {
    uint32_t x, off, len, dend, seg_end;
    bool have, simple, syn, ack_ok;
    uint8_t fast_action;
    __device__ __forceinline__ Seg(uint4 g, bool have_, uint32_t snd) {
        const uint32_t flags = (g.z >> 16) & 0xFFu;
        x = g.x;
        off = g.w & 0xFFFFu;
        len = g.w >> 16;
        have = have_;
        simple = have && !(flags & 0x07u);
        syn = have && (flags & 0x07u) == 0x02u;  // SYN without FIN or RST
        ack_ok = (flags & 0x10u) && le(g.y, snd);
        fast_action = !(flags & 0x10u) ? DK_TCP_NO_ACK : !ack_ok ? DK_TCP_ACK_UNSENT : len > 0 ? DK_TCP_DELIVERED : DK_TCP_NO_DATA;
        dend = x + len;
        const uint32_t full = len + ((flags >> 1) & 1u) + (flags & 1u);  // SYN and FIN take a number each
        seg_end = full ? x + (full - 1) : x;
    }
    // Candidates: data ending inside the window that moves RCV.NXT to its end if RCV.NXT reaches its start (in-order
    // data, or a partial retransmission: its old front is trimmed and the rest delivered).
    __device__ __forceinline__ bool cand(bool beyond, uint32_t wend) const {
        return simple && !beyond && ack_ok && len > 0 && !ge(dend - 1u, wend);
    }
};
struct Verdict {
    bool ok;  // the outcome needs no state machine
    uint8_t act;
    uint32_t voff, vlen;
};
// The segment against RCV.NXT as it stands before it (rn) and the rest of the connection's state (process_packet,
// ctrlblk.rs:403-440, for the outcomes that change nothing but RCV.NXT and the deliveries):
//   ending before rn: DUPLICATE; starting at or past the window end (and not at rn): OUT_OF_WINDOW;
//   plain data (no SYN/FIN/RST) starting at rn, or before it and ending after it (the old front trimmed,
//   check_segment_in_window ctrlblk.rs:480-500), ending inside the window: NO_ACK / ACK_UNSENT / DELIVERED / NO_DATA;
//   plain data past rn inside the window with the store full and after every entry: STORED with no change
//   (ctrlblk.rs:933-940); a SYN (without FIN/RST) at or past rn that ends inside the window: SYN.
// receive_data drains the store (and completes a pending FIN) only when a push ends exactly at the store's first
// entry (at fin_seq): such a push is left to process(), as is everything else. Branch-free (selects).
__device__ __forceinline__ Verdict classify(const Seg& q, uint32_t rn, uint32_t wend, bool beyond, uint32_t nooo,
                                            uint32_t front, uint32_t fin_pending, uint32_t fin_seq,
                                            bool syn_reach = false) {
    const bool drains = q.ack_ok && q.len > 0 && ((nooo && q.dend == front) || (fin_pending && q.dend == fin_seq));
    const bool at = q.x == rn, before = lt(q.x, rn), dup = before && lt(q.seg_end, rn);
    const bool oow = !at && !before && ge(q.x, wend);
    const bool past = !at && !before && !oow;  // inside the window, after rn
    const bool data_in = !ge(q.dend - 1u, wend), plain = q.simple && !beyond && !drains;
    const bool syn_ok = q.syn && (at || past) && !ge(q.seg_end, wend);
    // syn_reach (the caller's RCV.NXT accounts for it): a SYN starting before rn and ending at or after it loses its
    // SYN and old front (check_segment_in_window) and is then plain data ending at seg_end
    const uint32_t send1 = q.seg_end + 1u;
    const bool syn_part_ok = syn_reach && q.syn && before && !dup && !ge(q.seg_end, wend) &&
                             !(q.ack_ok && ((nooo && send1 == front) || (fin_pending && send1 == fin_seq)));
    // plain segments past rn that carry no deliverable data (no ACK, ACK of unsent data, or no payload) change nothing
    // in process_packet either (ctrlblk.rs:403-440): NO_ACK / ACK_UNSENT / NO_DATA at any place in the window
    const bool ok = dup || oow || syn_ok || syn_part_ok || (at && plain && (q.len == 0 || data_in)) ||
                    (before && plain && data_in) || (past && beyond) ||
                    (past && q.simple && q.fast_action != DK_TCP_DELIVERED);
    Verdict r;
    r.ok = ok && q.have;
    r.act = dup ? (uint8_t)DK_TCP_DUPLICATE
          : oow ? (uint8_t)DK_TCP_OUT_OF_WINDOW
          : syn_ok ? (uint8_t)DK_TCP_SYN
          : past && q.fast_action == DK_TCP_DELIVERED ? (uint8_t)DK_TCP_STORED : q.fast_action;
    const bool trim = before && !dup;
    const uint32_t sh = q.syn ? 1u : 0u;  // the SYN's sequence number
    r.voff = trim ? q.off + (rn - q.x - sh) : q.off;
    r.vlen = trim ? q.dend + sh - rn
           : past && !q.syn && q.len > 0 && ge(q.x + (q.len - 1), wend) ? wend - q.x  // check_segment_in_window's end trim
           : q.len;
    return r;
}

// One wave's walk state for a connection: the scalar state, the out-of-order store (entry k in lane k), deliveries.
struct WaveWalk {
    const Params& P;
    Walk w;
    RegStore s;
    Out o;
    uint32_t open_until, wend, cnt, lane;
    WaveScan::storage_type& scan;

    // The segments base + lo0 .. base + 63 (frame indices i, records g; lanes below lo0 already decided), in order.
    __device__ __forceinline__ void window(uint32_t base, uint32_t i, uint4 g, uint32_t lo0 = 0) {
        const uint32_t lim = min(cnt - base, kWave);
        const Seg q(g, lane < lim, w.snd);
        uint32_t lo = lo0;
        while (lo < lim) {
            if (w.state != DK_TCP_ESTABLISHED) {  // queued behind the close
                if (lane >= lo && q.have) {
                    P.out.action[i] = DK_TCP_UNPROCESSED;
                    P.out.view[i] = dk_tcp_view{i, q.off, q.len};
                }
                break;
            }
            // Parallel classification of lanes lo.. against RCV.NXT as it stands before each: accepted candidates
            // move it to their end, so it is the running maximum of the candidates' ends (relative to RCV.NXT at lo).
            // Entirely old (DUPLICATE) and past-the-window (OUT_OF_WINDOW) segments change nothing and are taken with
            // the store in any state; the first other segment goes through process().
            const bool mine = lane >= lo;
            // With the store full, a segment that starts after every stored entry is inserted at the end and popped
            // again (ctrlblk.rs:933-940): STORED with no change (a stuck hole makes every later segment one)
            bool beyond = false;
            if (w.nooo == DK_TCP_OOO_MAX && mine && q.simple) {
                beyond = true;
                for (uint32_t k = 0; k < DK_TCP_OOO_MAX; k++) beyond = beyond && lt(s.start(k) + (s.len(k) - 1), q.x);
            }
            const uint32_t rel = mine && q.cand(beyond, wend) && lt(w.rn, q.dend) ? q.dend - w.rn : 0u;
            uint32_t mx_prev;  // max over the lanes before this one (DPP scan)
            WaveScan().exclusive_scan(rel, mx_prev, 0u, scan, rocprim::maximum<uint32_t>());
            const uint32_t mx = max(mx_prev, rel);
            const Verdict r = classify(q, w.rn + mx_prev, wend, beyond, w.nooo, w.nooo ? s.start(0) : 0u,
                                       w.fin_pending, w.fin_seq);
            const uint64_t bad = __ballot(mine && !(r.ok && mine));
            const uint32_t f = min(bad ? (uint32_t)__builtin_ctzll(bad) : kWave, lim);
            const bool taken = mine && lane < f;
            const bool pushed = taken && r.act == DK_TCP_DELIVERED;
            const uint64_t pm = __ballot(pushed);
            const uint32_t before =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0u));
            if (taken) {
                P.out.action[i] = r.act;
                P.out.view[i] = dk_tcp_view{i, r.voff, r.vlen};
                if (pushed && o.n + before < o.cap) o.d[o.n + before] = dk_tcp_view{i, r.voff, r.vlen};
            }
            o.n += (uint32_t)__builtin_popcountll(pm);
            if (f > lo) w.rn += (uint32_t)__builtin_amdgcn_readlane(mx, f - 1);
            if (f >= lim) break;
            const uint4 gf = make_uint4(__builtin_amdgcn_readlane(g.x, f), __builtin_amdgcn_readlane(g.y, f),
                                        __builtin_amdgcn_readlane(g.z, f), __builtin_amdgcn_readlane(g.w, f));
            const uint32_t i_f = __builtin_amdgcn_readlane(i, f);
            dk_tcp_view v;
            const uint32_t a_f = process(s, w, gf, i_f, o, v);
            if (lane == 0) {
                P.out.action[i_f] = (uint8_t)a_f;
                P.out.view[i_f] = v;
            }
            if (w.state != DK_TCP_ESTABLISHED) open_until = i_f + 1;  // this segment closed the connection
            lo = f + 1;
        }
    }
};

// The windows v0 .. v1 - 1 of a connection's cnt segments (sorted frame indices at P.svals + k0) through W, streamed into LDS
// rings. Window u's indices land in sidx[u % 16] (DMA issued at window u - 2H, read at u - H and u), its records in
// srec[u % 8] (issued at window u - H, read at u). Window v issues records(v + H), then indices(v + 2H), so at least
// 2H - 2 vector-memory operations follow indices(v + H) and 2H - 1 follow records(v): vmcnt(2H - 2) has both landed
// whatever else (result stores) was issued in between (vmcnt retires in order).
__device__ __forceinline__ void ring_walk(const Params& P, WaveWalk& W, uint32_t (&sidx)[kIdxSlots][kWave],
                                          uint4 (&srec)[kRecSlots][kWave], uint32_t k0, uint32_t cnt, uint32_t v0,
                                          uint32_t v1) {
    const uint32_t lane = W.lane, last = cnt ? cnt - 1 : 0u;
    const auto idx_dma = [&](uint32_t u) {
        __builtin_amdgcn_global_load_lds((const void*)(P.svals + k0 + min(u * kWave + lane, last)),
                                         (lds_void*)&sidx[u % kIdxSlots][0], 4, 0, 0);
    };
    const auto rec_dma = [&](uint32_t u, uint32_t fi) {
        __builtin_amdgcn_global_load_lds((const void*)(P.rec + fi), (lds_void*)&srec[u % kRecSlots][0], 16, 0, 0);
    };
    // The ring is read by inline-asm LDS loads: the compiler cannot tell ring slots apart and would wait for every
    // LDS-DMA load (vmcnt(0)) before each LDS read.
    const auto idx_at = [&](uint32_t u) { return lds_addr(&sidx[u % kIdxSlots][lane]); };
    if (v0 >= v1) return;  // (k0 may be n when cnt is 0)
    for (uint32_t u = v0; u < v0 + kRingH; u++) idx_dma(u);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (uint32_t u = v0; u < v0 + kRingH; u++) {
        rec_dma(u, lds_read_u32(idx_at(u)));
        idx_dma(u + kRingH);
    }
    for (uint32_t v = v0; v < v1; v++) {
        asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
        uint32_t i, fi;
        uint4 g;
        lds_read_window(idx_at(v), lds_addr(&srec[v % kRecSlots][lane]), idx_at(v + kRingH), i, g, fi);
        rec_dma(v + kRingH, fi);
        idx_dma(v + 2 * kRingH);
        W.window(v * kWave, i, g);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA write outlives the workgroup
}

#define DK_U(x) (uint32_t) __builtin_amdgcn_readfirstlane((int)(x))

template <bool kRing>
__global__ __launch_bounds__(kWave) void dk_tcp_wave_walk_kernel(Params P) {
    __shared__ WaveScan::storage_type scan_tmp;
    __shared__ uint32_t sidx[kRing ? kIdxSlots : 1][kWave];
    __shared__ uint4 srec[kRing ? kRecSlots : 1][kWave];
    const uint32_t c = blockIdx.x, lane = threadIdx.x;
    dk_tcp_conn* t = P.conns + c;
    const uint32_t k0 = P.range[2 * c], cnt = P.range[2 * c + 1] - k0, all = P.range[2 * c + 2] - k0;
    const uint32_t d0 = k0 + DK_TCP_DELIV_EXTRA * c;
    // the connection's scalar state, wave-uniform: held in scalar registers
    const Walk w0{DK_U(t->state), DK_U(t->receive_next), DK_U(t->reader_next), DK_U(t->buffer_size),
                  DK_U(t->send_next), DK_U(t->fin_pending), DK_U(t->fin_seq), DK_U(min(t->ooo_count, DK_TCP_OOO_MAX))};
    RegStore s0{0u, 0u, 0u, 0u, lane};
    if (lane < w0.nooo) {
        const dk_tcp_view v = t->ooo[lane];
        s0 = RegStore{t->ooo_start[lane], v.ref, v.off, v.len, lane};
    }
    WaveWalk W{P, w0, s0, Out{P.out.deliv + d0, 0, all + DK_TCP_DELIV_EXTRA},
               w0.state == DK_TCP_ESTABLISHED ? 0xFFFFFFFFu : 0u, w0.reader + w0.bufsz, cnt, lane, scan_tmp};
    // Loads are unconditional: positions past the connection's last segment read its last one again (unused).
    const uint32_t last = cnt ? cnt - 1 : 0u;
    if constexpr (kRing) {
        ring_walk(P, W, sidx, srec, k0, cnt, 0u, (uint32_t)(((uint64_t)cnt + kWave - 1) / kWave));
    } else {
        // frame indices two windows ahead, records one
        const auto idx = [&](uint32_t u) { return P.svals[k0 + min(u * kWave + lane, last)]; };
        uint32_t i = 0, i1 = 0;
        uint4 g = make_uint4(0u, 0u, 0u, 0u);
        if (cnt) {
            i = idx(0);
            i1 = idx(1);
            g = P.rec[i];
        }
        for (uint32_t v = 0; v * kWave < cnt; v++) {
            const uint32_t i2 = idx(v + 2);
            const uint4 g1 = P.rec[i1];
            W.window(v * kWave, i, g);
            i = i1;
            i1 = i2;
            g = g1;
        }
    }
    if (lane == 0) {
        P.out.deliv_start[c] = d0;
        P.open_until[c] = W.open_until;
        t->state = W.w.state;
        t->receive_next = W.w.rn;
        t->fin_pending = W.w.fin_pending;
        t->fin_seq = W.w.fin_seq;
        t->ooo_count = W.w.nooo;
        P.out.deliv_count[c] = W.o.n;
    }
    if (lane < DK_TCP_OOO_MAX) {
        const bool live = lane < W.w.nooo;
        t->ooo_start[lane] = live ? W.s.st : 0u;
        t->ooo[lane] = live ? dk_tcp_view{W.s.rf, W.s.of, W.s.ln} : dk_tcp_view{0, 0, 0};
    }
}

// The relay walk: kRelayWaves waves per connection take its 64-segment windows round-robin and pass the connection's
// state from window to window through LDS (the baton: RCV.NXT, deliveries so far, and the rest of the state with an
// epoch that only windows running the state machine bump). Before waiting for the baton a wave does everything about
// its window that does not depend on RCV.NXT at the window start (R): the loads, the fields, the candidates' ends and
// their running maximum (DPP scans), and for the state as of epoch e0 each lane's condition on R (below: the window
// is decided by classify() iff A <= R <= U). Under the baton, if the epoch is still e0 and R is in range, the wave
// hands on RCV.NXT = max(R, window max) and the deliveries count at once (a few instructions) and writes its results
// after; otherwise the lanes before the first undecided one are taken and the one-wave walk continues from there on
// the baton's state (the store moving between LDS and lane registers) before the baton moves on. 1 connection, 1M
// in-order segments: 4.2 ms against 12.7 ms for the one-wave walk (session r05r).
// waves per connection: DK_TCP_RELAY_WAVES = 4 | 8 | 16
struct alignas(16) Baton {
    uint32_t turn;   // the window whose owner holds the baton
    uint32_t epoch;  // bumped by every window that went through the state machine (state, store, FIN may change)
    uint32_t rn, n;  // n: deliveries so far
    uint32_t state, nooo, front;  // front: the store's first entry's start (nooo > 0)
    uint32_t fin_pending, fin_seq, open_until;
};
__device__ __forceinline__ uint32_t lds_relaxed(uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// The fast hand-off relies on the LDS executing one wave's LDS instructions in issue order (the same order the
// LGKM counter retires them in): a holder that writes {rn, n} and then turn, as two back-to-back instructions, cannot
// have turn seen before {rn, n}; a waiter that reads turn and then {epoch, rn, n} in one poll gets, once turn shows
// its window, values at least as new as the holder's. One LDS round trip each way instead of a wait for the stores
// before a release store and a read after an acquire poll.
__device__ __forceinline__ void baton_poll(const Baton* bt, uint32_t& turn, uint32_t& epoch, uint32_t& rn,
                                           uint32_t& n) {
    const uint32_t a = (uint32_t)reinterpret_cast<uintptr_t>(bt);
    uint32_t t, e;
    uint2 rv;
    asm volatile(
        "ds_read_b32 %0, %3\n\t"
        "ds_read_b32 %1, %3 offset:4\n\t"
        "ds_read_b64 %2, %3 offset:8\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=v"(t), "=v"(e), "=v"(rv)
        : "v"(a)
        : "memory");
    turn = DK_U(t);
    epoch = DK_U(e);
    rn = DK_U(rv.x);
    n = DK_U(rv.y);
}
__device__ __forceinline__ void baton_pass(Baton* bt, uint32_t turn, uint32_t rn, uint32_t n) {  // one lane
    const uint32_t a = (uint32_t)reinterpret_cast<uintptr_t>(bt);
    const uint2 rv = make_uint2(rn, n);
    asm volatile(
        "ds_write_b64 %0, %1 offset:8\n\t"
        "ds_write_b32 %0, %2"
        :
        : "v"(a), "v"(rv), "v"(turn)
        : "memory");
}

template <uint32_t kRelayWaves>
__global__ __launch_bounds__(kRelayWaves * kWave) void dk_tcp_relay_walk_kernel(Params P) {
    __shared__ WaveScan::storage_type scan_tmp[kRelayWaves];
    __shared__ Baton bt;
    __shared__ uint32_t sto[4][DK_TCP_OOO_MAX];  // the out-of-order store: start, ref, off, len
    const uint32_t c = blockIdx.x, lane = threadIdx.x & (kWave - 1), wv = DK_U(threadIdx.x / kWave);
    dk_tcp_conn* t = P.conns + c;
    const uint32_t k0 = P.range[2 * c], cnt = P.range[2 * c + 1] - k0, all = P.range[2 * c + 2] - k0;
    const uint32_t d0 = k0 + DK_TCP_DELIV_EXTRA * c, cap = all + DK_TCP_DELIV_EXTRA;
    dk_tcp_view* const dv = P.out.deliv + d0;
    const uint32_t rn0 = DK_U(t->receive_next), reader = DK_U(t->reader_next), bufsz = DK_U(t->buffer_size),
                   snd = DK_U(t->send_next), wend = reader + bufsz;
    if (wv == 0) {
        const uint32_t state = t->state, nooo = min(t->ooo_count, DK_TCP_OOO_MAX);
        if (lane < DK_TCP_OOO_MAX) {
            const dk_tcp_view e = t->ooo[lane];
            sto[0][lane] = t->ooo_start[lane];
            sto[1][lane] = e.ref;
            sto[2][lane] = e.off;
            sto[3][lane] = e.len;
        }
        if (lane == 0)
            bt = Baton{0u, 0u, rn0, 0u, state, nooo, nooo ? t->ooo_start[0] : 0u, t->fin_pending, t->fin_seq,
                       state == DK_TCP_ESTABLISHED ? 0xFFFFFFFFu : 0u};
    }
    __syncthreads();
    const uint32_t nwin = (uint32_t)(((uint64_t)cnt + kWave - 1) / kWave), last = cnt ? cnt - 1 : 0u;
    const auto idx = [&](uint32_t v) { return P.svals[k0 + min(v * kWave + lane, last)]; };
    // this wave's next window: records one round ahead, frame indices two
    uint32_t i = 0, i1 = 0;
    uint4 g = make_uint4(0u, 0u, 0u, 0u);
    if (wv < nwin) {
        i = idx(wv);
        i1 = idx(wv + kRelayWaves);
        g = P.rec[i];
    }
    for (uint32_t v = wv; v < nwin; v += kRelayWaves) {
        const uint32_t base = v * kWave, lim = min(cnt - base, kWave);
        const Seg q(g, lane < lim, snd);
        // candidates' ends (relative to rn0) and their running maximum; then the SYNs that start before that
        // maximum (reached whatever R is: a retransmitted SYN is plain data to seg_end once reached) join them
        const bool cand = q.cand(false, wend);
        const uint32_t key1 = cand && lt(rn0, q.dend) ? q.dend - rn0 : 0u;
        uint32_t pm1;
        WaveScan().exclusive_scan(key1, pm1, 0u, scan_tmp[wv], rocprim::maximum<uint32_t>());
        const bool syn_r = q.syn && !ge(q.seg_end, wend) && (int)(q.x - rn0) < (int)pm1;  // reached, no end trim
        const bool synd = syn_r && q.ack_ok;  // ... and delivers up to seg_end
        const uint32_t key = synd && lt(rn0, q.seg_end + 1u) ? max(key1, q.seg_end + 1u - rn0) : key1;
        uint32_t pm;
        WaveScan().exclusive_scan(key, pm, 0u, scan_tmp[wv], rocprim::maximum<uint32_t>());
        const uint32_t wmax = (uint32_t)__builtin_amdgcn_readlane(max(pm, key), kWave - 1);
        // The window's transfer, before the baton: with the connection's state other than RCV.NXT as it stands now
        // (epoch e0; only windows that run the state machine change it), lane j is decided by classify() iff
        // rn_j = max(R, pm_j) >= T_j (R: RCV.NXT at the window start, everything relative to rn0), except a SYN that
        // is neither old nor past the window, decided iff rn_j <= its start (R <= U). So the whole window is iff
        // A <= R <= U (A = max of the T_j that pm_j does not already meet), it moves RCV.NXT to max(R, wmax), and its
        // deliveries are the candidates with max(R, pm_j) < their end. With the baton the check is a few instructions.
        const uint32_t e0 = DK_U(lds_relaxed(&bt.epoch));
        const uint32_t s_state = DK_U(lds_relaxed(&bt.state)), s_nooo = DK_U(lds_relaxed(&bt.nooo)),
                       s_front = DK_U(lds_relaxed(&bt.front)), s_finp = DK_U(lds_relaxed(&bt.fin_pending)),
                       s_fins = DK_U(lds_relaxed(&bt.fin_seq));
        const bool transparent = s_state == DK_TCP_ESTABLISHED && s_nooo < DK_TCP_OOO_MAX;
        const int xr = (int)(q.x - rn0), er = (int)(q.seg_end - rn0), dr = (int)(q.dend - rn0), pmi = (int)pm;
        int T = INT_MIN, U = INT_MAX;
        if (q.have) {
            const bool drains =
                q.ack_ok && q.len > 0 && ((s_nooo && q.dend == s_front) || (s_finp && q.dend == s_fins));
            if (ge(q.x, wend))
                T = q.x == wend ? INT_MAX : INT_MIN;  // past the window end; at it only while RCV.NXT is not
            else if (q.syn) {
                const bool send_drains = (s_nooo && q.seg_end + 1u == s_front) || (s_finp && q.seg_end + 1u == s_fins);
                if (pmi > er) {
                } else if (synd) {
                    if (send_drains) T = er + 1;  // delivered up to the store's front / a FIN: state machine
                } else if (syn_r) {
                    // reached whatever R, no ACK / an unsent one: NO_ACK / ACK_UNSENT with its front trimmed, or old
                } else if (ge(q.seg_end, wend) || pmi > xr) {
                    T = er + 1;  // decided only as old
                } else {
                    U = xr;  // at or past RCV.NXT: SYN
                }
            } else if (!q.simple)
                T = er + 1;  // FIN / RST: decided only as old
            else if (cand)
                T = drains ? dr : xr;
            else
                T = q.len == 0 || !ge(q.dend - 1u, wend) ? INT_MIN : er + 1;  // (decided at any R: classify())
            if (pmi >= T) T = INT_MIN;
        }
        // wave max of T and min of U (order-preserving unsigned maps through the max scan)
        uint32_t tm, um;
        WaveScan().inclusive_scan((uint32_t)T ^ 0x80000000u, tm, scan_tmp[wv], rocprim::maximum<uint32_t>());
        WaveScan().inclusive_scan(~((uint32_t)U ^ 0x80000000u), um, scan_tmp[wv], rocprim::maximum<uint32_t>());
        const int A = (int)((uint32_t)__builtin_amdgcn_readlane(tm, kWave - 1) ^ 0x80000000u);
        const int Umin = (int)(~(uint32_t)__builtin_amdgcn_readlane(um, kWave - 1) ^ 0x80000000u);
        const int E = synd ? er + 1 : dr;  // a candidate's end
        const bool deliv0 = (cand || synd) && pmi < E;
        // wait for the baton: the next wave in line spins, the others sleep between polls
        uint32_t tv, ep, rn_now, n_now;
        for (;;) {
            baton_poll(&bt, tv, ep, rn_now, n_now);
            if (tv == v) break;
            if (v - tv > 1) __builtin_amdgcn_s_sleep(2);
        }
        {
            const int Rq = (int)(rn_now - rn0);
            if (transparent && ep == e0 && Rq >= A && Rq <= Umin) {
                const uint64_t pk = __ballot(deliv0 && Rq < E);
                if (lane == 0)
                    baton_pass(&bt, v + 1, rn0 + (uint32_t)max(Rq, (int)wmax), n_now + (uint32_t)__builtin_popcountll(pk));
                const uint32_t i2 = idx(v + 2 * kRelayWaves);
                const uint4 g1 = P.rec[i1];
                const Verdict r =
                    classify(q, rn0 + (uint32_t)max(Rq, pmi), wend, false, s_nooo, s_front, s_finp, s_fins, syn_r);
                const uint32_t before =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(pk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pk, 0u));
                if (q.have) {
                    const dk_tcp_view view{i, r.voff, r.vlen};
                    P.out.action[i] = r.act;
                    P.out.view[i] = view;
                    if (r.act == DK_TCP_DELIVERED && n_now + before < cap) dv[n_now + before] = view;
                }
                i = i1;
                i1 = i2;
                g = g1;
                continue;
            }
        }
        const Baton b{v, 0u, DK_U(bt.rn), DK_U(bt.n), DK_U(bt.state), DK_U(bt.nooo), DK_U(bt.front),
                      DK_U(bt.fin_pending), DK_U(bt.fin_seq), DK_U(bt.open_until)};
        // lanes below f are decided by the check against the baton's state (all of them in the common case)
        const bool plain_state = b.state == DK_TCP_ESTABLISHED && b.nooo < DK_TCP_OOO_MAX;
        const uint32_t R = b.rn - rn0;
        uint32_t f = 0;
        Verdict r{};
        uint64_t pmk = 0;
        if (plain_state) {
            r = classify(q, rn0 + max(R, pm), wend, false, b.nooo, b.front, b.fin_pending, b.fin_seq, syn_r);
            const uint64_t bad = __ballot(q.have && !r.ok);
            f = bad ? (uint32_t)__builtin_ctzll(bad) : kWave;
            pmk = __ballot(q.have && lane < f && r.act == DK_TCP_DELIVERED);
            if (!bad && lane == 0) baton_pass(&bt, v + 1, rn0 + max(R, wmax), b.n + (uint32_t)__builtin_popcountll(pmk));
        }
        const uint32_t i2 = idx(v + 2 * kRelayWaves);
        const uint4 g1 = P.rec[i1];
        if (q.have && lane < f) {
            const uint32_t before =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(pmk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pmk, 0u));
            const dk_tcp_view view{i, r.voff, r.vlen};
            P.out.action[i] = r.act;
            P.out.view[i] = view;
            if (r.act == DK_TCP_DELIVERED && b.n + before < cap) dv[b.n + before] = view;
        }
        if (f < kWave) {  // the one-wave walk from lane f on, on the baton's state (the store through lane registers)
            RegStore s{0u, 0u, 0u, 0u, lane};
            if (lane < b.nooo) s = RegStore{sto[0][lane], sto[1][lane], sto[2][lane], sto[3][lane], lane};
            const uint32_t rn_f = rn0 + max(R, (uint32_t)__builtin_amdgcn_readlane(pm, f));  // f = 0: the baton's
            WaveWalk W{P, Walk{b.state, rn_f, reader, bufsz, snd, b.fin_pending, b.fin_seq, b.nooo}, s,
                       Out{dv, b.n + (uint32_t)__builtin_popcountll(pmk), cap}, b.open_until, wend, cnt, lane,
                       scan_tmp[wv]};
            if (plain_state) {  // lane f needs the state machine: process() it, then the parallel check resumes
                const uint4 gf = make_uint4(__builtin_amdgcn_readlane(g.x, f), __builtin_amdgcn_readlane(g.y, f),
                                            __builtin_amdgcn_readlane(g.z, f), __builtin_amdgcn_readlane(g.w, f));
                const uint32_t i_f = __builtin_amdgcn_readlane(i, f);
                dk_tcp_view vf;
                const uint32_t a_f = process(W.s, W.w, gf, i_f, W.o, vf);
                if (lane == 0) {
                    P.out.action[i_f] = (uint8_t)a_f;
                    P.out.view[i_f] = vf;
                }
                if (W.w.state != DK_TCP_ESTABLISHED) W.open_until = i_f + 1;
                W.window(base, i, g, f + 1);
            } else {
                W.window(base, i, g, 0);
            }
            if (lane < DK_TCP_OOO_MAX) {
                sto[0][lane] = W.s.st;
                sto[1][lane] = W.s.rf;
                sto[2][lane] = W.s.of;
                sto[3][lane] = W.s.ln;
            }
            const uint32_t front = W.w.nooo ? W.s.start(0) : 0u;
            if (lane == 0) {
                bt.state = W.w.state;
                bt.rn = W.w.rn;
                bt.nooo = W.w.nooo;
                bt.front = front;
                bt.fin_pending = W.w.fin_pending;
                bt.fin_seq = W.w.fin_seq;
                bt.n = W.o.n;
                bt.open_until = W.open_until;
                bt.epoch = bt.epoch + 1;  // (only the baton's holder writes it)
            }
            // the store entries are written by lanes 0..15 and the baton by lane 0: the release store waits for all
            // of this wave's LDS writes (one wave: in order)
            if (lane == 0) __hip_atomic_store(&bt.turn, v + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        i = i1;
        i1 = i2;
        g = g1;
    }
    __syncthreads();
    if (wv == 0) {
        if (lane == 0) {
            P.out.deliv_start[c] = d0;
            P.open_until[c] = bt.open_until;
            t->state = bt.state;
            t->receive_next = bt.rn;
            t->fin_pending = bt.fin_pending;
            t->fin_seq = bt.fin_seq;
            t->ooo_count = bt.nooo;
            P.out.deliv_count[c] = bt.n;
        }
        if (lane < DK_TCP_OOO_MAX) {
            const bool live = lane < bt.nooo;
            t->ooo_start[lane] = live ? sto[0][lane] : 0u;
            t->ooo[lane] = live ? dk_tcp_view{sto[1][lane], sto[2][lane], sto[3][lane]} : dk_tcp_view{0, 0, 0};
        }
    }
}

// ---------------- The scan walk (round 5): few connections with many segments each ----------------
// The relay walk's per-window work splits into what does not depend on RCV.NXT at the window start (R) and a serial
// hand-off, and on one connection the relay runs both on one CU. The scan walk spreads the first part over the chip
// and turns the hand-off into wave scans:
//   dk_tcp_scan_pre_kernel (every window of every connection in parallel, against the connection's state at the
//     call's start): the relay's precompute (candidates' running maximum, the thresholds A <= R <= U under which
//     classify() decides the whole window, the window's maximum) and each lane's candidate end if it delivers;
//   dk_tcp_scan_kernel (one wave per connection, 64 windows at a time): R of each window = max(R at the batch start,
//     the maxima of the windows before it in the batch) while every window is decided (an exclusive max scan and one
//     compare per window), the deliveries each window makes at its R (its lanes' ends against R) and before it (a
//     sum scan); the first undecided window runs here as in the relay (the state machine for its undecided lanes) and
//     the scan resumes after it; once a window changes the state other than RCV.NXT (store, FIN, connection state)
//     the precomputed windows after it are stale and the wave walks the rest of the connection as the wave walk does
//     (LDS rings); after two undecided windows in a row the next ones go through the rings too (ring runs);
//   dk_tcp_scan_post_kernel (every window in parallel): the decided windows' segments classified at their R, their
//     outputs and deliveries written.
// Same outputs as the other walks (every GPU TCP test runs it).
struct Pre {  // a window's candidates against rn0 (the relay's precompute)
    uint32_t pm, key, wmax;
    bool cand, syn_r, synd;
};
__device__ __forceinline__ Pre pre_window(const Seg& q, uint32_t rn0, uint32_t wend, WaveScan::storage_type& scan) {
    Pre r;
    r.cand = q.cand(false, wend);
    const uint32_t key1 = r.cand && lt(rn0, q.dend) ? q.dend - rn0 : 0u;
    uint32_t pm1;
    WaveScan().exclusive_scan(key1, pm1, 0u, scan, rocprim::maximum<uint32_t>());
    r.syn_r = q.syn && !ge(q.seg_end, wend) && (int)(q.x - rn0) < (int)pm1;
    r.synd = r.syn_r && q.ack_ok;
    r.key = r.synd && lt(rn0, q.seg_end + 1u) ? max(key1, q.seg_end + 1u - rn0) : key1;
    WaveScan().exclusive_scan(r.key, r.pm, 0u, scan, rocprim::maximum<uint32_t>());
    r.wmax = (uint32_t)__builtin_amdgcn_readlane(max(r.pm, r.key), kWave - 1);
    return r;
}
// The connection's state at the call's start, as the scan walk's kernels read it (wave-uniform).
struct ConnHead {
    uint32_t state, rn0, reader, bufsz, snd, wend, nooo, front, finp, fins;
    __device__ __forceinline__ explicit ConnHead(const dk_tcp_conn* t) {
        state = DK_U(t->state);
        rn0 = DK_U(t->receive_next);
        reader = DK_U(t->reader_next);
        bufsz = DK_U(t->buffer_size);
        snd = DK_U(t->send_next);
        wend = reader + bufsz;
        nooo = DK_U(min(t->ooo_count, DK_TCP_OOO_MAX));
        front = nooo ? DK_U(t->ooo_start[0]) : 0u;
        finp = DK_U(t->fin_pending);
        fins = DK_U(t->fin_seq);
    }
};
__device__ __forceinline__ uint32_t scan_ws(const Params& P, uint32_t c) { return P.range[2 * c] / kWave + c; }

#ifndef DK_TCP_SCAN_STATS
#define DK_TCP_SCAN_STATS 0  // diagnostics build: the scan kernel prints its per-connection step counts
#endif
constexpr uint32_t kScanBlock = 256, kScanWaves = kScanBlock / kWave;
#ifndef DK_TCP_SCAN_DEPTH
#define DK_TCP_SCAN_DEPTH 8
#endif
constexpr uint32_t kScanDepth = DK_TCP_SCAN_DEPTH;  // summary batches of 64 windows the scan kernel keeps in flight
#ifndef DK_TCP_SCAN_PREFETCH
#define DK_TCP_SCAN_PREFETCH 1
#endif
constexpr bool kScanPrefetch = DK_TCP_SCAN_PREFETCH != 0;
constexpr uint32_t kScanSum = 3;  // uint4 per window in scan_sum: thresholds, then the delivery-count summary
constexpr uint32_t kScanLow = 4;  // smallest delivering ends a window's count summary carries
constexpr uint32_t kScanPost = 1024;  // decided windows' post records the scan kernel gathers in LDS per burst
// windows the scan kernel walks in the rings after two undecided in a row: kScanRingRun, doubled while that repeats
// (up to kScanRingRunMax), back to kScanRingRun once the scan took more than a batch again
constexpr uint32_t kScanRingRun = 8, kScanRingRunMax = 512;
__global__ __launch_bounds__(kScanBlock) void dk_tcp_scan_pre_kernel(Params P) {
    __shared__ WaveScan::storage_type scan_tmp[kScanWaves];
    const uint32_t c = blockIdx.y, lane = threadIdx.x & (kWave - 1), wv = DK_U(threadIdx.x / kWave);
    const dk_tcp_conn* t = P.conns + c;
    const uint32_t k0 = P.range[2 * c], cnt = P.range[2 * c + 1] - k0;
    const uint32_t nwin = (uint32_t)(((uint64_t)cnt + kWave - 1) / kWave), last = cnt ? cnt - 1 : 0u;
    if (blockIdx.x * kScanWaves >= nwin) return;
    const ConnHead h(t);
    const uint32_t ws0 = scan_ws(P, c);
    for (uint32_t v = blockIdx.x * kScanWaves + wv; v < nwin; v += gridDim.x * kScanWaves) {
        const uint32_t base = v * kWave, lim = min(cnt - base, kWave);
        const uint32_t i = P.svals[k0 + min(base + lane, last)];
        const uint4 g = P.rec[i];
        P.scan_idx[(size_t)(ws0 + v) * kWave + lane] = i;
        P.scan_rec[(size_t)(ws0 + v) * kWave + lane] = g;
        const Seg q(g, lane < lim, h.snd);
        const Pre pr = pre_window(q, h.rn0, h.wend, scan_tmp[wv]);
        // lane j is decided by classify() iff max(R, pm_j) >= T_j, or for a SYN at or past RCV.NXT iff R <= U_j
        // (the relay walk's thresholds, against the state at the call's start) — or, for that SYN, once R is past its
        // end (old: DUPLICATE), R >= Aalt_j; a retransmitted SYN no earlier lane reaches is decided either way
        const int xr = (int)(q.x - h.rn0), er = (int)(q.seg_end - h.rn0), dr = (int)(q.dend - h.rn0), pmi = (int)pr.pm;
        int T = INT_MIN, U = INT_MAX, Aalt = INT_MIN;
        if (q.have) {
            const bool drains =
                q.ack_ok && q.len > 0 && ((h.nooo && q.dend == h.front) || (h.finp && q.dend == h.fins));
            if (ge(q.x, h.wend))
                T = q.x == h.wend ? INT_MAX : INT_MIN;
            else if (q.syn) {
                const bool send_drains = (h.nooo && q.seg_end + 1u == h.front) || (h.finp && q.seg_end + 1u == h.fins);
                if (pmi > er) {
                } else if (pr.synd) {
                    if (send_drains) T = er + 1;
                } else if (pr.syn_r) {
                } else if (ge(q.seg_end, h.wend) || pmi > xr) {
                    T = er + 1;
                } else {
                    U = xr;
                    Aalt = er + 1;
                }
            } else if (!q.simple)
                T = er + 1;
            else if (pr.cand)
                T = drains ? dr : xr;
            else
                T = q.len == 0 || !ge(q.dend - 1u, h.wend) ? INT_MIN : er + 1;  // (decided at any R: classify())
            if (pmi >= T) T = INT_MIN;
        }
        uint32_t tm, um;
        WaveScan().inclusive_scan((uint32_t)T ^ 0x80000000u, tm, scan_tmp[wv], rocprim::maximum<uint32_t>());
        WaveScan().inclusive_scan(~((uint32_t)U ^ 0x80000000u), um, scan_tmp[wv], rocprim::maximum<uint32_t>());
        const int A = (int)((uint32_t)__builtin_amdgcn_readlane(tm, kWave - 1) ^ 0x80000000u);
        const int Umin = (int)(~(uint32_t)__builtin_amdgcn_readlane(um, kWave - 1) ^ 0x80000000u);
        // the window is also decided at R >= A2 when its one upper bound is such a SYN's (no upper bound then)
        const uint64_t ul = __ballot(U != INT_MAX);
        const int A2 = __popcll(ul) == 1 ? max(A, __builtin_amdgcn_readlane(Aalt, (uint32_t)__builtin_ctzll(ul))) : INT_MAX;
        const int E = pr.synd ? er + 1 : dr;
        const bool deliv0 = (pr.cand || pr.synd) && pmi < E;
        P.scan_ends[(size_t)(ws0 + v) * kWave + lane] = deliv0 ? E : INT_MIN;
        // the count summary: n0 delivering lanes, their kScanLow smallest ends ascending and the next one (lo): at any
        // R below lo the window delivers n0 less those of the smallest ends at or below R (a retransmission's end
        // sits below the R its window starts at: the in-order stream's usual outlier)
        int e = deliv0 ? E : INT_MAX, low[kScanLow + 1];
#pragma unroll
        for (uint32_t k = 0; k <= kScanLow; k++) {
            uint32_t mm;  // the wave's minimum by a DPP scan (a shuffle tree is an LDS round trip per level)
            WaveScan().inclusive_scan((uint32_t)e ^ 0x80000000u, mm, scan_tmp[wv], rocprim::minimum<uint32_t>());
            const int m = (int)((uint32_t)__builtin_amdgcn_readlane(mm, kWave - 1) ^ 0x80000000u);
            low[k] = m;
            const uint64_t hit = __ballot(e == m && m != INT_MAX);
            if (hit && lane == (uint32_t)__builtin_ctzll(hit)) e = INT_MAX;
        }
        const uint32_t n0 = (uint32_t)__popcll(__ballot(deliv0));
        if (lane == 0) {
            uint4* sw = P.scan_sum + kScanSum * (size_t)(ws0 + v);
            sw[0] = make_uint4((uint32_t)A, (uint32_t)Umin, pr.wmax, (uint32_t)A2);
            sw[1] = make_uint4(n0, (uint32_t)low[kScanLow], (uint32_t)low[0], (uint32_t)low[1]);
            sw[2] = make_uint4((uint32_t)low[2], (uint32_t)low[3], 0u, 0u);
        }
    }
}

__global__ __launch_bounds__(kWave) void dk_tcp_scan_kernel(Params P) {
    __shared__ WaveScan::storage_type scan_tmp[1];
    __shared__ uint32_t sidx[kIdxSlots][kWave];
    __shared__ uint4 srec[kRecSlots][kWave];
    __shared__ uint4 spost[kScanPost];
    const uint32_t c = blockIdx.x, lane = threadIdx.x;
    dk_tcp_conn* t = P.conns + c;
    const ConnHead h(t);
    const uint32_t k0 = P.range[2 * c], cnt = P.range[2 * c + 1] - k0, all = P.range[2 * c + 2] - k0;
    const uint32_t d0 = k0 + DK_TCP_DELIV_EXTRA * c, cap = all + DK_TCP_DELIV_EXTRA;
    dk_tcp_view* const dv = P.out.deliv + d0;
    const uint32_t nwin = (uint32_t)(((uint64_t)cnt + kWave - 1) / kWave), last = cnt ? cnt - 1 : 0u;
    const uint32_t ws0 = scan_ws(P, c);
    const auto idx = [&](uint32_t v) { return P.svals[k0 + min(v * kWave + lane, last)]; };
    // the walk's state: scalars wave-uniform, the store in lane registers (entry k in lane k)
    Walk w{h.state, h.rn0, h.reader, h.bufsz, h.snd, h.finp, h.fins, h.nooo};
    RegStore s{0u, 0u, 0u, 0u, lane};
    if (lane < h.nooo) {
        const dk_tcp_view e = t->ooo[lane];
        s = RegStore{t->ooo_start[lane], e.ref, e.off, e.len, lane};
    }
    if (lane < 7) {  // the post kernel runs after this one has written the connection back
        const uint32_t hv[7] = {h.rn0, h.wend, h.snd, h.nooo, h.front, h.finp, h.fins};
        uint32_t x = hv[0];
#pragma unroll
        for (uint32_t k = 1; k < 7; k++) x = lane == k ? hv[k] : x;
        P.scan_head[8 * c + lane] = x;
    }
    uint32_t n = 0, open_until = h.state == DK_TCP_ESTABLISHED ? 0xFFFFFFFFu : 0u;
    const bool transparent = h.state == DK_TCP_ESTABLISHED && h.nooo < DK_TCP_OOO_MAX;
    bool stale = !transparent;  // the precomputed windows no longer describe the state
    // lane k of a batch at v: window v + k's two summaries (unconditional loads, clamped to the last window; a lane past
    // it fails the check). Its 64 lanes' ends are read only when R reaches the smallest of them (cx.y).
    struct Batch {
        uint4 sm, c1, c2;
    };
    const auto load_batch = [&](uint32_t v0, Batch& b) {
        const uint4* sw = P.scan_sum + kScanSum * (size_t)(ws0 + min(v0 + lane, nwin - 1));
        b.sm = sw[0];
        b.c1 = sw[1];
        b.c2 = sw[2];
    };
    uint32_t v = 0;
#if DK_TCP_SCAN_STATS
    uint32_t st_batch = 0, st_full = 0, st_slow = 0, st_ring = 0, st_runs = 0, st_restart = 0;
    uint64_t ck_batch = 0, ck_slow = 0, ck_ring = 0, ck_t0 = wall_clock64(), ck_a;
#endif
    // One batch at v from b (loaded for v): the decided windows' R and deliveries; returns how many windows it took
    // (64: all; fewer: window v + f is undecided, or the connection ends).
    // The decided windows' post records ({R, deliveries before it, 1}) gather in LDS (spost, windows vflush ..) and go
    // out in bursts: a global store pending while the next batches' loads are in flight makes every later wait a full
    // vmcnt(0) (loads and stores complete out of order), which would expose the prefetch's latency at every step.
    uint32_t vflush = 0;
    const auto flush_post = [&]() {
        for (uint32_t u = lane; u < v - vflush; u += kWave) P.scan_post[ws0 + vflush + u] = spost[u];
        vflush = v;
    };
    // One batch at v from b (loaded for v): the decided windows' R and deliveries; returns how many windows it took
    // (64: all; fewer: window v + f is undecided, or the connection ends).
    const auto batch_step = [&](const Batch& b) -> uint32_t {
#if DK_TCP_SCAN_STATS
        ck_a = wall_clock64();
#endif
        const uint32_t R0 = w.rn - h.rn0;
        const bool have = v + lane < nwin;
        uint32_t wx;
        WaveScan().exclusive_scan(b.sm.z, wx, 0u, scan_tmp[0], rocprim::maximum<uint32_t>());
        const uint32_t Rk = max(R0, wx);
        const int R = (int)Rk;
        // every test on the batch unconditional (bitwise, no short circuit): a load used only under a branch is sunk
        // into it by the compiler and issued there, a full round trip at every step
        const bool dec = ((R >= (int)b.sm.x) & (R <= (int)b.sm.y)) | (R >= (int)b.sm.w);
        const uint64_t bad = __ballot(!(have & dec));
        const uint32_t f = bad ? (uint32_t)__builtin_ctzll(bad) : kWave;
        // below lo: n0 less the smallest ends at or below R
        const uint32_t fast = b.c1.x - (R >= (int)b.c1.z ? 1u : 0u) - (R >= (int)b.c1.w ? 1u : 0u) -
                              (R >= (int)b.c2.x ? 1u : 0u) - (R >= (int)b.c2.y ? 1u : 0u);
        const bool exact = (lane < f) & (R >= (int)b.c1.y);
        uint32_t cntk = lane < f ? fast : 0u;
        if (exact) {  // count the window's ends above R
            const int4* er = reinterpret_cast<const int4*>(P.scan_ends + (size_t)(ws0 + v + lane) * kWave);
            cntk = 0;
#pragma unroll
            for (uint32_t m = 0; m < kWave / 4; m++) {
                const int4 e = er[m];
                cntk += (R < e.x ? 1u : 0u) + (R < e.y ? 1u : 0u) + (R < e.z ? 1u : 0u) + (R < e.w ? 1u : 0u);
            }
        }
        uint32_t nx;
        WaveScan().exclusive_scan(cntk, nx, 0u, scan_tmp[0], rocprim::plus<uint32_t>());
        if (lane < f) spost[v - vflush + lane] = make_uint4(Rk, n + nx, 1u, 0u);
        if (f > 0) {
            w.rn = h.rn0 + (uint32_t)__builtin_amdgcn_readlane(max(Rk, b.sm.z), f - 1);
            n += (uint32_t)__builtin_amdgcn_readlane(nx + cntk, f - 1);
        }
        v += f;
#if DK_TCP_SCAN_STATS
        st_batch++;
        st_full += f == kWave;
        ck_batch += wall_clock64() - ck_a;
#endif
        return f;
    };
    // window v is not decided by the thresholds: the relay's slow path on the walk's state
    const auto slow_window = [&]() {
#if DK_TCP_SCAN_STATS
        st_slow++;
        const uint64_t ck_s = wall_clock64();
#endif
        const uint32_t base = v * kWave, lim = min(cnt - base, kWave);
        const uint32_t i = P.scan_idx[(size_t)(ws0 + v) * kWave + lane];
        const uint4 g = P.scan_rec[(size_t)(ws0 + v) * kWave + lane];
        if (lane == 0) P.scan_post[ws0 + v] = make_uint4(0u, 0u, 0u, 0u);
        const Seg q(g, lane < lim, h.snd);
        const Pre pr = pre_window(q, h.rn0, h.wend, scan_tmp[0]);
        const uint32_t R = w.rn - h.rn0;
        const Verdict r = classify(q, h.rn0 + max(R, pr.pm), h.wend, false, w.nooo, w.nooo ? s.start(0) : 0u,
                                   w.fin_pending, w.fin_seq, pr.syn_r);
        const uint64_t bl = __ballot(q.have && !r.ok);
        const uint32_t fl = bl ? (uint32_t)__builtin_ctzll(bl) : kWave;
        const uint64_t pmk = __ballot(q.have && lane < fl && r.act == DK_TCP_DELIVERED);
        if (q.have && lane < fl) {
            const uint32_t before =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(pmk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pmk, 0u));
            const dk_tcp_view view{i, r.voff, r.vlen};
            P.out.action[i] = r.act;
            P.out.view[i] = view;
            if (r.act == DK_TCP_DELIVERED && n + before < cap) dv[n + before] = view;
        }
        n += (uint32_t)__builtin_popcountll(pmk);
        if (fl == kWave) {
            w.rn = h.rn0 + max(R, pr.wmax);
        } else {  // lane fl needs the state machine, then the one-wave walk resumes after it
            w.rn = h.rn0 + max(R, (uint32_t)__builtin_amdgcn_readlane(pr.pm, fl));
            WaveWalk W{P, w, s, Out{dv, n, cap}, open_until, h.wend, cnt, lane, scan_tmp[0]};
            const uint4 gf = make_uint4(__builtin_amdgcn_readlane(g.x, fl), __builtin_amdgcn_readlane(g.y, fl),
                                        __builtin_amdgcn_readlane(g.z, fl), __builtin_amdgcn_readlane(g.w, fl));
            const uint32_t i_f = __builtin_amdgcn_readlane(i, fl);
            dk_tcp_view vf;
            const uint32_t a_f = process(W.s, W.w, gf, i_f, W.o, vf);
            if (lane == 0) {
                P.out.action[i_f] = (uint8_t)a_f;
                P.out.view[i_f] = vf;
            }
            if (W.w.state != DK_TCP_ESTABLISHED) W.open_until = i_f + 1;
            W.window(base, i, g, fl + 1);
            w = W.w;
            s = W.s;
            n = W.o.n;
            open_until = W.open_until;
        }
        v++;
#if DK_TCP_SCAN_STATS
        ck_slow += wall_clock64() - ck_s;
#endif
    };
    // windows v .. v1 - 1 as the wave walk does (the LDS rings)
    const auto ring_run = [&](uint32_t v1) {
#if DK_TCP_SCAN_STATS
        st_ring += v1 - v;
        st_runs++;
        const uint64_t ck_r = wall_clock64();
#endif
        for (uint32_t u = v + lane; u < v1; u += kWave) P.scan_post[ws0 + u] = make_uint4(0u, 0u, 0u, 0u);
        WaveWalk W{P, w, s, Out{dv, n, cap}, open_until, h.wend, cnt, lane, scan_tmp[0]};
        ring_walk(P, W, sidx, srec, k0, cnt, v, v1);
        w = W.w;
        s = W.s;
        n = W.o.n;
        open_until = W.open_until;
        v = v1;
#if DK_TCP_SCAN_STATS
        ck_ring += wall_clock64() - ck_r;
#endif
    };
    // Super-rounds of kScanDepth batches (b[j] for v + 64 j, 48 bytes per lane each) loaded together and then stepped
    // through: one load latency per kScanDepth steps. (Reloading each batch kScanDepth - 1 ahead as it is used keeps
    // loads in flight across the loop's back edge, where the compiler's waits fall back to vmcnt(0) and expose a
    // reload's latency every other step.)
    Batch b[kScanDepth];
    uint32_t last_slow = 0xFFFFFFFEu, run = kScanRingRun;  // the last window the slow path took, the next ring run
    uint32_t pre = 0xFFFFFFFFu;  // the window b[] was loaded for ahead of the super-round (the slow path's successor)
    while (v < nwin && !stale) {
#if DK_TCP_SCAN_STATS
        st_restart++;
#endif
        bool more = true;
        while (more && v < nwin) {
            if (v + kScanDepth * kWave > vflush + kScanPost) flush_post();  // room for this round's records
            if (pre != v) {
#pragma unroll
                for (uint32_t j = 0; j < kScanDepth; j++)
                    if (v + j * kWave < nwin) load_batch(v + j * kWave, b[j]);  // (wave-uniform: no loads past the end)
            }
            pre = 0xFFFFFFFFu;
#pragma unroll
            for (uint32_t j = 0; j < kScanDepth; j++)
                if (more && batch_step(b[j]) < kWave) more = false;
        }
        flush_post();  // before the slow path's and the rings' own stores
        if (v >= nwin) break;
        if (v == last_slow + 1) {  // two undecided windows in a row (reordering): the next ones in the rings
            ring_run(v + min(run, nwin - v));
            last_slow = v - 1;
            run = min(2 * run, kScanRingRunMax);
        } else {
            if (v - last_slow > kWave) run = kScanRingRun;
            last_slow = v;
            // the batches after this window, loaded under the slow path's own round trip (DK_TCP_SCAN_PREFETCH)
            if (kScanPrefetch) {
#pragma unroll
                for (uint32_t j = 0; j < kScanDepth; j++)
                    if (v + 1 + j * kWave < nwin) load_batch(v + 1 + j * kWave, b[j]);
                pre = v + 1;
            }
            slow_window();
        }
        vflush = v;
        const uint32_t front = w.nooo ? s.start(0) : 0u;
        stale = w.state != h.state || w.nooo != h.nooo || front != h.front || w.fin_pending != h.finp ||
                w.fin_seq != h.fins;
    }
    if (v < nwin) ring_run(nwin);  // stale: the rest as the wave walk does
#if DK_TCP_SCAN_STATS
    if (lane == 0)
        printf("{\"scan_stats\": 1, \"conn\": %u, \"windows\": %u, \"batch_steps\": %u, \"full_steps\": %u, "
               "\"slow_windows\": %u, \"ring_windows\": %u, \"ring_runs\": %u, \"restarts\": %u, \"stale\": %u, "
               "\"us_total\": %.2f, \"us_batch_steps\": %.2f, \"us_slow\": %.2f, \"us_ring\": %.2f}\n",
               c, nwin, st_batch, st_full, st_slow, st_ring, st_runs, st_restart, (uint32_t)stale,
               (double)(wall_clock64() - ck_t0) / 100.0, (double)ck_batch / 100.0, (double)ck_slow / 100.0,
               (double)ck_ring / 100.0);
#endif
    if (lane == 0) {
        P.out.deliv_start[c] = d0;
        P.open_until[c] = open_until;
        t->state = w.state;
        t->receive_next = w.rn;
        t->fin_pending = w.fin_pending;
        t->fin_seq = w.fin_seq;
        t->ooo_count = w.nooo;
        P.out.deliv_count[c] = n;
    }
    if (lane < DK_TCP_OOO_MAX) {
        const bool live = lane < w.nooo;
        t->ooo_start[lane] = live ? s.st : 0u;
        t->ooo[lane] = live ? dk_tcp_view{s.rf, s.of, s.ln} : dk_tcp_view{0, 0, 0};
    }
}

__global__ __launch_bounds__(kScanBlock) void dk_tcp_scan_post_kernel(Params P) {
    __shared__ WaveScan::storage_type scan_tmp[kScanWaves];
    const uint32_t c = blockIdx.y, lane = threadIdx.x & (kWave - 1), wv = DK_U(threadIdx.x / kWave);
    const uint32_t k0 = P.range[2 * c], cnt = P.range[2 * c + 1] - k0, all = P.range[2 * c + 2] - k0;
    const uint32_t nwin = (uint32_t)(((uint64_t)cnt + kWave - 1) / kWave), last = cnt ? cnt - 1 : 0u;
    if (blockIdx.x * kScanWaves >= nwin) return;
    const uint32_t d0 = k0 + DK_TCP_DELIV_EXTRA * c, cap = all + DK_TCP_DELIV_EXTRA;
    dk_tcp_view* const dv = P.out.deliv + d0;
    const uint32_t ws0 = scan_ws(P, c);
    // the state at the call's start (the scan kernel has written the connection's final state back by now): decided
    // windows only exist while the state other than RCV.NXT equals it
    const uint32_t* hd = P.scan_head + 8 * c;
    const uint32_t rn0 = DK_U(hd[0]), wend = DK_U(hd[1]), snd = DK_U(hd[2]), nooo = DK_U(hd[3]), front = DK_U(hd[4]),
                   finp = DK_U(hd[5]), fins = DK_U(hd[6]);
    for (uint32_t v = blockIdx.x * kScanWaves + wv; v < nwin; v += gridDim.x * kScanWaves) {
        const uint4 po = P.scan_post[ws0 + v];
        const uint32_t i = P.scan_idx[(size_t)(ws0 + v) * kWave + lane];  // (issued with po: one round trip)
        const uint4 g = P.scan_rec[(size_t)(ws0 + v) * kWave + lane];
        if (DK_U(po.z) != 1u) continue;
        const uint32_t base = v * kWave, lim = min(cnt - base, kWave);
        const Seg q(g, lane < lim, snd);
        const Pre pr = pre_window(q, rn0, wend, scan_tmp[wv]);
        const int Rq = (int)DK_U(po.x), pmi = (int)pr.pm;
        const int er = (int)(q.seg_end - rn0), dr = (int)(q.dend - rn0);
        const int E = pr.synd ? er + 1 : dr;
        const bool deliv0 = (pr.cand || pr.synd) && pmi < E;
        const uint64_t pk = __ballot(deliv0 && Rq < E);
        const uint32_t n0 = DK_U(po.y);
        const Verdict r = classify(q, rn0 + (uint32_t)max(Rq, pmi), wend, false, nooo, front, finp, fins, pr.syn_r);
        const uint32_t before =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(pk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pk, 0u));
        if (q.have) {
            const dk_tcp_view view{i, r.voff, r.vlen};
            P.out.action[i] = r.act;
            P.out.view[i] = view;
            if (r.act == DK_TCP_DELIVERED && n0 + before < cap) dv[n0 + before] = view;
        }
    }
}
#undef DK_U

// Which walk runs: `force` (dk_diag_tcp_set_walk: 0 lane, 1 wave, 2 relay, 3 scan, -1 the rule); otherwise one lane
// per connection below kWaveWalkMinSegs segments per connection, the scan walk from kScanMinSegs (16 windows) for up
// to DK_TCP_SCAN_MAX_CONNS connections — unless the context's last finished call showed a reordered stream (below) —,
// else one wave per connection.
// 1M segments (sessions r05zt-r05zv, profiles/r05_tcp_walks.jsonl): 1 connection scan 0.87 ms, relay 3.8, wave 12.7;
// 16: scan 0.29, wave 0.94; 64: scan 0.22, relay 0.23, wave 0.31; 256: scan 0.19, wave 0.18; 1,024: wave 0.14, relay
// 0.16, scan 0.18 (a wave per connection fills the chip). The relay walk stays selectable.
constexpr uint32_t kWaveWalkMinSegs = 8;
constexpr uint32_t kScanMinSegs = 16 * kWave;
#ifndef DK_TCP_SCAN_MAX_CONNS
#define DK_TCP_SCAN_MAX_CONNS 256
#endif
// Up to this many connections (waves) the wave walk streams through LDS rings (kRing): 8 waves per CU at most on
// 256 CUs, 12 KiB of LDS each.
#ifndef DK_TCP_DEEP_MAX_CONNS
#define DK_TCP_DEEP_MAX_CONNS 2048
#endif
constexpr uint32_t kDeepAheadMaxConns = DK_TCP_DEEP_MAX_CONNS;
// The stream's shape (the scan walk's weak spot): a window in which a segment goes to the out-of-order store is not
// decided by the scan's thresholds and runs the state machine through the rings, as the wave walk does, after the
// precompute the scan walk paid for it — so on reordered streams the wave walk is ahead (the bench's 1M-segment stream
// with local reordering: 16 / 64 / 256 connections 0.60 / 0.39 / 0.22 ms against the scan walk's 0.63 / 0.42 / 0.25,
// at 29 % / 6.6 % / 0.1 % of the segments STORED, i.e. 100 % / 99 % / 6 % of its 64-segment windows storing), while on
// in-order streams (no segment stored) the scan walk is (1 / 16 / 64 / 256 connections 0.41 / 0.21 / 0.18 / 0.17
// against 12.7 / 0.85 / 0.28 / 0.17 ms). STORED is the same in every walk (bit-exact outputs), so the count the fix
// kernel takes is a walk-independent measure of the shape. Rule: from kShapeMinConns connections on, a context whose
// last finished call stored at least 1 segment in kShapeStoredDen (0.1 %: ~6 % of the windows) takes the wave walk.
// Below 16 connections one wave per connection is too little of the chip (1 connection: 12.7 ms) whatever the shape.
constexpr uint32_t kShapeMinConns = 16, kShapeStoredDen = 1024;
enum Walker { kLaneWalk = 0, kWaveWalk = 1, kRelayWalk = 2, kScanWalk = 3 };
Walker pick_walk(uint32_t n, uint32_t nconns, int force, bool reordered) {
    if (nconns > (1u << 24)) return kLaneWalk;  // grid of nconns workgroups
    if (force == 3 && nconns > 65535) return kRelayWalk;  // the scan walk's grids have one row per connection
    if (force >= 0 && force <= 3) return (Walker)force;
    if ((uint64_t)n < (uint64_t)kWaveWalkMinSegs * nconns) return kLaneWalk;
    if ((uint64_t)n >= (uint64_t)kScanMinSegs * nconns && nconns <= DK_TCP_SCAN_MAX_CONNS &&
        !(reordered && nconns >= kShapeMinConns))
        return kScanWalk;
    return kWaveWalk;
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

template <class T>
int grow(T*& p, size_t& cap, size_t n) {
    if (cap >= n) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return ENOMEM;
    cap = n;
    return 0;
}

}  // namespace
}  // namespace dk_tcp

// One scratch set per context (sort keys, sorted pairs, records, ranges, sort temp). Calls are ordered on their
// streams; a call on a different stream than the previous one first waits for the previous call's work (`last`), so
// two streams never overlap on the scratch, and growing it waits for that work before freeing.
struct dk_tcp_ctx {
    int device = 0;
    int walk = -1;  // dk_diag_tcp_set_walk: 0 lane, 1 wave, 2 relay, 3 scan, -1 the engine's rule
    int relay_waves = 8;  // dk_diag_tcp_set_walk (4 / 8 / 16; 8 measured best, session r05r)
    hipEvent_t last = nullptr;
    hipStream_t last_stream = nullptr;
    bool used = false;
    uint32_t *keys = nullptr, *skeys = nullptr, *svals = nullptr, *range = nullptr, *cls = nullptr, *open_until = nullptr;
    size_t keys_cap = 0, skeys_cap = 0, svals_cap = 0, range_cap = 0, cls_cap = 0, open_cap = 0;
    uint32_t* csort = nullptr;  // the counting pass's per-tile key counts
    size_t csort_cap = 0;
    uint4* rec = nullptr;
    size_t rec_cap = 0;
    uint8_t* temp = nullptr;
    size_t temp_cap = 0;
    uint4 *scan_sum = nullptr, *scan_post = nullptr;  // the scan walk's per-window scratch (dk_tcp::Params)
    int* scan_ends = nullptr;
    uint32_t* scan_idx = nullptr;
    uint4* scan_rec = nullptr;
    size_t scan_idx_cap = 0, scan_rec_cap = 0;
    uint32_t* scan_head = nullptr;
    size_t scan_sum_cap = 0, scan_post_cap = 0, scan_ends_cap = 0, scan_head_cap = 0;
    // the stream's shape (pick_walk): the fix kernel's STORED count of each call, in host-mapped memory
    uint32_t* shape = nullptr;            // device u64 (8-byte aligned: hipMalloc), zero between calls
    volatile uint32_t* shape_host = nullptr;  // host-mapped [3] {STORED, n, call}
    uint32_t* shape_host_dev = nullptr;   // its device alias
    uint32_t calls = 0;                   // calls issued (the number the next fix kernel writes is calls + 1)
    uint32_t seen = 0;                    // the last call whose count was read
    bool reordered = false;               // the last read count: >= 1 in kShapeStoredDen segments STORED
    int last_walk = -1;                   // the walk the last call ran (dk_diag_tcp_last_walk)
    int sort = -1;                        // dk_diag_tcp_set_sort: 1 the radix sort always, -1 the rule
};

extern "C" {

int dk_tcp_ctx_create(int32_t device, dk_tcp_ctx** out) {
    if (!out) return EINVAL;
    *out = nullptr;
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || device < 0 || device >= nd) return EINVAL;
    dk_tcp::DeviceGuard g(device);
    dk_tcp_ctx* t = new dk_tcp_ctx();
    t->device = device;
    void* hs = nullptr;
    if (hipEventCreateWithFlags(&t->last, hipEventDisableTiming) != hipSuccess) {
        delete t;
        return EINVAL;
    }
    if (hipMalloc(&t->shape, 2 * sizeof(uint32_t)) != hipSuccess || hipMemset(t->shape, 0, 8) != hipSuccess ||
        hipHostMalloc(&hs, 4 * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&t->shape_host_dev), hs, 0) != hipSuccess) {
        if (hs) (void)hipHostFree(hs);
        if (t->shape) (void)hipFree(t->shape);
        (void)hipEventDestroy(t->last);
        delete t;
        return ENOMEM;
    }
    t->shape_host = static_cast<volatile uint32_t*>(hs);
    t->shape_host[0] = t->shape_host[1] = t->shape_host[2] = 0;
    *out = t;
    return 0;
}

int dk_diag_tcp_last_walk(const dk_tcp_ctx* t) { return t ? t->last_walk : -1; }

int dk_diag_tcp_set_walk(dk_tcp_ctx* t, int32_t walk, int32_t relay_waves) {
    if (!t || walk < -1 || walk > 3) return EINVAL;
    t->walk = walk;
    t->relay_waves = relay_waves == 4 || relay_waves == 16 ? relay_waves : 8;
    return 0;
}

int dk_diag_tcp_set_sort(dk_tcp_ctx* t, int32_t sort) {
    if (!t || (sort != -1 && sort != 1)) return EINVAL;
    t->sort = sort;
    return 0;
}

void dk_tcp_ctx_destroy(dk_tcp_ctx* t) {
    if (!t) return;
    dk_tcp::DeviceGuard g(t->device);
    if (t->used) (void)hipEventSynchronize(t->last);
    for (void* p : {(void*)t->keys, (void*)t->skeys, (void*)t->svals, (void*)t->range, (void*)t->rec, (void*)t->temp,
                    (void*)t->cls, (void*)t->open_until, (void*)t->scan_sum, (void*)t->scan_post, (void*)t->scan_ends,
                    (void*)t->scan_idx, (void*)t->scan_rec,
                    (void*)t->scan_head, (void*)t->shape, (void*)t->csort})
        if (p) (void)hipFree(p);
    if (t->shape_host) (void)hipHostFree(const_cast<uint32_t*>(t->shape_host));
    (void)hipEventDestroy(t->last);
    delete t;
}

int dk_tcp_rx_process(dk_tcp_ctx* t, const dk_rx_results* rx, uint32_t n, dk_tcp_conn* conns, uint32_t nconns,
                      const dk_tcp_out* out, void* stream) {
    using namespace dk_tcp;
    if (!t || !rx || !out) return EINVAL;
    if (n && (!rx->meta || !rx->flow_id || !rx->payload || !rx->tcp_seq || !rx->tcp_ack || !out->action || !out->view))
        return EINVAL;
    if (nconns && (!conns || !out->deliv || !out->deliv_start || !out->deliv_count)) return EINVAL;
    if (reinterpret_cast<uintptr_t>(conns) & 15) return EINVAL;  // the key kernel reads each entry's head as 16 bytes
    if (n > 0x7FFFFFFFu || nconns > 0x7FFFFFFFu ||
        (uint64_t)n + (uint64_t)DK_TCP_DELIV_EXTRA * nconns > 0xFFFFFFFFull)
        return EINVAL;
    if (n == 0 && nconns == 0) return 0;
    DeviceGuard g(t->device);
    const hipStream_t s = (hipStream_t)stream;
    int rc = 0;
    if (t->used && t->last_stream != s && hipStreamWaitEvent(s, t->last, 0) != hipSuccess) return EINVAL;
    const bool grows = t->keys_cap < n || t->rec_cap < n || t->range_cap < 2 * (size_t)nconns + 1 || t->cls_cap < n ||
                       t->open_cap < nconns;
    if (t->used && grows && hipEventSynchronize(t->last) != hipSuccess) return EINVAL;  // in-flight work on the scratch
    if ((rc = grow(t->keys, t->keys_cap, n)) || (rc = grow(t->skeys, t->skeys_cap, n)) ||
        (rc = grow(t->svals, t->svals_cap, n)) || (rc = grow(t->rec, t->rec_cap, n)) ||
        (rc = grow(t->range, t->range_cap, 2 * (size_t)nconns + 1)) || (rc = grow(t->cls, t->cls_cap, n)) ||
        (rc = grow(t->open_until, t->open_cap, nconns)))
        return rc;
    // The shape of the stream from the last call whose fix kernel has completed (never waited for: a call still in
    // flight leaves the previous reading in place).
    if (t->calls != t->seen && t->shape_host[2] != t->seen) {
        const uint32_t call = t->shape_host[2];
        const uint32_t stored = t->shape_host[0], segs = t->shape_host[1];
        if (call == t->shape_host[2] && call != t->seen) {  // a consistent snapshot of that call's words
            t->seen = call;
            t->reordered = (uint64_t)stored * dk_tcp::kShapeStoredDen >= (uint64_t)std::max(segs, 1u);
        }
    }
    const dk_tcp::Walker walker = nconns ? dk_tcp::pick_walk(n, nconns, t->walk, t->reordered) : dk_tcp::kLaneWalk;
    t->last_walk = (int)walker;
    if (walker == dk_tcp::kScanWalk) {  // windows: ws = range[2c] / 64 + c + v < n / 64 + nconns + 1
        const size_t nw = (size_t)n / 64 + nconns + 1;
        if (t->used &&
            (t->scan_sum_cap < dk_tcp::kScanSum * nw || t->scan_ends_cap < nw * 64 || t->scan_head_cap < 8ull * nconns ||
             t->scan_idx_cap < nw * 64 || t->scan_rec_cap < nw * 64) &&
            hipEventSynchronize(t->last) != hipSuccess)
            return EINVAL;
        if ((rc = grow(t->scan_sum, t->scan_sum_cap, dk_tcp::kScanSum * nw)) || (rc = grow(t->scan_post, t->scan_post_cap, nw)) ||
            (rc = grow(t->scan_ends, t->scan_ends_cap, nw * 64)) || (rc = grow(t->scan_idx, t->scan_idx_cap, nw * 64)) ||
            (rc = grow(t->scan_rec, t->scan_rec_cap, nw * 64)) ||
            (rc = grow(t->scan_head, t->scan_head_cap, 8 * (size_t)nconns)))
            return rc;
    }
    int bits = 1;
    while (bits < 32 && (1ull << bits) <= 2ull * nconns) bits++;  // keys are 0 .. 2 nconns
    const rocprim::counting_iterator<uint32_t> index(0);
    // the batch's order by connection: one counting pass over the whole key (its scan writes the ranges) up to
    // kSortMaxRows table rows, else the radix sort and the range kernel
    const uint32_t nkeys = 2 * nconns + 1, ntiles = (n + dk_tcp::kSortTile - 1) / dk_tcp::kSortTile;
    const bool csort = nconns && n && nconns <= dk_tcp::kSortMaxRows && t->sort != 1;
    if (csort) {
        const size_t hb = (size_t)nkeys * ntiles;
        if (t->used && t->csort_cap < hb && hipEventSynchronize(t->last) != hipSuccess) return EINVAL;
        if ((rc = grow(t->csort, t->csort_cap, hb))) return rc;
    } else {
        size_t sort_bytes = 0;
        if (rocprim::radix_sort_pairs<SortConfig>(nullptr, sort_bytes, t->keys, t->skeys, index, t->svals, n, 0, bits,
                                                  s) != hipSuccess)
            return EINVAL;
        if (t->used && t->temp_cap < sort_bytes && hipEventSynchronize(t->last) != hipSuccess) return EINVAL;
        if ((rc = grow(t->temp, t->temp_cap, sort_bytes))) return rc;
    }

    Params P{};
    P.meta = rx->meta;
    P.flow_id = rx->flow_id;
    P.seq = rx->tcp_seq;
    P.ack = rx->tcp_ack;
    P.payload = rx->payload;
    P.n = n;
    P.conns = conns;
    P.nconns = nconns;
    P.keys = t->keys;
    P.skeys = t->skeys;
    P.svals = t->svals;
    P.rec = t->rec;
    P.range = t->range;
    P.cls = t->cls;
    P.open_until = t->open_until;
    P.scan_sum = t->scan_sum;
    P.scan_post = t->scan_post;
    P.scan_ends = t->scan_ends;
    P.scan_idx = t->scan_idx;
    P.scan_rec = t->scan_rec;
    P.scan_head = t->scan_head;
    P.shape = t->shape;
    P.shape_host = t->shape_host_dev;
    P.call = t->calls + 1;
    P.out = *out;
    const dim3 gn((n + kBlock - 1) / kBlock), gr((2 * nconns + kBlock) / kBlock), gc((nconns + kWalkBlock - 1) / kWalkBlock);
    if (n) hipLaunchKernelGGL(dk_tcp_key_kernel, gn, dim3(kBlock), 0, s, P);
    if (csort) {
        const auto pass = [&](const SortPass& S, uint32_t* range) {
            hipLaunchKernelGGL(dk_tcp_sort_count_kernel, dim3(ntiles), dim3(kSortBlock), 0, s, n, S);
            hipLaunchKernelGGL(dk_tcp_sort_scan_kernel, dim3(1), dim3(kSortScanBlock), 0, s, S.H, S.nbuck * ntiles,
                               ntiles, range);
            hipLaunchKernelGGL(dk_tcp_sort_scatter_kernel, dim3(ntiles), dim3(kSortBlock), 0, s, n, S);
        };
        uint32_t mask = 1;  // the key's bits: 2^bits - 1 >= nkeys - 1
        while (mask < nkeys - 1) mask = 2 * mask + 1;
        pass(SortPass{t->keys, nullptr, nullptr, t->svals, t->csort, 0u, mask, nkeys}, t->range);
    } else {
        if (n) {
            size_t b = t->temp_cap;
            if (rocprim::radix_sort_pairs<SortConfig>(t->temp, b, t->keys, t->skeys, index, t->svals, n, 0, bits, s) !=
                hipSuccess)
                return EINVAL;
        }
        if (nconns) hipLaunchKernelGGL(dk_tcp_range_kernel, gr, dim3(kBlock), 0, s, P);
    }
    if (nconns) {
        switch (walker) {
            case kScanWalk: {
                const uint32_t per = (uint32_t)(((uint64_t)n / kWave / nconns + kScanWaves) / kScanWaves);
                const dim3 gs(std::min<uint32_t>(std::max<uint32_t>(per, 1u), 65535u), nconns);
                hipLaunchKernelGGL(dk_tcp_scan_pre_kernel, gs, dim3(kScanBlock), 0, s, P);
                hipLaunchKernelGGL(dk_tcp_scan_kernel, dim3(nconns), dim3(kWave), 0, s, P);
                hipLaunchKernelGGL(dk_tcp_scan_post_kernel, gs, dim3(kScanBlock), 0, s, P);
                break;
            }
            case kRelayWalk:
                if (t->relay_waves == 4)
                    hipLaunchKernelGGL(dk_tcp_relay_walk_kernel<4>, dim3(nconns), dim3(4 * kWave), 0, s, P);
                else if (t->relay_waves == 16)
                    hipLaunchKernelGGL(dk_tcp_relay_walk_kernel<16>, dim3(nconns), dim3(16 * kWave), 0, s, P);
                else
                    hipLaunchKernelGGL(dk_tcp_relay_walk_kernel<8>, dim3(nconns), dim3(8 * kWave), 0, s, P);
                break;
            case kWaveWalk:
                if (nconns <= kDeepAheadMaxConns)
                    hipLaunchKernelGGL(dk_tcp_wave_walk_kernel<true>, dim3(nconns), dim3(kWave), 0, s, P);
                else
                    hipLaunchKernelGGL(dk_tcp_wave_walk_kernel<false>, dim3(nconns), dim3(kWave), 0, s, P);
                break;
            default:
                hipLaunchKernelGGL(dk_tcp_walk_kernel, gc, dim3(kWalkBlock), 0, s, P);
        }
    }
    if (n && nconns) {
        hipLaunchKernelGGL(dk_tcp_fix_kernel, gn, dim3(kBlock), 0, s, P);
        t->calls++;
    }
    if (hipGetLastError() != hipSuccess) return EINVAL;
    if (hipEventRecord(t->last, s) != hipSuccess) return EINVAL;
    t->last_stream = s;
    t->used = true;
    return 0;
}

}  // extern "C"
