// rx_host.cpp — host driver behind include/dk_rx.h: receive contexts, the device socket table, the HBM-resident
// batch call, and the pinned-host pipeline (NIC ring / raw-socket buffer -> HBM -> results -> host).
//
// Replaces, on the receive side, the state SharedInetStack::new sets up (src/rust/inetstack/mod.rs:69-93): the local
// IPv4 address (demikernel/config.rs:115), the rx checksum offload flags (runtime/network/config/tcp.rs:48-51,
// udp.rs:26-30) and the socket maps TcpPeer::addresses / UdpPeer::addresses (tcp/peer.rs, udp/peer.rs:38).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "lds_table.h"
#include "rx_common.h"
#include "rx_plan.h"

static_assert(sizeof(dk_tcp_opt) == 12 && sizeof(dk_tcp_opts) == 96, "dk_rx.h tcp option record layout");

namespace {

constexpr int kPipeStreams = 3;
constexpr uint32_t kDefaultChunkFrames = 1u << 16;
constexpr uint64_t kMaxChunkBytes = 256ull << 20;
constexpr size_t kMaxStreamSlots = 8;

// Counter scratch of one stream's launches: the per-workgroup counter rows (flush_counters, rx_kernels.hip) in two
// halves (a launch writes one while the previous launch's rows may still be pending in the other), the small-frame
// kernel's deferral masks, and the pending-rows state of DK_RX_BATCH_DEFER_COUNTS: the rows of the last deferred launch,
// which the next launch on the stream adds to that launch's counters in-kernel (RowCombine, rx_common.h), or
// dk_rx_counts_flush with dk_flow_reduce_kernel.
struct CountScratch {
    uint32_t* rows = nullptr;
    size_t rows_words = 0;   // words per half
    uint32_t half = 0;       // the half the next launch writes
    uint64_t* defer = nullptr;  // the small-frame kernel's per-chunk deferral masks
    size_t ndefer = 0;
    bool pending = false;
    dk::RowCombine pend{};       // rows, nrows, row_words, row_stride, flow_words, nflows, counts, verdicts
    uint32_t* tail = nullptr;    // the staged kernel's dynamic-tail counters: two sets of dk::kTailSetWords (zeroed)
    uint32_t tail_set = 0;       // the set the next tail launch uses (each launch zeroes the other one)
};

// A context's scratch is keyed by stream: calls on different streams never share counter rows, so their
// launches may run concurrently. Past kMaxStreamSlots streams the least recently used slot is taken over, and the new
// stream first waits for the slot's last launch (its event). Streams must outlive the context or be released with
// dk_rx_stream_forget (dk_rx.h), so the handle a slot keeps is valid whenever it is used.
struct StreamSlot {
    hipStream_t stream = nullptr;
    CountScratch cs;
    hipEvent_t last = nullptr;  // ordering event for a takeover (created with the slot's first use)
    bool used = false;          // the slot belongs to `stream`
    bool recorded = false;      // `last` was recorded after the slot's most recent launch
    uint64_t stamp = 0;
};

struct Stage {  // device staging for one pipeline stream
    hipStream_t stream = nullptr;
    uint8_t* frames = nullptr;
    uint64_t frames_cap = 0;
    uint32_t* desc_off = nullptr;
    uint16_t* desc_len = nullptr;
    uint32_t* res = nullptr;  // 9 result arrays of chunk_cap entries
    uint32_t cap = 0;
    dk_tcp_opts* opts = nullptr;  // tcp_opts records of chunk_cap entries (allocated when a call asks for them)
    uint32_t opts_cap = 0;
};

// Tuning overrides (-1 = the host rule). A context starts on the built-in rule; only dk_diag_rx_set_tuning changes
// them (dk_diag.h). The process environment is never read: a LibOS process cannot inherit a different kernel family.
struct Tuning {
    int32_t stage = -1, split = -1, small = -1, sched = -1, grid = -1, grid_per_cu = -1, debug = 0;
    int32_t lds_table = -1;  // 0: Active lookups never use the LDS table
    int32_t tail = -1;       // staged kernel's dynamic tail rounds (0 off)
    int32_t udp_table = -1;  // small-frame kernel, local UDP binds: 0 the port table, 1 the LDS bind table whenever it
                             // fits
    int32_t host_zc = -1;  // dk_rx_process_host: read mapped pinned frames in place (-1/1 when mapped, 0 never)
};

}  // namespace

struct dk_rx_ctx {
    dk_rx_cfg cfg{};
    uint32_t* table = nullptr;  // device: (mask + 1) * 4 u32 of Active slots, the kPortTabWords port table, the LDS
                                // Active table's lt_words, then the compact UDP bind table's ub_words (rx_common.h; 0
                                // when not built)
    uint32_t table_mask = 0;
    uint32_t lt_n = 0, lt_b = 0, lt_words = 0;
    uint32_t lt_occ_dyn = ~0u, lt_occ_family = ~0u, lt_occ_blocks = 0;  // occupancy cache with the LDS table
    uint32_t ub_words = 0, ub_seed = 0;  // the compact UDP bind table (rx_common.h; 0 words: not built)
    bool ub_scattered = false;  // the local binds' port-table words span more lines than the compact table
    uint32_t ub_occ_dyn = ~0u, ub_occ_blocks = 0;  // small-kernel occupancy cache with the table in LDS
    uint32_t nflows = 0;
    // host pipeline state (lazily allocated)
    Stage stages[kPipeStreams];
    uint64_t* d_flow_counts = nullptr;
    uint32_t d_flow_cap = 0;
    uint64_t* d_verdict_counts = nullptr;
    StreamSlot slots[kMaxStreamSlots];
    uint64_t clock = 0;
    bool saturated = false;  // a slot has been taken over: slot events are recorded after each launch
    Tuning tune;
    uint32_t cu_count = 0;
    uint32_t occ_dyn = ~0u;   // occupancy cache: dynamic LDS bytes -> resident blocks per CU
    uint32_t occ_blocks = 0;
    uint32_t occ_family = ~0u;
    unsigned long long* d_path_stats = nullptr;  // dk_diag path counters (nullptr = off)
};

namespace {

struct DeviceGuard {  // set cfg.device for the duration of a call, restore afterwards
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

uint32_t next_pow2(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

int upload_table(dk_rx_ctx* c, const std::vector<uint32_t>& slots, uint32_t mask) {
    uint32_t* d = nullptr;
    if (hipMalloc(&d, slots.size() * sizeof(uint32_t)) != hipSuccess) return ENOMEM;
    if (hipMemcpy(d, slots.data(), slots.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(d);
        return EIO;
    }
    // Launches still in flight may read the old table (any stream, including ones that take no scratch slot): this
    // relies on hipFree synchronizing the device before it releases memory (HIP runtime semantics).
    if (c->table) (void)hipFree(c->table);
    c->table = d;
    c->table_mask = mask;
    c->lt_n = c->lt_b = c->lt_words = 0;
    c->lt_occ_family = ~0u;
    c->ub_words = 0;
    c->ub_scattered = false;
    c->ub_occ_dyn = ~0u;
    return 0;
}

void free_slot(StreamSlot& s) {  // the caller has flushed and waited for the slot's launches
    if (s.cs.rows) (void)hipFree(s.cs.rows);
    if (s.cs.defer) (void)hipFree(s.cs.defer);
    if (s.cs.tail) (void)hipFree(s.cs.tail);
    if (s.last) (void)hipEventDestroy(s.last);
    s = StreamSlot{};
}

// Add the slot's pending counter rows (a deferred launch's) to their counters: dk_flow_reduce_kernel on the slot's
// stream, after that launch.
int flush_pending(StreamSlot& s) {
    if (!s.used || !s.cs.pending) return 0;
    s.cs.pending = false;
    s.recorded = false;  // the slot's event no longer follows its last launch
    return dk_launch_reduce(s.cs.pend, s.stream) ? EIO : 0;
}

// Wait (host side) for every launch that used the slot: its recorded event, else its stream; if neither can be waited
// for, the whole device.
void wait_slot(StreamSlot& s) {
    if (!s.used) return;
    if (s.recorded ? hipEventSynchronize(s.last) == hipSuccess : hipStreamSynchronize(s.stream) == hipSuccess) return;
    (void)hipGetLastError();
    (void)hipDeviceSynchronize();
}

// The slot of `stream`. Past kMaxStreamSlots streams the least recently used slot is taken over: the new stream waits
// for an event that completes after every launch that used the slot. From the first takeover on, the context records
// each slot's event right after its launches (`saturated`), so a later takeover waits on an event recorded while its
// stream was in use; before that (<= 8 streams: the common case) no launch pays for an event record (~3 us).
#ifndef DK_SLOT_EVENTS
#define DK_SLOT_EVENTS 0  // 1: record the slot's event after every launch (measured: costs the launch gap)
#endif
int acquire_slot(dk_rx_ctx* c, hipStream_t stream, StreamSlot** out) {
    StreamSlot* pick = nullptr;
    for (StreamSlot& s : c->slots)
        if (s.used && s.stream == stream) pick = &s;
    if (!pick)
        for (StreamSlot& s : c->slots)
            if (!s.used) {
                if (!s.last && hipEventCreateWithFlags(&s.last, hipEventDisableTiming) != hipSuccess) {
                    s.last = nullptr;
                    return EIO;
                }
                s.stream = stream;
                s.used = true;
                s.recorded = false;
                pick = &s;
                break;
            }
    if (!pick) {  // every slot belongs to another stream: take over the least recently used one, behind its work
        pick = &c->slots[0];
        for (StreamSlot& s : c->slots)
            if (s.stamp < pick->stamp) pick = &s;
        c->saturated = true;
        if (flush_pending(*pick)) return EIO;  // its deferred rows reach their counters on the old stream first
        // Always record anew: flush_pending may just have queued a reduce launch on the old stream, after any event
        // recorded earlier.
        const bool ordered = hipEventRecord(pick->last, pick->stream) == hipSuccess;
        if (ordered) {
            if (hipStreamWaitEvent(stream, pick->last, 0) != hipSuccess) return EIO;
        } else {  // the old stream cannot be recorded on: wait for its work on the host instead
            (void)hipGetLastError();
            if (hipDeviceSynchronize() != hipSuccess) return EIO;
        }
        pick->stream = stream;
        pick->recorded = false;
    }
    pick->stamp = ++c->clock;
    *out = pick;
    return 0;
}

// Rows for `grid` workgroups (two halves) and `ndefer` deferral masks. Growing flushes the slot's pending rows and
// waits for its launches before freeing.
int ensure_counts(StreamSlot& s, uint32_t grid, uint32_t row_stride, size_t ndefer) {
    CountScratch& cs = s.cs;
    const size_t words = (size_t)grid * row_stride;
    if (cs.rows_words >= words && cs.ndefer >= ndefer) return 0;
    if (flush_pending(s)) return EIO;
    if (hipStreamSynchronize(s.stream) != hipSuccess) return EIO;  // launches still using the old buffers
    if (cs.rows_words < words) {
        if (cs.rows) (void)hipFree(cs.rows);
        cs.rows = nullptr;
        cs.rows_words = 0;
        if (hipMalloc(&cs.rows, 2 * words * sizeof(uint32_t)) != hipSuccess) return ENOMEM;
        cs.rows_words = words;
    }
    if (cs.ndefer < ndefer) {
        if (cs.defer) (void)hipFree(cs.defer);
        cs.defer = nullptr;
        cs.ndefer = 0;
        if (hipMalloc(&cs.defer, ndefer * sizeof(uint64_t)) != hipSuccess) return ENOMEM;
        cs.ndefer = ndefer;
    }
    return 0;
}

// The slot's dynamic-tail counters, allocated (and zeroed) on first use; they never grow.
int ensure_tail(StreamSlot& s) {
    if (s.cs.tail) return 0;
    if (hipMalloc(&s.cs.tail, 2 * dk::kTailSetWords * sizeof(uint32_t)) != hipSuccess) return ENOMEM;
    if (hipMemset(s.cs.tail, 0, 2 * dk::kTailSetWords * sizeof(uint32_t)) != hipSuccess) return EIO;  // synchronous
    s.cs.tail_set = 0;
    return 0;
}

// Choose the flow-count mode and the persistent grid, then launch on `stream` with that stream's counter scratch.
// size_hint = bytes of blob the batch covers (the family and grid follow the mean bytes per frame).

int launch_batch(dk_rx_ctx* c, dk::RxParams& p, uint64_t size_hint, hipStream_t stream, bool defer) {
    if (p.n == 0) return 0;
    const Tuning& T = c->tune;
    const uint32_t ntiles = (p.n + 255) / 256;
    p.flow_mode = dk::kFlowNone;
    p.flow_words = 0;
    p.row_words = 0;
    p.row_stride = 0;
    p.flow_scratch = nullptr;
    p.defer = nullptr;
    uint32_t dyn = 0;
    if (p.res.flow_counts && c->nflows) {
        const uint32_t words = (c->nflows + 1) / 2;
        if (words <= dk::kMaxLdsFlowWords) {
            p.flow_mode = dk::kFlowLds;
            p.flow_words = words;
            dyn = words * 4;
        } else {
            p.flow_mode = dk::kFlowGlobal;
        }
    }
    // Kernel instantiation, schedule and resident workgroups per CU (measured, DESIGN.md §8 "Tuning log"):
    //  - >= 1,280 bytes of blob per frame (the frames a stream wave streams with 6 loads per lane): the split kernel
    //    (stream waves + finish waves, one 512-thread workgroup per CU). Below, the staged kernel's 12 waves per CU
    //    keep more medium frames in flight (round 4, C1's 1078-byte frames: staged 27.9 vs split 30.2 us at 131,072
    //    frames, 177.9 vs 186.8 at 1M; 1500-byte frames: split ahead from 131,072 frames up, C5 -5.5 %);
    //  - >= 128 bytes: the result-staging kernel (stores leave in one burst per 6 chunks instead of between the frame
    //    reads; -11 % at C2 before the split kernel, -4 % IMIX);
    //  - <= 96 bytes: the small-frame kernel (issue/latency-bound, wants occupancy);
    //  - round-robin 256-frame tiles (sched 0) for every frame size.
    // Never more workgroups per CU than the occupancy admits (large socket tables take LDS).
    const uint64_t bytes_per_frame = size_hint / p.n;
    p.stage = bytes_per_frame >= 128 ? 1u : 0u;
    p.split = bytes_per_frame >= 1280 ? 1u : 0u;
    p.small = bytes_per_frame <= 96 ? 1u : 0u;
    if (T.stage >= 0) p.stage = T.stage ? 1u : 0u;
    if (T.split >= 0) p.split = T.split ? 1u : 0u;
    if (T.small >= 0) p.small = T.small ? 1u : 0u;
    if (p.small) p.split = p.stage = 0;
    p.sched = T.sched >= 0 ? (uint32_t)std::min(T.sched, 1) : 0u;
    const uint32_t family = p.small ? dk::kFamilySmall
                            : p.split ? dk::kFamilySplit
                            : p.stage ? dk::kFamilyStaged
                                      : dk::kFamilyUnstaged;
    if (c->occ_dyn != dyn || c->occ_family != family) {
        c->occ_blocks = (uint32_t)std::max(dk_rx_resident_blocks(dyn, family), 1);
        c->occ_dyn = dyn;
        c->occ_family = family;
    }
    const uint32_t fam_cap = p.small ? 8u : p.split ? 1u : p.stage ? 3u : 4u;
    uint32_t per_cu = std::min<uint32_t>(c->occ_blocks, fam_cap);
    // The LDS Active table (not the small-frame kernel: its five workgroups per CU have no LDS to spare, and its
    // batches are UDP-bound) when it costs no occupancy.
    if (c->lt_words && !p.small && T.lds_table != 0) {
        const uint32_t off = (dyn / 4 + 3) & ~3u;
        const uint32_t dyn2 = (off + c->lt_words) * 4;
        if (c->lt_occ_dyn != dyn2 || c->lt_occ_family != family) {
            c->lt_occ_blocks = (uint32_t)std::max(dk_rx_resident_blocks(dyn2, family), 0);
            c->lt_occ_dyn = dyn2;
            c->lt_occ_family = family;
        }
        if (std::min(c->lt_occ_blocks, fam_cap) >= per_cu) {
            p.lt_words = c->lt_words;
            p.lt_off = off;
            dyn = dyn2;
        }
    }
    // Local UDP binds (rx_common.h): the small-frame kernel's instantiation with the compact bind table in LDS when the
    // binds' port-table words are scattered and the table costs no occupancy; else the port table.
    if (c->ub_words && p.small && (T.udp_table > 0 || (T.udp_table < 0 && c->ub_scattered))) {
        const uint32_t off = (dyn / 4 + 3) & ~3u;
        const uint32_t dyn2 = (off + c->ub_words) * 4;
        if (c->ub_occ_dyn != dyn2) {
            c->ub_occ_blocks = (uint32_t)std::max(dk_rx_resident_blocks(dyn2, dk::kFamilySmallUb), 0);
            c->ub_occ_dyn = dyn2;
        }
        if (std::min(c->ub_occ_blocks, fam_cap) >= per_cu) {
            p.ub = c->table + (size_t)(c->table_mask + 1) * 4 + dk::kPortTabWords + c->lt_words;
            p.ub_off = off;
            dyn = dyn2;
        }
    }
    if (T.grid_per_cu > 0) per_cu = (uint32_t)T.grid_per_cu;
    // workgroups of the small-frame kernel take (waves / 4) 256-frame tiles per round
    const uint32_t small_waves = p.small ? dk_rx_small_block_waves(p.ub != nullptr) : 0u;
    const uint32_t tiles_per_wg = p.small ? std::max(small_waves / 4u, 1u) : 1u;
    uint32_t grid = std::min((ntiles + tiles_per_wg - 1) / tiles_per_wg, per_cu * c->cu_count);
    if (T.grid > 0) grid = std::min(ntiles, (uint32_t)T.grid);
    if (p.flow_mode == dk::kFlowLds)
        grid = std::max(grid, (ntiles + dk::kMaxTilesPerBlockLds - 1) / dk::kMaxTilesPerBlockLds);
    p.small_kmin = p.small ? ((p.n + 63) / 64) / (grid * small_waves) : 0u;
    // The staged kernel's dynamic tail (rx_common.h): with `per` whole round-robin rounds of chunks per wave, the
    // first per + 1 - d stay round-robin and the rest (d - 1 rounds + the partial one) are grabbed from per-XCD
    // counters; at least 2 round-robin rounds (the first grab is issued during round ks - 2).
    p.tail_ks = 0;
    p.tail_pools = 1;
    p.tail_ctr = p.tail_next = nullptr;
    const int32_t tail_d = T.tail >= 0 ? T.tail : 2;
    if (family == dk::kFamilyStaged && p.sched == 0 && tail_d > 0) {
        const uint32_t nwaves = grid * dk::kStagedWaves, nchunk = (p.n + 63) / 64;
        const uint32_t per = nchunk / nwaves;
        if (per + 1 >= (uint32_t)tail_d + 2) p.tail_ks = per + 1 - (uint32_t)tail_d;
        p.tail_pools = grid % 8 == 0 ? 8u : grid % 4 == 0 ? 4u : grid % 2 == 0 ? 2u : 1u;
    }
    // Per-workgroup histogram rows (flow pairs, then verdicts; dk_flow_reduce_kernel adds them up, or the next launch
    // on the stream when this one defers them) and the small-frame kernel's deferral masks: a launch that needs either,
    // or that has a previous launch's rows to combine, uses the stream's scratch slot.
    StreamSlot* slot = nullptr;
    int rc = 0;
    bool has_pending = false;
    for (StreamSlot& s : c->slots)
        if (s.used && s.stream == stream && s.cs.pending) has_pending = true;
    p.row_words = p.flow_words + (p.res.verdict_counts ? dk::kVerdictWords : 0u);
    // per (wave, chunk): at most ceil(n / 64) + 2 chunks per wave of the grid (sched 1's partial chunks)
    const size_t ndefer = p.small ? ((size_t)p.n + 63) / 64 + 2ull * grid * small_waves : 0;
    if (p.row_words || ndefer || has_pending || p.tail_ks) {
        if ((rc = acquire_slot(c, stream, &slot))) return rc;
        if (p.tail_ks) {
            if ((rc = ensure_tail(*slot))) return rc;
            p.tail_ctr = slot->cs.tail + (size_t)slot->cs.tail_set * dk::kTailSetWords;
            p.tail_next = slot->cs.tail + (size_t)(slot->cs.tail_set ^ 1u) * dk::kTailSetWords;
        }
        if (p.row_words)
            p.row_stride = (p.row_words + dk::kRowAlignWords - 1) / dk::kRowAlignWords * dk::kRowAlignWords;
        if ((rc = ensure_counts(*slot, grid, p.row_stride, ndefer))) return rc;
        if (p.row_words) p.flow_scratch = slot->cs.rows + (size_t)slot->cs.half * slot->cs.rows_words;
        p.defer = slot->cs.defer;
    }
    CountScratch* cs = slot ? &slot->cs : nullptr;
    p.comb = dk::RowCombine{};
    if (cs && cs->pending) {  // the previous deferred launch's rows (in the other half) are added inside this launch
        p.comb = cs->pend;
        p.comb.rpb = p.comb.row_words > 16 * dk::kCombCols ? 4 * dk::kCombRows : dk::kCombRows;
        p.comb.ncolblk = (p.comb.row_words + dk::kCombCols - 1) / dk::kCombCols;
        p.comb.nblk = p.comb.ncolblk * ((p.comb.nrows + p.comb.rpb - 1) / p.comb.rpb);
    }
    p.defer_rows = defer && p.row_words ? 1u : 0u;
    if (T.debug > 0)
        fprintf(stderr, "dk_rx: n=%u tiles=%u grid=%u occ=%u cus=%u flow_mode=%u words=%u sched=%u stage=%u split=%u "
                        "small=%u lds_table=%u defer=%u combine=%u tail_ks=%u udp_table=%u\n",
                p.n, ntiles, grid, c->occ_blocks, c->cu_count, p.flow_mode, p.flow_words, p.sched, p.stage, p.split,
                p.small, p.lt_words ? p.lt_n : 0u, p.defer_rows, p.comb.nblk, p.tail_ks,
                p.ub ? 1u : 0u);
    rc = dk_launch_rx(p, grid, stream);
    if (rc == 0 && cs && p.tail_ks) cs->tail_set ^= 1u;  // this launch zeroed the other set for the next one
    if (rc == 0 && cs) {
        if (p.comb.rows) cs->pending = false;
        if (p.row_words) {
            if (p.defer_rows) {
                cs->pend = dk::RowCombine{};
                cs->pend.rows = p.flow_scratch;
                cs->pend.nrows = grid;
                cs->pend.row_words = p.row_words;
                cs->pend.row_stride = p.row_stride;
                cs->pend.flow_words = p.flow_words;
                cs->pend.nflows = p.nflows;
                cs->pend.counts = p.flow_mode == dk::kFlowLds ? p.res.flow_counts : nullptr;
                cs->pend.verdicts = p.res.verdict_counts;
                cs->pending = true;
            }
            cs->half ^= 1u;
        }
    }
    if (rc == 0 && slot && (DK_SLOT_EVENTS || c->saturated)) {
        if (hipEventRecord(slot->last, stream) != hipSuccess) return EIO;
        slot->recorded = true;
    }
    return rc;
}

void free_stage(Stage& s) {
    if (s.opts) (void)hipFree(s.opts);
    if (s.frames) (void)hipFree(s.frames);
    if (s.desc_off) (void)hipFree(s.desc_off);
    if (s.desc_len) (void)hipFree(s.desc_len);
    if (s.res) (void)hipFree(s.res);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    s = Stage{};
}

int ensure_stage(Stage& s, uint32_t cap, uint64_t bytes, bool opts) {
    if (!s.stream && hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess) return EIO;
    if (opts && s.opts_cap < cap) {
        if (s.opts) (void)hipFree(s.opts);
        s.opts = nullptr;
        s.opts_cap = 0;
        if (hipMalloc(&s.opts, (size_t)cap * sizeof(dk_tcp_opts)) != hipSuccess) return ENOMEM;
        s.opts_cap = cap;
    }
    if (s.cap < cap) {
        if (s.desc_off) (void)hipFree(s.desc_off);
        if (s.desc_len) (void)hipFree(s.desc_len);
        if (s.res) (void)hipFree(s.res);
        s.desc_off = nullptr; s.desc_len = nullptr; s.res = nullptr; s.cap = 0;
        if (hipMalloc(&s.desc_off, cap * sizeof(uint32_t)) != hipSuccess) return ENOMEM;
        if (hipMalloc(&s.desc_len, cap * sizeof(uint16_t)) != hipSuccess) return ENOMEM;
        if (hipMalloc(&s.res, (size_t)cap * 9 * sizeof(uint32_t)) != hipSuccess) return ENOMEM;
        s.cap = cap;
    }
    if (s.frames_cap < bytes) {
        if (s.frames) (void)hipFree(s.frames);
        s.frames = nullptr; s.frames_cap = 0;
        if (hipMalloc(&s.frames, bytes) != hipSuccess) return ENOMEM;
        s.frames_cap = bytes;
    }
    return 0;
}

// TX tuning overrides (-1 = host rule), set only by dk_diag_tx_set_tuning (never from the environment).
struct TxTuning {
    std::atomic<int32_t> split{-1}, sched{-1}, grid_per_cu{-1};
};
TxTuning& tx_tuning() {
    static TxTuning t;
    return t;
}

dk::RxParams base_params(const dk_rx_ctx* c) {
    dk::RxParams p{};
    p.path_stats = c->d_path_stats;
    p.local_ip = c->cfg.local_ipv4;
    p.tcp_offload = c->cfg.tcp_rx_checksum_offload ? 1u : 0u;
    p.udp_offload = c->cfg.udp_rx_checksum_offload ? 1u : 0u;
    p.table = c->table;
    p.table_mask = c->table_mask;
    p.port_tab = c->table + (size_t)(c->table_mask + 1) * 4;
    p.lt = p.port_tab + dk::kPortTabWords;
    p.lt_words = p.lt_off = 0;
    p.lt_n = c->lt_n;
    p.lt_b = c->lt_b;
    p.ub = nullptr;
    p.ub_off = 0;
    p.ub_words = c->ub_words;
    p.ub_mask = c->ub_words ? c->ub_words / 2 - 1 : 0u;
    p.ub_seed = c->ub_seed;
    p.nflows = c->nflows;
    return p;
}

}  // namespace

extern "C" {

uint32_t dk_rx_abi_version(void) { return DK_RX_ABI_VERSION; }

#ifndef DK_BUILD_ID
#define DK_BUILD_ID "unversioned"
#endif
// The marker prefix lets __graft_entry__ read the id from the file without loading the library.
static const char kBuildIdMarker[] = "DK_BUILD_ID=" DK_BUILD_ID;
const char* dk_rx_build_id(void) { return kBuildIdMarker + 12; }

int dk_rx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int dk_rx_ctx_create(const dk_rx_cfg* cfg, dk_rx_ctx** out) {
    if (!cfg || !out) return EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || cfg->device < 0 || cfg->device >= ndev) return EINVAL;
    DeviceGuard g(cfg->device);
    dk_rx_ctx* c = new dk_rx_ctx();
    c->cfg = *cfg;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cfg->device) != hipSuccess || cus <= 0)
        cus = 256;
    c->cu_count = (uint32_t)cus;
    // c->tune: the built-in rule (every override -1) until dk_diag_rx_set_tuning
    // Empty socket table: every probe misses.
    std::vector<uint32_t> slots(dk::kMinTableSlots * 4 + dk::kPortTabWords, 0u);
    std::fill(slots.begin() + dk::kMinTableSlots * 4, slots.end(), DK_FLOW_NONE);
    int rc = upload_table(c, slots, dk::kMinTableSlots - 1);
    if (rc) {
        delete c;
        return rc;
    }
    *out = c;
    return 0;
}

void dk_rx_ctx_destroy(dk_rx_ctx* c) {
    if (!c) return;
    DeviceGuard g(c->cfg.device);
    // Deferred counter rows reach their counters first; then wait for the launches that use slot scratch (each slot's
    // stream, or its last recorded event) and the pipeline's own streams, and free the scratch. A launch that took no
    // slot (no counters, not the small-frame kernel) may still be reading the socket table: freeing the table relies on
    // hipFree synchronizing the device first (HIP runtime semantics), as upload_table does.
    for (StreamSlot& s : c->slots) (void)flush_pending(s);
    for (StreamSlot& s : c->slots) wait_slot(s);
    for (Stage& s : c->stages)
        if (s.stream) (void)hipStreamSynchronize(s.stream);
    for (StreamSlot& s : c->slots) free_slot(s);
    if (c->table) (void)hipFree(c->table);
    for (Stage& s : c->stages) free_stage(s);
    if (c->d_flow_counts) (void)hipFree(c->d_flow_counts);
    if (c->d_verdict_counts) (void)hipFree(c->d_verdict_counts);
    if (c->d_path_stats) (void)hipFree(c->d_path_stats);
    delete c;
}

int dk_rx_flow_table_set(dk_rx_ctx* c, const dk_flow* flows, uint32_t n) {
    if (!c || (n && !flows) || n > dk::kMaxFlows) return EINVAL;
    uint32_t nact = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t k = flows[i].kind;
        if (k != DK_FLOW_TCP_ACTIVE && k != DK_FLOW_TCP_PASSIVE && k != DK_FLOW_UDP) return EINVAL;
        nact += k == DK_FLOW_TCP_ACTIVE;
    }
    // Active connections: open addressing at load factor <= 1/8 (rx_common.h), up to 2^26 slots (1 GiB; 32-bit slot
    // offsets), never above 1/2.
    const uint64_t want = std::min<uint64_t>(8ull * std::max(nact, 1u), 1ull << 26);
    const uint32_t cap = std::max({dk::kMinTableSlots, next_pow2((uint32_t)want), next_pow2(2 * std::max(nact, 1u))});
    const uint32_t mask = cap - 1;
    std::vector<uint32_t> slots((size_t)cap * 4 + dk::kPortTabWords, 0u);
    uint32_t* ports_tab = slots.data() + (size_t)cap * 4;
    std::fill(ports_tab, ports_tab + dk::kPortTabWords, DK_FLOW_NONE);
    const uint32_t cfg_ip = c->cfg.local_ipv4;
    for (uint32_t i = 0; i < n; i++) {  // in table order: HashMap::insert, the last duplicate wins
        const dk_flow& f = flows[i];
        if (f.kind == DK_FLOW_UDP) {
            // SocketAddrV4 keys: udp/peer.rs looks up (local_ipv4_addr, port), then (0.0.0.0, port) (udp/peer.rs:147-165);
            // a bind to any other address is never looked up
            if (f.local_ip == cfg_ip) ports_tab[dk::kPortUdpLocal + f.local_port] = i;
            if (f.local_ip == 0) ports_tab[dk::kPortUdpAny + f.local_port] = i;
            continue;
        }
        if (f.kind == DK_FLOW_TCP_PASSIVE) {  // SocketId::Passive(local_ipv4_addr, port) (tcp/peer.rs:246-251)
            if (f.local_ip == cfg_ip) ports_tab[dk::kPortTcpPassive + f.local_port] = i;
            continue;
        }
        const uint32_t lip = f.local_ip, rip = f.remote_ip, ports = f.local_port | (uint32_t)f.remote_port << 16;
        uint32_t h = dk::flow_hash(f.kind, lip, rip, ports) & mask;
        for (;;) {
            uint32_t* s = &slots[(size_t)h * 4];
            if (s[0] == 0 || (s[1] == lip && s[2] == rip && s[3] == ports)) {
                s[0] = (f.kind << 24) | i;
                s[1] = lip;
                s[2] = rip;
                s[3] = ports;
                break;
            }
            h = (h + 1) & mask;
        }
    }
    uint32_t lt_n = 0, lt_b = 0, lt_w = 0;
    {
        std::vector<uint32_t> lt;
        if (dk::build_lds_table(slots, cap, cfg_ip, lt, lt_n, lt_b)) {
            lt_w = (uint32_t)lt.size();
            slots.insert(slots.end(), lt.begin(), lt.end());
        }
    }
    uint32_t ub_mask = 0, ub_seed = 0, ub_lines = 0, ub_w = 0;
    {
        std::vector<uint32_t> ub;
        if (dk::build_udp_table(slots.data() + (size_t)cap * 4 + dk::kPortUdpLocal, ub, ub_mask, ub_seed, ub_lines)) {
            ub_w = (uint32_t)ub.size();
            slots.insert(slots.end(), ub.begin(), ub.end());
        }
    }
    DeviceGuard g(c->cfg.device);
    int rc = upload_table(c, slots, mask);
    if (rc == 0) {
        c->nflows = n;
        c->lt_n = lt_n;
        c->lt_b = lt_b;
        c->lt_words = lt_w;
        c->ub_words = ub_w;
        c->ub_seed = ub_seed;
        c->ub_scattered = ub_w && ub_lines > ub_w / 32;  // 32 words per 128-byte line
        c->ub_occ_dyn = ~0u;
    }
    return rc;
}

uint32_t dk_rx_flow_table_size(const dk_rx_ctx* c) { return c ? c->nflows : 0; }

int dk_rx_process(dk_rx_ctx* c, const dk_rx_batch* b, const dk_rx_results* r, void* stream) {
    if (!c || !b || !r) return EINVAL;
    if (b->n && (!b->frames || !b->off || !b->len)) return EINVAL;
    if (b->n && (!r->meta || !r->src_ip || !r->ports || !r->payload || !r->flow_id)) return EINVAL;
    if (b->frames_bytes > DK_RX_MAX_BLOB) return EINVAL;
    DeviceGuard g(c->cfg.device);
    dk::RxParams p = base_params(c);
    p.frames = b->frames;
    p.frames_bytes = b->frames_bytes;
    p.off = b->off;
    p.len = b->len;
    p.n = b->n;
    p.aligned16 = (b->flags & DK_RX_BATCH_ALIGNED16) ? 1u : 0u;
    p.res = *r;
    return launch_batch(c, p, b->frames_bytes, (hipStream_t)stream, (b->flags & DK_RX_BATCH_DEFER_COUNTS) != 0);
}

int dk_rx_counts_flush(dk_rx_ctx* c, void* stream) {
    if (!c) return EINVAL;
    DeviceGuard g(c->cfg.device);
    for (StreamSlot& s : c->slots)
        if (s.used && s.stream == (hipStream_t)stream) return flush_pending(s);
    return 0;
}

int dk_rx_stream_forget(dk_rx_ctx* c, void* stream) {
    if (!c) return EINVAL;
    DeviceGuard g(c->cfg.device);
    for (StreamSlot& s : c->slots) {
        if (!s.used || s.stream != (hipStream_t)stream) continue;
        if (flush_pending(s)) return EIO;
        const bool ok = s.recorded ? hipEventSynchronize(s.last) == hipSuccess
                                   : hipStreamSynchronize(s.stream) == hipSuccess;
        if (!ok) return EIO;
        s.used = false;  // scratch buffers and the event stay for the slot's next stream
        s.recorded = false;
        s.stream = nullptr;
        s.stamp = 0;
    }
    return 0;
}

namespace {
// The device alias of a page-locked, GPU-mapped host range (hipHostMalloc, hipHostRegister), or nullptr when any part
// of [p, p + bytes) is not (pageable memory: the caller stages through copies instead). Both ends are checked and
// must map to one contiguous device range.
const uint8_t* mapped_alias(const uint8_t* p, uint64_t bytes) {
    if (!p || !bytes) return nullptr;
    hipPointerAttribute_t a0{}, a1{};
    const uint8_t* q = p + bytes - 1;
    if (hipPointerGetAttributes(&a0, p) != hipSuccess || hipPointerGetAttributes(&a1, q) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (a0.type != hipMemoryTypeHost || a1.type != hipMemoryTypeHost) return nullptr;
    if (!a0.devicePointer || !a1.devicePointer || !a0.hostPointer || !a1.hostPointer) return nullptr;
    const uint8_t* d0 = static_cast<const uint8_t*>(a0.devicePointer) + (p - static_cast<const uint8_t*>(a0.hostPointer));
    const uint8_t* d1 = static_cast<const uint8_t*>(a1.devicePointer) + (q - static_cast<const uint8_t*>(a1.hostPointer));
    return d1 - d0 == (ptrdiff_t)(bytes - 1) ? d0 : nullptr;
}
}  // namespace

namespace {
int process_host(dk_rx_ctx* c, const dk_rx_batch* b, const dk_rx_results* r, uint32_t chunk_frames, bool allow_zc);
}  // namespace

int dk_rx_process_host(dk_rx_ctx* c, const dk_rx_batch* b, const dk_rx_results* r, uint32_t chunk_frames) {
    if (!c) return EINVAL;
    return process_host(c, b, r, chunk_frames, c->tune.host_zc != 0);
}

}  // extern "C"

// A TPACKET_V3 ring's frames go through staged copies by default: the copy engine moves each chunk's byte range
// (headers included) to HBM, which is blind to the ring's layout and to the NUMA node of its pages, where the kernel
// reading the ring in place over PCIe loses to both (tools/ring_numa.py, session r6s3: staged 46.2-46.4 GB/s whatever
// the placement; in place 45.0 from the GPU's node, 42.4 from the other). host_zc = 1 (dk_diag) forces the
// in-place reads for A/B.
int dk_rx_process_ring_host(dk_rx_ctx* c, const dk_rx_batch* b, const dk_rx_results* r) {
    if (!c) return EINVAL;
    return process_host(c, b, r, 0, c->tune.host_zc > 0);
}

namespace {
int process_host(dk_rx_ctx* c, const dk_rx_batch* b, const dk_rx_results* r, uint32_t chunk_frames, bool allow_zc) {
    if (!c || !b || !r) return EINVAL;
    if (b->n && (!b->frames || !b->off || !b->len)) return EINVAL;
    if (b->n && (!r->meta || !r->src_ip || !r->ports || !r->payload || !r->flow_id)) return EINVAL;
    if (b->frames_bytes > DK_RX_MAX_BLOB) return EINVAL;
    if (b->n == 0) return 0;
    DeviceGuard g(c->cfg.device);
    const uint32_t chunk = chunk_frames ? chunk_frames : kDefaultChunkFrames;

    // Zero-copy: frames in mapped page-locked memory are read by the kernel in place over PCIe (no staging copy):
    // one launch over the whole batch unless the caller asks for chunks (descriptors H2D and results D2H around it).
    // For packed frames both forms run at the PCIe rate (C5 shard 51-53 GB/s); for frames scattered in
    // mbuf slots the staged copies would also move the unused bytes between them. Chunked zero-copy launches
    // measured slower (44 GB/s).
    const uint8_t* zc = allow_zc ? mapped_alias(b->frames, b->frames_bytes) : nullptr;
    const uint32_t chunk_n = zc && !chunk_frames ? b->n : chunk;
    // Chunk boundaries: consecutive frame ranges whose covering byte range stays under kMaxChunkBytes (staged).
    std::vector<dk::HostChunk> chunks;
    const uint64_t max_bytes = dk::plan_host_chunks(b->off, b->len, b->n, b->frames_bytes, chunk_n, zc != nullptr,
                                                    kMaxChunkBytes, chunks);
    uint32_t cap = 0;
    for (auto& ch : chunks) cap = std::max(cap, ch.e - ch.a);
    const size_t nstages = std::min<size_t>(chunks.size(), kPipeStreams);  // stages this call uses
    for (size_t k = 0; k < nstages; k++) {
        int rc = ensure_stage(c->stages[k], cap, zc ? 16 : std::max<uint64_t>(max_bytes, 16), r->tcp_opts != nullptr);
        if (rc) return rc;
    }
    const uint32_t nfl = std::max(c->nflows, 1u);
    if (r->flow_counts && c->d_flow_cap < nfl) {
        if (c->d_flow_counts) (void)hipFree(c->d_flow_counts);
        c->d_flow_counts = nullptr;
        c->d_flow_cap = 0;
        if (hipMalloc(&c->d_flow_counts, nfl * sizeof(uint64_t)) != hipSuccess) return ENOMEM;
        c->d_flow_cap = nfl;
    }
    if (r->verdict_counts && !c->d_verdict_counts &&
        hipMalloc(&c->d_verdict_counts, DK_V_COUNT * sizeof(uint64_t)) != hipSuccess)
        return ENOMEM;
    hipStream_t s0 = c->stages[0].stream;
    if (r->flow_counts && hipMemsetAsync(c->d_flow_counts, 0, nfl * sizeof(uint64_t), s0) != hipSuccess) return EIO;
    if (r->verdict_counts && hipMemsetAsync(c->d_verdict_counts, 0, DK_V_COUNT * sizeof(uint64_t), s0) != hipSuccess)
        return EIO;
    // Counter memsets on stage 0 must land before any stage's kernel: make the other stages wait on stage 0.
    hipEvent_t ev0;
    if (hipEventCreateWithFlags(&ev0, hipEventDisableTiming) != hipSuccess) return EIO;
    (void)hipEventRecord(ev0, s0);
    for (int k = 1; k < kPipeStreams; k++)
        if (c->stages[k].stream) (void)hipStreamWaitEvent(c->stages[k].stream, ev0, 0);

    int rc = 0;
    for (size_t k = 0; k < chunks.size() && rc == 0; k++) {
        const dk::HostChunk& ch = chunks[k];
        Stage& st = c->stages[k % kPipeStreams];
        const uint32_t m = ch.e - ch.a;
        // The staged copy starts at a 16-aligned host offset; a virtual base keeps the descriptors unchanged.
        if ((!zc && hipMemcpyAsync(st.frames, b->frames + ch.lo, ch.hi - ch.lo, hipMemcpyHostToDevice, st.stream) !=
                        hipSuccess) ||
            hipMemcpyAsync(st.desc_off, b->off + ch.a, m * sizeof(uint32_t), hipMemcpyHostToDevice, st.stream) != hipSuccess ||
            hipMemcpyAsync(st.desc_len, b->len + ch.a, m * sizeof(uint16_t), hipMemcpyHostToDevice, st.stream) != hipSuccess) {
            rc = EIO;
            break;
        }
        dk::RxParams p = base_params(c);
        p.frames = zc ? zc : st.frames - ch.lo;
        p.frames_bytes = zc ? b->frames_bytes : ch.hi;
        p.off = st.desc_off;
        p.len = st.desc_len;
        p.n = m;
        p.aligned16 = (b->flags & DK_RX_BATCH_ALIGNED16) ? 1u : 0u;  // the staging keeps every offset mod 16
        uint32_t* R = st.res;
        p.res.meta = R;
        p.res.src_ip = R + (size_t)st.cap;
        p.res.dst_ip = r->dst_ip ? R + 2 * (size_t)st.cap : nullptr;
        p.res.ports = R + 3 * (size_t)st.cap;
        p.res.payload = R + 4 * (size_t)st.cap;
        p.res.flow_id = R + 5 * (size_t)st.cap;
        p.res.tcp_seq = r->tcp_seq ? R + 6 * (size_t)st.cap : nullptr;
        p.res.tcp_ack = r->tcp_ack ? R + 7 * (size_t)st.cap : nullptr;
        p.res.tcp_win = r->tcp_win ? R + 8 * (size_t)st.cap : nullptr;
        p.res.tcp_opts = r->tcp_opts ? st.opts : nullptr;
        if (r->tcp_opts && hipMemsetAsync(st.opts, 0, (size_t)m * sizeof(dk_tcp_opts), st.stream) != hipSuccess) {
            rc = EIO;
            break;
        }
        p.res.flow_counts = r->flow_counts ? c->d_flow_counts : nullptr;
        p.res.verdict_counts = r->verdict_counts ? c->d_verdict_counts : nullptr;
        rc = launch_batch(c, p, ch.hi - ch.lo, st.stream, false);  // synchronous: counters current at return
        if (rc) break;
        uint32_t* outs[9] = {r->meta, r->src_ip, r->dst_ip, r->ports, r->payload, r->flow_id,
                             r->tcp_seq, r->tcp_ack, r->tcp_win};
        for (int a = 0; a < 9; a++) {
            if (!outs[a]) continue;
            if (hipMemcpyAsync(outs[a] + ch.a, R + a * (size_t)st.cap, m * sizeof(uint32_t), hipMemcpyDeviceToHost,
                               st.stream) != hipSuccess) {
                rc = EIO;
                break;
            }
        }
        if (rc == 0 && r->tcp_opts &&
            hipMemcpyAsync(r->tcp_opts + ch.a, st.opts, m * sizeof(dk_tcp_opts), hipMemcpyDeviceToHost, st.stream) !=
                hipSuccess)
            rc = EIO;
    }
    for (Stage& s : c->stages)
        if (s.stream && hipStreamSynchronize(s.stream) != hipSuccess) rc = rc ? rc : EIO;
    (void)hipEventDestroy(ev0);
    if (rc) return rc;
    if (r->flow_counts) {
        std::vector<uint64_t> tmp(nfl);
        if (hipMemcpy(tmp.data(), c->d_flow_counts, nfl * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
            return EIO;
        for (uint32_t k = 0; k < c->nflows; k++) r->flow_counts[k] += tmp[k];
    }
    if (r->verdict_counts) {
        uint64_t tmp[DK_V_COUNT];
        if (hipMemcpy(tmp, c->d_verdict_counts, sizeof(tmp), hipMemcpyDeviceToHost) != hipSuccess) return EIO;
        for (int k = 0; k < DK_V_COUNT; k++) r->verdict_counts[k] += tmp[k];
    }
    return 0;
}
}  // namespace

extern "C" {

#ifdef DK_DIAG_STAMPS
constexpr size_t kPathStatsWords = 4 + (1u << 21);  // + 16 stamps per wave
#else
constexpr size_t kPathStatsWords = 4;
#endif
int dk_diag_path_stats_enable(dk_rx_ctx* c, int on) {
    if (!c) return EINVAL;
    DeviceGuard g(c->cfg.device);
    if (!on) {
        if (c->d_path_stats) (void)hipFree(c->d_path_stats);
        c->d_path_stats = nullptr;
        return 0;
    }
    if (!c->d_path_stats && hipMalloc(&c->d_path_stats, kPathStatsWords * sizeof(unsigned long long)) != hipSuccess)
        return ENOMEM;
    return hipMemset(c->d_path_stats, 0, kPathStatsWords * sizeof(unsigned long long)) == hipSuccess ? 0 : EIO;
}

#ifdef DK_DIAG_STAMPS
// Diagnostic build only: the per-wave stamps the small-frame kernel writes after the path counters.
extern "C" int dk_diag_stamps_read(dk_rx_ctx* c, uint64_t* out, uint64_t n) {
    if (!c || !out || !c->d_path_stats || n > kPathStatsWords - 4) return EINVAL;
    DeviceGuard g(c->cfg.device);
    if (hipDeviceSynchronize() != hipSuccess) return EIO;
    return hipMemcpy(out, c->d_path_stats + 4, n * sizeof(uint64_t), hipMemcpyDeviceToHost) == hipSuccess ? 0 : EIO;
}
#endif

int dk_diag_path_stats_read(dk_rx_ctx* c, uint64_t out[4]) {
    if (!c || !out || !c->d_path_stats) return EINVAL;
    DeviceGuard g(c->cfg.device);
    if (hipDeviceSynchronize() != hipSuccess) return EIO;
    return hipMemcpy(out, c->d_path_stats, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost) == hipSuccess ? 0 : EIO;
}

int dk_diag_rx_set_tuning(dk_rx_ctx* c, const int32_t* knobs, uint32_t nknobs) {
    if (!c || (nknobs && !knobs)) return EINVAL;
    int32_t k[DK_DIAG_RX_KNOBS];
    for (uint32_t i = 0; i < DK_DIAG_RX_KNOBS; i++) k[i] = i < nknobs ? knobs[i] : -1;
    Tuning t;
    t.stage = k[0];
    t.split = k[1];
    t.small = k[2];
    t.sched = k[3];
    t.grid = k[4];
    t.grid_per_cu = k[5];
    t.debug = k[6] < 0 ? 0 : k[6];
    t.lds_table = k[7];
    t.tail = k[8];
    t.udp_table = k[9];
    t.host_zc = k[10];
    c->tune = t;
    c->occ_family = ~0u;
    c->lt_occ_family = ~0u;
    return 0;
}

int dk_diag_tx_set_tuning(int32_t split, int32_t sched, int32_t grid_per_cu) {
    TxTuning& t = tx_tuning();
    t.split = split;
    t.sched = sched;
    t.grid_per_cu = grid_per_cu;
    return 0;
}

namespace {
// dk_tx_checksum / dk_tx_checksum_fields: persistent grid on the current device, the receive kernel's schedule rule.
int tx_launch(uint8_t* frames, uint64_t frames_bytes, const uint32_t* off, const uint16_t* len, uint32_t n,
              uint32_t* fields, void* stream) {
    if (n && (!frames || !off || !len)) return EINVAL;
    if (frames_bytes > DK_RX_MAX_BLOB) return EINVAL;
    if (n == 0) return 0;
    static thread_local int dev_cached = -1;
    static thread_local uint32_t cus = 0, occ = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return ENODEV;
    if (dev != dev_cached) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
            return ENODEV;
        cus = (uint32_t)c;
        occ = (uint32_t)std::max(dk_tx_resident_blocks(), 1);
        dev_cached = dev;
    }
    // Large frames: the split kernel (stream waves + finish waves, one 512-thread workgroup per CU, sched 0).
    const bool big = frames_bytes / n >= 1024;
    dk::TxParams p{frames, frames_bytes, off, len, n, big ? 1u : 0u, big ? 1u : 0u, fields};
    const TxTuning& T = tx_tuning();
    if (T.split >= 0) p.split = T.split ? 1u : 0u;
    uint32_t per_cu = p.split ? 1u : std::min<uint32_t>(occ, p.sched ? 3u : 4u);
    if (T.sched >= 0) p.sched = (uint32_t)std::min<int32_t>(T.sched, 1);
    if (T.grid_per_cu > 0) per_cu = (uint32_t)T.grid_per_cu;
    const uint32_t grid = std::min((n + 255) / 256, per_cu * cus);
    return dk_launch_tx(p, grid, stream);
}
}  // namespace

int dk_tx_checksum(uint8_t* frames, uint64_t frames_bytes, const uint32_t* off, const uint16_t* len, uint32_t n,
                   void* stream) {
    return tx_launch(frames, frames_bytes, off, len, n, nullptr, stream);
}

int dk_tx_checksum_fields(const uint8_t* frames, uint64_t frames_bytes, const uint32_t* off, const uint16_t* len,
                          uint32_t n, uint32_t* fields, void* stream) {
    if (n && !fields) return EINVAL;
    // the kernels only read the frames in this form (TxParams::fields set)
    return tx_launch(const_cast<uint8_t*>(frames), frames_bytes, off, len, n, fields, stream);
}

const char* dk_rx_verdict_name(int v) {
    static const char* const names[DK_V_COUNT] = {
        "OK_TCP",         "OK_UDP",        "ARP",          "ICMP",           "IPV6",          "ETH_SHORT",
        "ETH_TYPE",       "IP_SHORT",      "IP_VERSION",   "IP_IHL_SMALL",   "IP_HDR_TRUNC",  "IP_TOTLEN_SMALL",
        "IP_TOTLEN_BIG",  "IP_EVIL",       "IP_MF",        "IP_FRAGOFF",     "IP_TTL",        "IP_PROTO",
        "IP_CSUM_FFFF",   "IP_CSUM",       "IP_DST",       "IP_SRC",         "TCP_SHORT",     "TCP_DOFF_TRUNC",
        "TCP_DOFF_SMALL", "TCP_CSUM",      "TCP_OPT",      "TCP_OPT_EIO",    "TCP_NOSOCK",    "UDP_SHORT",
        "UDP_LEN",        "UDP_CSUM",      "UDP_NOSOCK",   "BAD_DESC",       "ARP_SHORT",     "ARP_UNSUP",
        "ICMP_SHORT",     "ICMP_CSUM",     "ICMP_TYPE"};
    return (v >= 0 && v < DK_V_COUNT) ? names[v] : "UNKNOWN";
}

int dk_rx_verdict_errno(int v) {
    switch (v) {
        case DK_V_ETH_TYPE: case DK_V_IP_VERSION: case DK_V_IP_MF: case DK_V_IP_FRAGOFF: case DK_V_IP_PROTO:
        case DK_V_ARP_UNSUP:
            return 95;  // ENOTSUP
        case DK_V_TCP_OPT_EIO:
            return 5;   // EIO
        case DK_V_BAD_DESC:
            return 22;  // EINVAL
        case DK_V_ETH_SHORT: case DK_V_IP_SHORT: case DK_V_IP_IHL_SMALL: case DK_V_IP_HDR_TRUNC:
        case DK_V_IP_TOTLEN_SMALL: case DK_V_IP_TOTLEN_BIG: case DK_V_IP_EVIL: case DK_V_IP_TTL:
        case DK_V_IP_CSUM_FFFF: case DK_V_IP_CSUM: case DK_V_TCP_SHORT: case DK_V_TCP_DOFF_TRUNC:
        case DK_V_TCP_DOFF_SMALL: case DK_V_TCP_CSUM: case DK_V_TCP_OPT: case DK_V_UDP_SHORT: case DK_V_UDP_LEN:
        case DK_V_UDP_CSUM: case DK_V_ARP_SHORT: case DK_V_ICMP_SHORT: case DK_V_ICMP_CSUM: case DK_V_ICMP_TYPE:
            return 74;  // EBADMSG
        default:
            return 0;
    }
}

}  // extern "C"
