// rx_diag.h — diagnostic-build instrumentation of the receive kernels (rx_kernels.hip). Nothing here is on the
// product path: in the default build every macro below expands to nothing and kPathStatsOn is true.
//
// A -DDK_DIAG_STAMPS build (tools/variants.sh) records per-wave s_memtime / s_memrealtime stamps into the path-stats
// buffer (dk_diag.h: dk_diag_path_stats_enable, dk_diag_stamps_read), read back by tools/stamps.py (small-frame kernel)
// and tools/stamps_staged.py (staged kernel); that build gives up the per-path frame counters, whose buffer it reuses.
// Slot layout: 32 u64 per wave after the 4 path counters; wave = blockIdx.x * waves per workgroup + wave in group.
//   dk_rx_kernel:       0 entry, 1 after the start barrier, 2 + 3k / 3 + 3k / 4 + 3k chunk k (k < 3) before the
//                       stream / after the stream / after phase C, 11 after the loop, 14 after the combine, 15 exit,
//                       12 / 13 s_memrealtime at entry / exit
//   dk_rx_small_kernel: 0 entry, 11 after the barrier, 1 first window, 2 + 3k .. 4 + 3k chunk k (k < 3), 16 + 5k + j
//                       sub-phases j of phase C (k < 3), 14 after the combine, 15 exit, 12 / 13 realtime
//   both, totals over every chunk (DK_ACC_*): 20.. per-phase shader-clock totals, 26 the wave's chunk count
#pragma once

#ifdef DK_DIAG_STAMPS
namespace dk {
constexpr bool kPathStatsOn = false;  // the stamp build reuses the path-stats buffer
}
// stamp `t` into slot `slot` of the calling wave (wpg = waves per workgroup)
#define DK_DIAG_STAMP_AT(slot, t, wpg)                                                                             \
    do {                                                                                                            \
        const uint64_t t_ = (t);                                                                                    \
        if (P.path_stats && lane_id() == 0 && (slot) < 32)                                                         \
            P.path_stats[4 + 32 * (blockIdx.x * (wpg) + (threadIdx.x >> 6)) + (slot)] = t_;                         \
    } while (0)
// phase-C sub-phase j of a chunk whose stamp range starts at stamp_base (~0u: not stamped)
#define DK_SUB_STAMP(j)                                                                                             \
    do {                                                                                                            \
        if (stamp_base != ~0u) DK_DIAG_STAMP_AT(stamp_base + (j), __builtin_amdgcn_s_memtime(), blockDim.x >> 6);   \
    } while (0)
#else
namespace dk {
constexpr bool kPathStatsOn = true;
}
#define DK_DIAG_STAMP_AT(slot, t, wpg) do {} while (0)
#define DK_SUB_STAMP(j) do {} while (0)
#endif

// Section markers for the static per-block instruction budget (tools/isa_blocks.py on a -DDK_ISA_MARKS -S build): an
// assembly comment "; MARK_<name>" where a section starts. Nothing in the product build.
#ifdef DK_ISA_MARKS
#define DK_MARK(name) asm volatile("; MARK_" #name)
#else
#define DK_MARK(name) do {} while (0)
#endif

// Per-wave phase totals over ALL of a wave's chunks (stamps only cover chunks k < 3): DK_ACC_BEGIN() at a phase
// boundary, DK_ACC_SPLIT(j) adds the shader-clock ticks since the last boundary to total j (< 6); DK_ACC_WRITE
// stores the totals into slots 20..25 and the chunk count into slot 26. Nothing in the product build.
#ifdef DK_DIAG_STAMPS
#define DK_ACC_DECL uint64_t dk_acc_[6] = {0, 0, 0, 0, 0, 0}, dk_t_ = 0, dk_nch_ = 0
#define DK_ACC_BEGIN() (dk_t_ = __builtin_amdgcn_s_memtime())
#define DK_ACC_SPLIT(j)                                                                                             \
    do {                                                                                                            \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();                                                           \
        dk_acc_[j] += t_ - dk_t_;                                                                                   \
        dk_t_ = t_;                                                                                                 \
    } while (0)
#define DK_ACC_CHUNK() (dk_nch_++)
#define DK_ACC_WRITE(wpg)                                                                                           \
    do {                                                                                                            \
        for (int j_ = 0; j_ < 6; j_++) DK_DIAG_STAMP_AT(20 + j_, dk_acc_[j_], wpg);                                 \
        DK_DIAG_STAMP_AT(26, dk_nch_, wpg);                                                                         \
    } while (0)
#else
#define DK_ACC_DECL do {} while (0)
#define DK_ACC_BEGIN() do {} while (0)
#define DK_ACC_SPLIT(j) do {} while (0)
#define DK_ACC_CHUNK() do {} while (0)
#define DK_ACC_WRITE(wpg) do {} while (0)
#endif

// dk_rx_kernel / dk_rx_small_kernel shorthands: shader clock (per XCD) and the global 100 MHz clock
#define DK_STAMPW(slot) DK_DIAG_STAMP_AT(slot, __builtin_amdgcn_s_memtime(), kWaves)
#define DK_STAMPW_RT(slot) DK_DIAG_STAMP_AT(slot, __builtin_amdgcn_s_memrealtime(), kWaves)
#define DK_STAMP(slot) DK_DIAG_STAMP_AT(slot, __builtin_amdgcn_s_memtime(), kSmallWaves)
#define DK_STAMP_RT(slot) DK_DIAG_STAMP_AT(slot, __builtin_amdgcn_s_memrealtime(), kSmallWaves)
