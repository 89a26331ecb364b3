/*
 * dk_diag.h — diagnostics shipped in libdk_rx.so that are not part of the receive-path ABI (dk_rx.h).
 */
#ifndef DK_DIAG_H
#define DK_DIAG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Streaming read of `bytes` (multiple of 16) of device memory at `buf`; `scratch` = device u32[grid] (zeroed by the
 * caller). Used to measure the achievable HBM read bandwidth on the running box. Async on `stream`.
 * mode 0: grid-stride loads; 1: contiguous 8 KiB per wave step; 2: as 1 with nontemporal loads; 3: 16 KiB per wave
 * step, nontemporal; 4/5: 16 KiB per wave step by LDS-DMA (global_load_lds), nontemporal / default policy;
 * 6/7: as 3 with buffer_load_dwordx4 (32-bit offsets: bytes < 4 GiB), nontemporal / default policy;
 * 8: the receive kernel's phase-B pattern alone (1536-byte slots, quarter-waves reading 256-byte runs, nontemporal).
 * Returns 0, EINVAL or EIO. */
int dk_diag_read_probe(const void* buf, uint64_t bytes, uint32_t* scratch, uint32_t grid, int mode, void* stream);

/* The small-frame receive kernel's read/write mix alone: `bytes` (< 4 GiB, multiple of 64) read lane-contiguously in
 * 4 KiB wave steps, each step followed by nres u32 stores per lane into dst = nres arrays of bytes / 64 u32 (one per
 * 64-byte slot, as the result arrays are written); nres 0 reads only. The ceiling C3 is compared with. Async. */
int dk_diag_rw_probe(const void* buf, uint64_t bytes, uint32_t* dst, uint32_t nres, uint32_t* scratch, uint32_t grid,
                     void* stream);

/* The in-place TX checksum fill's memory pattern alone: the rw probe's read stream over `bytes` (< 4 GiB, multiple of
 * 64) plus one 64-byte line rewritten in place at the start of every `stride`-byte slot (multiple of 64; 0: none),
 * `late` wave-step rounds after it was read. flags bit 0: no read stream (the rewrites alone); bit 1: two 16-bit
 * stores at +24 and +50 (the IPv4 and TCP checksum fields) instead of the line; bit 2: the whole 128-byte line
 * (stride a multiple of 128). Overwrites the buffer. The ceiling
 * dk_tx_checksum is compared with. Async. */
int dk_diag_patch_probe(void* buf, uint64_t bytes, uint32_t stride, uint32_t late, uint32_t flags, uint32_t* scratch,
                        uint32_t grid, void* stream);

/* Per-path frame counters of a receive context (off by default). Paths: [0] vector path, frame <= 64 B in registers;
 * [1] vector path, frame streamed by a quarter-wave; [2] streamed but the L4 segment re-summed in-lane (IPv4
 * total_length far below the frame length); [3] per-lane byte-load path (unaligned frame, IHL != 5, or a frame too
 * short for the fixed headers). Enabling costs one atomic per wave per tile. */
struct dk_rx_ctx;
int dk_diag_path_stats_enable(struct dk_rx_ctx* ctx, int on);       /* 0, EINVAL or ENOMEM; on: counters reset */
int dk_diag_path_stats_read(struct dk_rx_ctx* ctx, uint64_t out[4]); /* synchronous; 0 or EINVAL */

/* Tuning overrides for A/B measurements and tests (-1 = the engine's own rule). A receive context starts on the
 * built-in rule and nothing but this call changes it: the process environment is never read (a LibOS process that
 * inherits an environment gets the same kernels as any other). knobs[] = {stage, split, small, sched, grid,
 * grid_per_cu, debug, lds_table, tail, udp_table, host_zc}:
 * stage/split/small force a kernel family on (1) or off (0), sched picks the wave schedule (0 round-robin tiles, 1 one
 * contiguous share per wave), grid / grid_per_cu fix the persistent grid, debug > 0 prints each launch's choice to
 * stderr, lds_table 0 keeps Active lookups on the global socket table (no LDS copy), tail sets the staged kernel's
 * dynamic tail (0 off, d > 0: the last ~d rounds of chunks handed out by per-pool counters instead of round-robin),
 * udp_table 0 / 1: the small-frame kernel looks local UDP binds up in the port table / in its LDS bind table whenever
 * that fits (the rule: when the binds are scattered over the port table), host_zc 0: dk_rx_process_host stages
 * frames through HBM copies even when they are in mapped page-locked memory (the rule reads them in place). */
#define DK_DIAG_RX_KNOBS 11
/* knobs[0 .. nknobs): the caller says how many it passes (knobs past nknobs are -1, the rule), so a caller built
 * against an older, shorter list never has its array read past its end. 0 or EINVAL. */
int dk_diag_rx_set_tuning(struct dk_rx_ctx* ctx, const int32_t* knobs, uint32_t nknobs);
/* The same for dk_tx_checksum / dk_tx_checksum_fields (process-wide, -1 = the rule). 0. */
int dk_diag_tx_set_tuning(int32_t split, int32_t sched, int32_t grid_per_cu);

/* Which walk dk_tcp_rx_process runs (dk_tcp.h): walk -1 the engine's rule, 0 one lane per connection, 1 one wave per
 * connection, 2 the relay walk (relay_waves 4 / 8 / 16 waves per connection, else 8), 3 the scan walk. A TCP context
 * starts on the rule; the environment is never read. 0 or EINVAL. */
struct dk_tcp_ctx;
int dk_diag_tcp_set_walk(struct dk_tcp_ctx* ctx, int32_t walk, int32_t relay_waves);
/* The walk the context's last dk_tcp_rx_process call ran (0 lane, 1 wave, 2 relay, 3 scan; -1 none yet). */
int dk_diag_tcp_last_walk(const struct dk_tcp_ctx* ctx);
/* How dk_tcp_rx_process orders the batch by connection: sort -1 the rule (one stable counting pass over the whole
 * key up to 255 table rows, rocPRIM's radix sort beyond), 1 the radix sort always. 0 or EINVAL. */
int dk_diag_tcp_set_sort(struct dk_tcp_ctx* ctx, int32_t sort);

#ifdef __cplusplus
}
#endif

#endif /* DK_DIAG_H */
