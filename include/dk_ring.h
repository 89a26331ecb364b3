/*
 * dk_ring.h — batch L1 ingest for the receive engine: a Linux AF_PACKET TPACKET_V3 receive
 * ring handed to the GPU a whole block range at a time.
 *
 * Replaces, on the receive side of the reference (paths relative to /root/reference/src/rust/):
 *   catpowder/linux/mod.rs:138-159   LinuxRuntime::receive: one recvfrom per frame into an 8 KiB stack buffer, then a
 *                                    full copy into a new DemiBuffer (DemiBuffer::from_slice + trim)
 *   runtime/network/consts.rs:42     RECEIVE_BATCH_SIZE = 4 frames per poll
 * The kernel fills fixed-size blocks of the mmap'd ring (PACKET_RX_RING + TPACKET_V3): a tpacket_block_desc, then a
 * chain of tpacket3_hdr + frame (tp_next_offset, frame at tp_mac, tp_snaplen bytes). A block the kernel has closed
 * carries TP_STATUS_USER. The engine turns the ready blocks into dk_rx_batch descriptors (offsets relative to the ring
 * base), copies the covered byte ranges to HBM with the host pipeline of dk_rx_process_host, runs the receive kernel
 * and returns the results; the caller then hands the blocks back (dk_ring_release_tpacket3).
 *
 * Conventions as dk_rx.h: 0 or a positive errno; the ring memory stays the caller's.
 */
#ifndef DK_RING_H
#define DK_RING_H

#include <stdint.h>

#include "dk_rx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Page-lock the ring (hipHostRegister) so the H2D copies run as DMA at full PCIe rate straight from it instead of
 * through a bounce buffer. EINVAL, EBUSY (already registered) or EIO. */
int dk_ring_register(void* ring, uint64_t ring_bytes);
int dk_ring_unregister(void* ring);

/* Walk blocks first_block .. first_block + nblocks - 1 (modulo ring_bytes / block_size) in order and write one
 * descriptor per frame: off = byte offset of the frame (tp_mac) from the ring base, len = tp_snaplen. Stops at the
 * first block that is not TP_STATUS_USER (still the kernel's). *n_frames = descriptors written, *n_blocks = blocks
 * consumed. A block whose packet chain leaves the block, or a frame longer than 65535 bytes, is malformed; a block
 * whose frames do not fit in the cap left is not consumed. Either stops the walk; then:
 *   - after at least one complete block: returns 0 with those blocks (the next call starts at the stopping block);
 *   - malformed first block: returns EBADMSG with *n_frames = 0 and *n_blocks = 1 (the block counts as consumed, so the
 *     caller hands it back with dk_ring_release_tpacket3 and the ring does not stall on it);
 *   - first block alone holds more than cap frames: returns ENOSPC with *n_blocks = 0 (retry with a larger cap). */
int dk_ring_scan_tpacket3(const void* ring, uint64_t ring_bytes, uint32_t block_size, uint32_t first_block,
                          uint32_t nblocks, uint32_t* off, uint16_t* len, uint32_t cap, uint32_t* n_frames,
                          uint32_t* n_blocks);

/* Hand blocks back to the kernel (block_status = TP_STATUS_KERNEL), as a TPACKET_V3 reader does after use. */
int dk_ring_release_tpacket3(void* ring, uint64_t ring_bytes, uint32_t block_size, uint32_t first_block,
                             uint32_t nblocks);

/* Scan up to nblocks ready blocks and process their frames through the receive engine (dk_rx_process_host pipeline;
 * results are host arrays of at least `cap` entries, in ring order). *n_frames / *n_blocks as dk_ring_scan_tpacket3.
 * Synchronous. Does not release the blocks (a malformed first block comes back as EBADMSG with *n_blocks = 1: release
 * it too). */
int dk_rx_process_tpacket3(dk_rx_ctx* ctx, const void* ring, uint64_t ring_bytes, uint32_t block_size,
                           uint32_t first_block, uint32_t nblocks, const dk_rx_results* res, uint32_t cap,
                           uint32_t* n_frames, uint32_t* n_blocks);

#ifdef __cplusplus
}
#endif

#endif /* DK_RING_H */
