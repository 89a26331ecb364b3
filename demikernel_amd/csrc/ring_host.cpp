// ring_host.cpp — TPACKET_V3 ring ingest (include/dk_ring.h).
//
// The reference's catpowder receive path (catpowder/linux/mod.rs:138-159) takes one frame per recvfrom syscall into an
// 8 KiB stack buffer and copies it again into a fresh DemiBuffer, at most RECEIVE_BATCH_SIZE = 4 frames per poll
// (runtime/network/consts.rs:42). Here the kernel's own TPACKET_V3 blocks are the batch: the ready blocks are walked on
// the host (header chain only, ~ns per frame), their frames become dk_rx_batch descriptors relative to the ring base,
// and dk_rx_process_host moves the covered byte ranges to HBM (DMA from the page-locked ring) and runs the kernel.
#include <hip/hip_runtime.h>
#include <linux/if_packet.h>

#include <algorithm>
#include <cerrno>
#include <cstddef>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/dk_ring.h"
#include "rx_common.h"

namespace {

// One ready block -> descriptors. Returns 0, EBADMSG (malformed chain) or ENOSPC (cap reached, nothing written).
int scan_block(const uint8_t* ring, uint64_t base, uint32_t block_size, uint32_t* off, uint16_t* len, uint32_t cap,
               uint32_t& n) {
    const uint8_t* b = ring + base;
    tpacket_block_desc bd;
    std::memcpy(&bd, b, sizeof(bd));
    const tpacket_hdr_v1& h = bd.hdr.bh1;
    if (h.num_pkts == 0) return 0;
    if ((uint64_t)n + h.num_pkts > cap) return ENOSPC;
    uint64_t p = h.offset_to_first_pkt;
    for (uint32_t k = 0; k < h.num_pkts; k++) {
        if (p + sizeof(tpacket3_hdr) > block_size) return EBADMSG;
        tpacket3_hdr t;
        std::memcpy(&t, b + p, sizeof(t));
        const uint64_t f = p + t.tp_mac;
        if (t.tp_snaplen > 0xFFFFu || f + t.tp_snaplen > block_size) return EBADMSG;
        off[n + k] = (uint32_t)(base + f);
        len[n + k] = (uint16_t)t.tp_snaplen;
        if (k + 1 < h.num_pkts) {
            if (t.tp_next_offset == 0) return EBADMSG;
            // the chain is a dependent walk through the block (one cache miss per frame): fetch the header a few
            // frames ahead, assuming the stride repeats (any address inside the block is harmless)
            const uint64_t ahead = p + 4ull * t.tp_next_offset;
            if (ahead < block_size) __builtin_prefetch(b + ahead, 0, 0);
            p += t.tp_next_offset;
        }
    }
    n += h.num_pkts;
    return 0;
}

// Page-locked descriptor staging for dk_rx_process_tpacket3 (one per host thread; contexts are single-threaded,
// dk_rx.h): the pipeline's descriptor copies then run as DMA like the frame copies instead of bouncing through
// pageable memory. Grown on demand and kept for the process lifetime (no destructor: freeing at thread exit could run
// after the HIP runtime has shut down).
struct PinnedDescs {
    uint32_t* off = nullptr;
    uint16_t* len = nullptr;
    uint32_t cap = 0;
    void release() {
        if (off) (void)hipHostFree(off);
        if (len) (void)hipHostFree(len);
        off = nullptr;
        len = nullptr;
        cap = 0;
    }
    int ensure(uint32_t n) {
        if (cap >= n) return 0;
        release();
        if (hipHostMalloc(reinterpret_cast<void**>(&off), (size_t)n * sizeof(uint32_t), hipHostMallocDefault) !=
                hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&len), (size_t)n * sizeof(uint16_t), hipHostMallocDefault) !=
                hipSuccess) {
            release();
            return ENOMEM;
        }
        cap = n;
        return 0;
    }
};
thread_local PinnedDescs t_descs;

constexpr uint32_t kScanThreads = 8;              // host threads a long ring scan may use
constexpr uint32_t kScanBlocksPerThread = 4;      // a thread walks at least this many blocks ...
constexpr uint32_t kScanFramesPerThread = 16384;  // ... and this many frames (~0.2 ms of walk: more than a thread start)

uint32_t* status_word(uint8_t* ring, uint64_t base) {
    return reinterpret_cast<uint32_t*>(ring + base + offsetof(tpacket_block_desc, hdr.bh1.block_status));
}

}  // namespace

extern "C" {

int dk_ring_register(void* ring, uint64_t ring_bytes) {
    if (!ring || ring_bytes == 0) return EINVAL;
    const hipError_t e = hipHostRegister(ring, ring_bytes, hipHostRegisterDefault);
    if (e == hipErrorHostMemoryAlreadyRegistered) return EBUSY;
    return e == hipSuccess ? 0 : EIO;
}

int dk_ring_unregister(void* ring) {
    if (!ring) return EINVAL;
    return hipHostUnregister(ring) == hipSuccess ? 0 : EINVAL;
}

int dk_ring_scan_tpacket3(const void* ring, uint64_t ring_bytes, uint32_t block_size, uint32_t first_block,
                          uint32_t nblocks, uint32_t* off, uint16_t* len, uint32_t cap, uint32_t* n_frames,
                          uint32_t* n_blocks) {
    if (!ring || !n_frames || !n_blocks || (cap && (!off || !len))) return EINVAL;
    *n_frames = *n_blocks = 0;
    if (block_size < sizeof(tpacket_block_desc) || ring_bytes < block_size || ring_bytes > DK_RX_MAX_BLOB) return EINVAL;
    const uint64_t nring = ring_bytes / block_size;
    if (first_block >= nring) return EINVAL;
    uint8_t* r = const_cast<uint8_t*>(static_cast<const uint8_t*>(ring));
    // Pass 1, block descriptors only: the ready blocks that fit in cap and each one's first output slot. A block that
    // would overflow cap ends the scan before it (ENOSPC when it is the first: nothing consumed).
    std::vector<uint32_t> start;
    uint32_t n = 0, k = 0;
    for (; k < nblocks && k < nring; k++) {
        const uint64_t base = ((first_block + k) % nring) * block_size;
        uint32_t status;
        __atomic_load(status_word(r, base), &status, __ATOMIC_ACQUIRE);  // pairs with the kernel's block close
        if (!(status & TP_STATUS_USER)) break;                            // still the kernel's
        tpacket_block_desc bd;
        std::memcpy(&bd, r + base, sizeof(bd));
        const uint32_t np = bd.hdr.bh1.num_pkts;
        if ((uint64_t)n + np > cap) {
            if (k == 0) return ENOSPC;
            break;
        }
        start.push_back(n);
        n += np;
        if (n == cap) {  // full: the next block cannot fit
            k++;
            break;
        }
    }
    const uint32_t nb = k;
    // Pass 2: each block's header chain into its slots. The chains are independent, so a long scan walks blocks on
    // several threads (the walk is one cache miss per frame: ~14 ns a frame on one core of the GPU box).
    std::vector<int> brc(nb, 0);
    auto walk = [&](uint32_t j0, uint32_t j1) {
        for (uint32_t j = j0; j < j1; j++) {
            uint32_t pos = start[j];
            brc[j] = scan_block(r, ((first_block + j) % nring) * block_size, block_size, off, len, cap, pos);
            if (brc[j]) break;  // later blocks of this range are not returned
        }
    };
    const uint32_t hw = std::max(1u, std::thread::hardware_concurrency());
    const uint32_t nt = std::min({kScanThreads, hw, nb / kScanBlocksPerThread, n / kScanFramesPerThread});
    if (nt > 1) {
        // thread t walks blocks [nb t / nt, nb (t + 1) / nt); the calling thread takes range 0 and, when a thread
        // could not be started, that range and every later one
        std::vector<std::thread> th;
        uint32_t started = 1;
        try {
            for (; started < nt; started++) th.emplace_back(walk, nb * started / nt, nb * (started + 1) / nt);
        } catch (...) {
        }
        walk(0, nb / nt);
        if (started < nt) walk(nb * started / nt, nb);
        for (std::thread& t : th) t.join();
    } else {
        walk(0, nb);
    }
    // The first malformed block ends the scan: the blocks before it are returned; when it is the first, it is reported
    // (EBADMSG) and counted as consumed so that the caller hands it back.
    for (uint32_t j = 0; j < nb; j++) {
        if (!brc[j]) continue;
        if (j == 0) {
            *n_frames = 0;
            *n_blocks = 1;
            return brc[j];
        }
        *n_frames = start[j];
        *n_blocks = j;
        return 0;
    }
    *n_frames = n;
    *n_blocks = nb;
    return 0;
}

int dk_ring_release_tpacket3(void* ring, uint64_t ring_bytes, uint32_t block_size, uint32_t first_block,
                             uint32_t nblocks) {
    if (!ring || block_size < sizeof(tpacket_block_desc) || ring_bytes < block_size) return EINVAL;
    const uint64_t nring = ring_bytes / block_size;
    if (first_block >= nring || nblocks > nring) return EINVAL;
    uint8_t* r = static_cast<uint8_t*>(ring);
    for (uint32_t k = 0; k < nblocks; k++) {
        uint32_t status = TP_STATUS_KERNEL;
        __atomic_store(status_word(r, ((first_block + k) % nring) * block_size), &status, __ATOMIC_RELEASE);
    }
    return 0;
}

int dk_rx_process_tpacket3(dk_rx_ctx* ctx, const void* ring, uint64_t ring_bytes, uint32_t block_size,
                           uint32_t first_block, uint32_t nblocks, const dk_rx_results* res, uint32_t cap,
                           uint32_t* n_frames, uint32_t* n_blocks) {
    if (!ctx || !res || !n_frames || !n_blocks) return EINVAL;
    *n_frames = *n_blocks = 0;
    int rc = t_descs.ensure(cap ? cap : 1);
    if (rc) return rc;
    rc = dk_ring_scan_tpacket3(ring, ring_bytes, block_size, first_block, nblocks, t_descs.off, t_descs.len, cap,
                               n_frames, n_blocks);
    if (rc || *n_frames == 0) return rc;
    const dk_rx_batch b{static_cast<const uint8_t*>(ring), ring_bytes, t_descs.off, t_descs.len, *n_frames, 0};
    return dk_rx_process_ring_host(ctx, &b, res);
}

}  // extern "C"
