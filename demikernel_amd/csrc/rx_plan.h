// rx_plan.h — host-only chunk planning of dk_rx_process_host (rx_host.cpp), kept apart from the HIP calls so the
// sanitizer build of the host code (tests/host_asan) can drive it on its own.
#pragma once

#include <algorithm>
#include <cstdint>
#include <vector>

namespace dk {

struct HostChunk {
    uint32_t a, e;    // frames [a, e) of the batch
    uint64_t lo, hi;  // blob bytes the chunk's in-blob frames cover, lo rounded down to 16 (hi == lo: none)
};

// Consecutive frame ranges of at most chunk_n frames each. Staged (zc == false): a chunk also stops before the frame
// that would take its covering byte range [lo, hi) past max_bytes (a chunk always takes at least one frame). Frames
// outside the blob (off + len > frames_bytes) cover no bytes: the kernel flags them BAD_DESC. Returns the largest
// chunk byte range.
inline uint64_t plan_host_chunks(const uint32_t* off, const uint16_t* len, uint32_t n, uint64_t frames_bytes,
                                 uint32_t chunk_n, bool zc, uint64_t max_bytes, std::vector<HostChunk>& out) {
    out.clear();
    uint64_t max_span = 0;
    if (chunk_n == 0) chunk_n = 1;
    for (uint32_t a = 0; a < n;) {
        uint64_t lo = UINT64_MAX, hi = 0;
        uint32_t e = a;
        while (e < n && e - a < chunk_n) {
            const uint64_t o = off[e], end = o + len[e];
            if (end <= frames_bytes) {
                const uint64_t nlo = std::min<uint64_t>(lo, o & ~(uint64_t)15), nhi = std::max(hi, end);
                if (!zc && e > a && nhi - nlo > max_bytes) break;
                lo = nlo;
                hi = nhi;
            }
            e++;
        }
        if (lo == UINT64_MAX) lo = hi = 0;
        out.push_back({a, e, lo, hi});
        max_span = std::max(max_span, hi - lo);
        a = e;
    }
    return max_span;
}

}  // namespace dk
