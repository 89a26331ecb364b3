// diag.hip — on-box HBM read-bandwidth probe (include/dk_diag.h). Not part of the receive path: bench.py uses it to
// report the measured streaming-read ceiling next to the 8 TB/s spec (SURVEY.md §8(d) "Roofline").
#include <hip/hip_runtime.h>

#include "../../include/dk_diag.h"

namespace {

constexpr int kBlock = 256;
constexpr int kUnroll = 8;

__device__ __forceinline__ uint4 ld(const uint4* p, bool nt) {
    if (nt) {
        uint4 v;
        v.x = __builtin_nontemporal_load(&p->x);
        v.y = __builtin_nontemporal_load(&p->y);
        v.z = __builtin_nontemporal_load(&p->z);
        v.w = __builtin_nontemporal_load(&p->w);
        return v;
    }
    return *p;
}

// mode 0: grid-stride, the 8 loads of a lane one grid-stride apart.
// mode 1: each wave streams a contiguous 8 KiB piece per step (lane-contiguous 16 B, 8 x 1 KiB in flight).
// mode 2: as mode 1 with nontemporal loads.
template <int kMode>
__global__ __launch_bounds__(kBlock) void read_probe(const uint4* __restrict__ p, uint64_t n16, uint32_t* out) {
    uint32_t acc = 0;
    if (kMode == 0) {
        const uint64_t stride = (uint64_t)gridDim.x * kBlock;
        uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
        for (; i + (kUnroll - 1) * stride < n16; i += kUnroll * stride) {
            uint4 v[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; u++) v[u] = p[i + u * stride];
#pragma unroll
            for (int u = 0; u < kUnroll; u++) acc ^= v[u].x + v[u].y + v[u].z + v[u].w;
        }
        for (; i < n16; i += stride) {
            const uint4 v = p[i];
            acc ^= v.x + v.y + v.z + v.w;
        }
    } else {
        const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
        const uint64_t w = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
        const uint32_t lane = threadIdx.x & 63;
        const uint64_t piece = 64 * kUnroll;  // 16-byte words per wave step
        for (uint64_t base = w * piece; base < n16; base += nwaves * piece) {
            uint4 v[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; u++) {
                const uint64_t i = base + u * 64 + lane;
                v[u] = i < n16 ? ld(p + i, kMode == 2) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < kUnroll; u++) acc ^= v[u].x + v[u].y + v[u].z + v[u].w;
        }
    }
    acc = __reduce_add_sync(~0ull, acc);
    if ((threadIdx.x & 63) == 0) atomicXor(out + blockIdx.x, acc);
}

// mode 3: register loads, 16 x 1 KiB per wave step in flight.
// mode 4 / 5: LDS-DMA (global_load_lds_dwordx4), nontemporal / default policy, 16 x 1 KiB per wave step into a
// per-wave 16 KiB LDS slot, read back with ds_read_b128 and summed.
// mode 6 / 7: as mode 3 with buffer_load_dwordx4 (SGPR resource, 32-bit lane offsets), nontemporal / default.
typedef __attribute__((address_space(3))) void lds_void;
template <int kMode>
__global__ __launch_bounds__(kBlock) void read_probe16(const uint4* __restrict__ p, uint64_t n16, uint32_t* out) {
    __shared__ uint4 slot[kBlock / 64][16][64];
    constexpr int U = 16;
    uint32_t acc = 0;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    const uint32_t wv = threadIdx.x >> 6;
    const uint64_t w = (uint64_t)blockIdx.x * (kBlock / 64) + wv;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t piece = 64 * U;
    for (uint64_t base = w * piece; base < n16; base += nwaves * piece) {
        if (kMode == 3) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint64_t i = base + u * 64 + lane;
                v[u] = i < n16 ? ld(p + i, true) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < U; u++) acc ^= v[u].x + v[u].y + v[u].z + v[u].w;
        } else if (kMode >= 6) {
            // buffer_load_dwordx4: SGPR resource + 32-bit per-lane offset (blob < 4 GiB), nt (6) / default (7)
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, 0xFFFFFFFF, 0x00020000);
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint64_t i = min(base + u * 64 + lane, n16 - 1);
                const auto r = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(i * 16), 0, kMode == 6 ? 2 : 0);
                v[u] = make_uint4(r[0], r[1], r[2], r[3]);
            }
#pragma unroll
            for (int u = 0; u < U; u++) acc ^= v[u].x + v[u].y + v[u].z + v[u].w;
        } else {
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint64_t i = min(base + u * 64 + lane, n16 - 1);
                __builtin_amdgcn_global_load_lds((const void*)(p + i), (lds_void*)&slot[wv][u][0], 16, 0,
                                                 kMode == 4 ? 2 : 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint4 v = slot[wv][u][lane];
                acc ^= v.x + v.y + v.z + v.w;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    }
    acc = __reduce_add_sync(~0ull, acc);
    if ((threadIdx.x & 63) == 0) atomicXor(out + blockIdx.x, acc);
}

// mode 8: the receive kernel's phase-B access pattern without the rest of the kernel: 1536-byte slots, a wave step
// covers 8 consecutive slots as 2 rounds of 4 quarter-waves x 6 buffer_load_dwordx4 (nt) of 256 contiguous bytes;
// grid-strided wave steps (as mode 6).
__global__ __launch_bounds__(kBlock) void read_probe_frames(const uint4* __restrict__ p, uint64_t n16, uint32_t* out) {
    constexpr uint32_t kSlot16 = 96;  // 1536-byte slot in 16-byte granules
    uint32_t acc = 0;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    const uint64_t w = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63, q = lane >> 4, l16 = lane & 15;
    const uint64_t piece = 8 * kSlot16;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, 0xFFFFFFFF, 0x00020000);
    for (uint64_t base = w * piece; base < n16; base += nwaves * piece) {
        uint4 v[12];
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
            for (int u = 0; u < 6; u++) {
                const uint64_t i = min(base + (4 * h + q) * kSlot16 + 16 * u + l16, n16 - 1);
                const auto r = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(i * 16), 0, 2);
                v[6 * h + u] = make_uint4(r[0], r[1], r[2], r[3]);
            }
#pragma unroll
        for (int u = 0; u < 12; u++) acc ^= v[u].x + v[u].y + v[u].z + v[u].w;
    }
    acc = __reduce_add_sync(~0ull, acc);
    if ((threadIdx.x & 63) == 0) atomicXor(out + blockIdx.x, acc);
}

// modes 9-11: the small-frame (64-byte slot) access pattern, buffer loads (nt), grid-strided 4 KiB wave chunks:
// 9: lane l reads the 4 granules of slot l (lane stride 64 B), one chunk (4 loads per lane) in flight per wave step;
// 10: as 9 with 4 chunks (16 loads per lane) in flight; 11: one chunk read lane-contiguously (1 KiB per load).
template <int kMode>
__global__ __launch_bounds__(kBlock) void read_probe_small(const uint4* __restrict__ p, uint64_t n16, uint32_t* out) {
    constexpr int C = kMode == 10 ? 4 : 1;  // chunks per wave step
    uint32_t acc = 0;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    const uint64_t w = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t piece = 256 * C;  // granules per wave step
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, 0xFFFFFFFF, 0x00020000);
    for (uint64_t base = w * piece; base < n16; base += nwaves * piece) {
        uint4 v[4 * C];
#pragma unroll
        for (int c = 0; c < C; c++)
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint64_t g = kMode == 11 ? base + 64 * k + lane : base + 256 * c + 4 * lane + k;
                const uint64_t i = min(g, n16 - 1);
                const auto r = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(i * 16), 0, 2);
                v[4 * c + k] = make_uint4(r[0], r[1], r[2], r[3]);
            }
#pragma unroll
        for (int u = 0; u < 4 * C; u++) acc ^= v[u].x + v[u].y + v[u].z + v[u].w;
    }
    acc = __reduce_add_sync(~0ull, acc);
    if ((threadIdx.x & 63) == 0) atomicXor(out + blockIdx.x, acc);
}

// The read/write mix of the small-frame kernel without the rest of it: grid-strided 4 KiB wave steps read
// lane-contiguously (4 x 1 KiB buffer loads, nt), each followed by `nres` u32 stores per lane (nt) into nres arrays of
// bytes / 64 entries (one u32 per 64-byte slot, as the result record's arrays are written per 64-frame chunk).
__global__ __launch_bounds__(kBlock) void rw_probe(const uint4* __restrict__ p, uint64_t n16, uint32_t* __restrict__ dst,
                                                   uint32_t nres, uint32_t* out) {
    uint32_t acc = 0;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    const uint64_t w = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nslots = n16 / 4;  // 64-byte slots: entries per result array
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, 0xFFFFFFFF, 0x00020000);
    for (uint64_t base = w * 256; base < n16; base += nwaves * 256) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t i = min(base + 64 * k + lane, n16 - 1);
            const auto r = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(i * 16), 0, 2);
            v[k] = make_uint4(r[0], r[1], r[2], r[3]);
        }
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) x ^= v[k].x + v[k].y + v[k].z + v[k].w;
        acc += x;
        const uint64_t slot = base / 4 + lane;
        if (slot < nslots)
            for (uint32_t a = 0; a < nres; a++) __builtin_nontemporal_store(x + a, dst + a * nslots + slot);
    }
    acc = __reduce_add_sync(~0ull, acc);
    if ((threadIdx.x & 63) == 0) atomicXor(out + blockIdx.x, acc);
}

// The in-place TX contract's memory pattern alone: the same 4 KiB wave-step read stream, plus one 64-byte line
// rewritten at the head of every `stride`-byte slot (a frame's header window) by the lane whose 16-byte piece starts
// it; `late` steps later (0: the step that read it), as the checksum is known only after the whole frame is read.
// flags bit 0: no read stream (the rewrites alone); bit 1: two 16-bit stores at +24 and +50 (the IPv4 and TCP
// checksum fields) instead of the 64-byte line; bit 2: the 128-byte line instead.
__global__ __launch_bounds__(kBlock) void patch_probe(uint4* __restrict__ p, uint64_t n16, uint32_t stride16,
                                                      uint32_t late, uint32_t flags, uint32_t* out) {
    uint32_t acc = 0;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    const uint64_t w = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, 0xFFFFFFFF, 0x00020000);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    for (uint64_t base = w * 256; base < n16; base += nwaves * 256) {
        uint32_t x = (uint32_t)base;
        if (!(flags & 1)) {
            uint4 v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint64_t i = min(base + 64 * k + lane, n16 - 1);
                const auto r = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(i * 16), 0, 2);
                v[k] = make_uint4(r[0], r[1], r[2], r[3]);
            }
#pragma unroll
            for (int k = 0; k < 4; k++) x ^= v[k].x + v[k].y + v[k].z + v[k].w;
        }
        acc += x;
        const uint64_t wb = base - (uint64_t)late * nwaves * 256;  // the step whose heads this one rewrites
        if (stride16 && base >= (uint64_t)late * nwaves * 256)
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint64_t i = wb + 64 * k + lane;
                if (i % stride16 == 0 && i + 8 <= n16) {
                    if (flags & 4) {  // the 128-byte line (the L2 line of gfx950)
                        u32x4* q = reinterpret_cast<u32x4*>(p + i);
#pragma unroll
                        for (int j = 0; j < 8; j++) q[j] = u32x4{x, x + 1, x + 2, x + j};
                    } else if (flags & 2) {
                        uint16_t* h = reinterpret_cast<uint16_t*>(p + i);
                        h[12] = (uint16_t)x;
                        h[25] = (uint16_t)(x >> 16);
                    } else {
                        u32x4* q = reinterpret_cast<u32x4*>(p + i);
#pragma unroll
                        for (int j = 0; j < 4; j++) q[j] = u32x4{x, x + 1, x + 2, x + j};
                    }
                }
            }
    }
    acc = __reduce_add_sync(~0ull, acc);
    if ((threadIdx.x & 63) == 0) atomicXor(out + blockIdx.x, acc);
}

}  // namespace

extern "C" int dk_diag_patch_probe(void* buf, uint64_t bytes, uint32_t stride, uint32_t late, uint32_t flags,
                                   uint32_t* scratch, uint32_t grid, void* stream) {
    if (!buf || !scratch || grid == 0 || stride % 64 || bytes % 64 || bytes > 0xFFFFFFFFull || flags > 7) return 22;
    if ((flags & 4) && stride % 128) return 22;
    hipLaunchKernelGGL(patch_probe, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, (uint4*)buf, bytes / 16,
                       stride / 16, late, flags, scratch);
    return hipGetLastError() == hipSuccess ? 0 : 5;
}

extern "C" int dk_diag_rw_probe(const void* buf, uint64_t bytes, uint32_t* dst, uint32_t nres, uint32_t* scratch,
                                uint32_t grid, void* stream) {
    if (!buf || !scratch || grid == 0 || (nres && !dst) || bytes > 0xFFFFFFFFull) return 22;
    hipLaunchKernelGGL(rw_probe, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, (const uint4*)buf, bytes / 16, dst,
                       nres, scratch);
    return hipGetLastError() == hipSuccess ? 0 : 5;
}

extern "C" int dk_diag_read_probe(const void* buf, uint64_t bytes, uint32_t* scratch, uint32_t grid, int mode,
                                  void* stream) {
    if (!buf || !scratch || grid == 0 || mode < 0 || mode > 11) return 22;
    if (mode >= 6 && bytes > 0xFFFFFFFFull) return 22;  // buffer offsets are 32-bit
    const uint4* p = (const uint4*)buf;
    const hipStream_t s = (hipStream_t)stream;
    if (mode == 0) hipLaunchKernelGGL(read_probe<0>, dim3(grid), dim3(kBlock), 0, s, p, bytes / 16, scratch);
    if (mode == 1) hipLaunchKernelGGL(read_probe<1>, dim3(grid), dim3(kBlock), 0, s, p, bytes / 16, scratch);
    if (mode == 2) hipLaunchKernelGGL(read_probe<2>, dim3(grid), dim3(kBlock), 0, s, p, bytes / 16, scratch);
    if (mode == 3) hipLaunchKernelGGL(read_probe16<3>, dim3(grid), dim3(kBlock), 0, s, p, bytes / 16, scratch);
    if (mode == 4) hipLaunchKernelGGL(read_probe16<4>, dim3(grid), dim3(kBlock), 0, s, p, bytes / 16, scratch);
    if (mode == 5) hipLaunchKernelGGL(read_probe16<5>, dim3(grid), dim3(kBlock), 0, s, p, bytes / 16, scratch);
    if (mode == 6) hipLaunchKernelGGL(read_probe16<6>, dim3(grid), dim3(kBlock), 0, s, p, bytes / 16, scratch);
    if (mode == 7) hipLaunchKernelGGL(read_probe16<7>, dim3(grid), dim3(kBlock), 0, s, p, bytes / 16, scratch);
    if (mode == 8) hipLaunchKernelGGL(read_probe_frames, dim3(grid), dim3(kBlock), 0, s, p, bytes / 16, scratch);
    if (mode == 9) hipLaunchKernelGGL(read_probe_small<9>, dim3(grid), dim3(kBlock), 0, s, p, bytes / 16, scratch);
    if (mode == 10) hipLaunchKernelGGL(read_probe_small<10>, dim3(grid), dim3(kBlock), 0, s, p, bytes / 16, scratch);
    if (mode == 11) hipLaunchKernelGGL(read_probe_small<11>, dim3(grid), dim3(kBlock), 0, s, p, bytes / 16, scratch);
    return hipGetLastError() == hipSuccess ? 0 : 5;
}
