// TEST INFRASTRUCTURE ONLY: driver for the ASan + UBSan build of the product's host-side code (tests/host_asan/Makefile):
// ring_host.cpp (TPACKET_V3 block walker), demi_host.cpp (results -> demi_sgarray_t) and the host chunk planner of
// dk_rx_process_host (rx_plan.h), compiled with -fsanitize=address,undefined. tests/test_host_asan.py feeds it valid,
// corrupted and fuzzed inputs and compares its outputs with the regular build of libdk_rx.so.
//
//   host_asan ring    in out   in:  u64 ring_bytes | u32 block_size | u32 first | u32 nblocks | u32 cap | ring bytes
//                              out: i32 rc | u32 n_frames | u32 n_blocks | off[n_frames] u32 | len[n_frames] u16
//   host_asan release in out   in:  u64 ring_bytes | u32 block_size | u32 first | u32 nblocks | ring bytes
//                              out: i32 rc | ring bytes
//   host_asan udp     in out   in:  u32 n | u32 cap | u32 use_tokens | u64 blob_bytes | off, meta, src, ports, payload
//                                   (u32[n] each) | blob
//                              out: i32 rc | u32 nout | frame_idx[nout] u32 | per sgarray: token, seg buf - blob, len,
//                                   numsegs, sockaddr_in (16 B)
//   host_asan tcp     in out   in:  u32 n | u32 count | u32 cap | u32 use_tokens | u64 blob_bytes | off u32[n] |
//                                   deliv (dk_tcp_view)[count] | blob
//                              out: i32 rc | u32 nout | per sgarray: token, seg buf - blob (or ~0), len, numsegs
//   host_asan plan    in out   in:  u32 n | u64 frames_bytes | u32 chunk_n | u32 zc | u64 max_bytes | off u32[n] |
//                                   len u16[n]
//                              out: u64 max_span | u32 nchunks | per chunk: u32 a, u32 e, u64 lo, u64 hi
//   host_asan ltable  in out   in:  u32 cap | u32 cfg_ip | slots u32[4 cap] (the Active table's open-addressing slots)
//                              out: i32 built | u32 n | u32 nbuckets | u32 nwords | words u32[nwords]
//                              (the LDS Active table builder of lds_table.h)
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../demikernel_amd/csrc/lds_table.h"
#include "../../demikernel_amd/csrc/rx_plan.h"
#include "../../include/dk_demi.h"
#include "../../include/dk_ring.h"

// dk_rx_process_tpacket3 (ring_host.cpp) hands the scanned frames to the GPU pipeline; this host-only build never
// reaches it (the driver exercises the scan and release entry points), so the symbol resolves to a refusal here.
extern "C" int dk_rx_process_host(dk_rx_ctx*, const dk_rx_batch*, const dk_rx_results*, uint32_t) { return ENOSYS; }
int dk_rx_process_ring_host(dk_rx_ctx*, const dk_rx_batch*, const dk_rx_results*) { return ENOSYS; }

namespace {
FILE* g_in;
FILE* g_out;
template <class T>
void rd(T* p, size_t n) {
    if (n && fread(p, sizeof(T), n, g_in) != n) {
        fprintf(stderr, "short read\n");
        exit(2);
    }
}
template <class T>
T rd1() {
    T v;
    rd(&v, 1);
    return v;
}
template <class T>
void wr(const T* p, size_t n) {
    if (n) fwrite(p, sizeof(T), n, g_out);
}
template <class T>
void wr1(T v) {
    wr(&v, 1);
}

int do_ring(bool release) {
    const uint64_t ring_bytes = rd1<uint64_t>();
    const uint32_t block_size = rd1<uint32_t>(), first = rd1<uint32_t>(), nblocks = rd1<uint32_t>();
    const uint32_t cap = release ? 0 : rd1<uint32_t>();
    std::vector<uint8_t> ring(ring_bytes);  // exactly the ring: any read past it is a heap overflow under ASan
    rd(ring.data(), ring.size());
    if (release) {
        const int rc = dk_ring_release_tpacket3(ring.data(), ring_bytes, block_size, first, nblocks);
        wr1<int32_t>(rc);
        wr(ring.data(), ring.size());
        return 0;
    }
    std::vector<uint32_t> off(cap);
    std::vector<uint16_t> len(cap);
    uint32_t nf = 0, nb = 0;
    const int rc = dk_ring_scan_tpacket3(ring.data(), ring_bytes, block_size, first, nblocks, cap ? off.data() : nullptr,
                                         cap ? len.data() : nullptr, cap, &nf, &nb);
    wr1<int32_t>(rc);
    wr1<uint32_t>(nf);
    wr1<uint32_t>(nb);
    wr(off.data(), nf);
    wr(len.data(), nf);
    return 0;
}

void wr_sga(const dk_demi_sgarray_t& s, const uint8_t* blob) {
    uint64_t tok;
    memcpy(&tok, &s.sga_buf, sizeof tok);
    void* sb;
    memcpy(&sb, &s.sga_segs[0].sgaseg_buf, sizeof sb);
    uint32_t sl, ns;
    memcpy(&sl, &s.sga_segs[0].sgaseg_len, sizeof sl);
    memcpy(&ns, &s.sga_numsegs, sizeof ns);
    wr1<uint64_t>(tok);
    wr1<uint64_t>(sb ? (uint64_t)((const uint8_t*)sb - blob) : ~0ull);
    wr1<uint32_t>(sl);
    wr1<uint32_t>(ns);
    uint8_t addr[16];
    memcpy(addr, &s.sga_addr, 16);
    wr(addr, 16);
}

int do_udp() {
    const uint32_t n = rd1<uint32_t>(), cap = rd1<uint32_t>(), use_tokens = rd1<uint32_t>();
    const uint64_t blob_bytes = rd1<uint64_t>();
    std::vector<uint32_t> off(n), meta(n), src(n), ports(n), payload(n);
    rd(off.data(), n);
    rd(meta.data(), n);
    rd(src.data(), n);
    rd(ports.data(), n);
    rd(payload.data(), n);
    std::vector<uint8_t> blob(blob_bytes ? blob_bytes : 1);
    rd(blob.data(), blob_bytes);
    std::vector<void*> tokens(n);
    for (uint32_t i = 0; i < n; i++) tokens[i] = reinterpret_cast<void*>((uintptr_t)(0x1000 + i));
    std::vector<dk_demi_sgarray_t> out(cap);
    std::vector<uint32_t> idx(cap);
    uint32_t nout = 0;
    const int rc = dk_rx_into_sgarrays(blob.data(), off.data(), n, meta.data(), src.data(), ports.data(),
                                       payload.data(), use_tokens ? tokens.data() : nullptr,
                                       cap ? out.data() : nullptr, cap ? idx.data() : nullptr, cap, &nout);
    wr1<int32_t>(rc);
    wr1<uint32_t>(nout);
    wr(idx.data(), nout);
    for (uint32_t k = 0; k < nout; k++) wr_sga(out[k], blob.data());
    return 0;
}

int do_tcp() {
    const uint32_t n = rd1<uint32_t>(), count = rd1<uint32_t>(), cap = rd1<uint32_t>(), use_tokens = rd1<uint32_t>();
    const uint64_t blob_bytes = rd1<uint64_t>();
    std::vector<uint32_t> off(n);
    rd(off.data(), n);
    std::vector<dk_tcp_view> deliv(count);
    rd(deliv.data(), count);
    std::vector<uint8_t> blob(blob_bytes ? blob_bytes : 1);
    rd(blob.data(), blob_bytes);
    std::vector<void*> tokens(n);
    for (uint32_t i = 0; i < n; i++) tokens[i] = reinterpret_cast<void*>((uintptr_t)(0x1000 + i));
    std::vector<dk_demi_sgarray_t> out(cap);
    uint32_t nout = 0;
    const int rc = dk_tcp_into_sgarrays(blob.data(), n ? off.data() : nullptr, n, count ? deliv.data() : nullptr, count,
                                        use_tokens ? tokens.data() : nullptr, cap ? out.data() : nullptr, cap, &nout);
    wr1<int32_t>(rc);
    wr1<uint32_t>(nout);
    for (uint32_t k = 0; k < nout; k++) wr_sga(out[k], blob.data());
    return 0;
}

int do_plan() {
    const uint32_t n = rd1<uint32_t>();
    const uint64_t frames_bytes = rd1<uint64_t>();
    const uint32_t chunk_n = rd1<uint32_t>(), zc = rd1<uint32_t>();
    const uint64_t max_bytes = rd1<uint64_t>();
    std::vector<uint32_t> off(n);
    std::vector<uint16_t> len(n);
    rd(off.data(), n);
    rd(len.data(), n);
    std::vector<dk::HostChunk> ch;
    const uint64_t span = dk::plan_host_chunks(off.data(), len.data(), n, frames_bytes, chunk_n, zc != 0, max_bytes, ch);
    wr1<uint64_t>(span);
    wr1<uint32_t>((uint32_t)ch.size());
    for (const auto& c : ch) {
        wr1<uint32_t>(c.a);
        wr1<uint32_t>(c.e);
        wr1<uint64_t>(c.lo);
        wr1<uint64_t>(c.hi);
    }
    return 0;
}

int do_ltable() {
    const uint32_t cap = rd1<uint32_t>(), cfg_ip = rd1<uint32_t>();
    std::vector<uint32_t> slots((size_t)cap * 4);
    rd(slots.data(), slots.size());
    std::vector<uint32_t> words;
    uint32_t n = 0, nb = 0;
    const bool ok = dk::build_lds_table(slots, cap, cfg_ip, words, n, nb);
    wr1<int32_t>(ok ? 1 : 0);
    wr1<uint32_t>(ok ? n : 0);
    wr1<uint32_t>(ok ? nb : 0);
    wr1<uint32_t>(ok ? (uint32_t)words.size() : 0);
    if (ok) wr(words.data(), words.size());
    return 0;
}
// utable: 65,536 port-table words (kPortUdpLocal) -> ok, mask, seed, direct lines, then the table's slots.
int do_utable() {
    std::vector<uint32_t> local(65536);
    rd(local.data(), local.size());
    std::vector<uint32_t> words;
    uint32_t mask = 0, seed = 0, lines = 0;
    const bool ok = dk::build_udp_table(local.data(), words, mask, seed, lines);
    wr1<int32_t>(ok ? 1 : 0);
    wr1<uint32_t>(ok ? mask : 0);
    wr1<uint32_t>(ok ? seed : 0);
    wr1<uint32_t>(lines);
    if (ok) wr(words.data(), words.size());
    return 0;
}
}  // namespace

int main(int argc, char** argv) {
    if (argc != 4) {
        fprintf(stderr, "usage: %s ring|release|udp|tcp|plan|ltable|utable in out\n", argv[0]);
        return 2;
    }
    g_in = fopen(argv[2], "rb");
    g_out = fopen(argv[3], "wb");
    if (!g_in || !g_out) return 2;
    const char* m = argv[1];
    int rc = !strcmp(m, "ring") ? do_ring(false) : !strcmp(m, "release") ? do_ring(true) : !strcmp(m, "udp") ? do_udp()
             : !strcmp(m, "tcp") ? do_tcp() : !strcmp(m, "plan") ? do_plan() : !strcmp(m, "ltable") ? do_ltable() : !strcmp(m, "utable") ? do_utable() : 2;
    fclose(g_out);
    fclose(g_in);
    return rc;
}
