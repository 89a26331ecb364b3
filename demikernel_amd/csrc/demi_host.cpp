// demi_host.cpp — dk_rx results -> demi_sgarray_t (include/dk_demi.h): what MemoryRuntime::into_sgarray
// (runtime/memory/mod.rs:38-54) and NetworkLibOS::pack_result (demikernel/libos/network/libos.rs:495-499) build for a
// popped buffer, for every delivered frame of a batch. Host code only.
#include <errno.h>
#include <string.h>

#include "../../include/dk_demi.h"

static_assert(sizeof(dk_demi_sgaseg_t) == 12, "demi_sgaseg_t is 12 bytes (tests/c/sizes.c)");
static_assert(sizeof(dk_demi_sgarray_t) == 40, "demi_sgarray_t is 40 bytes (tests/c/sizes.c)");

extern "C" int dk_rx_into_sgarrays(const uint8_t* frames, const uint32_t* off, uint32_t n, const uint32_t* meta,
                                   const uint32_t* src_ip, const uint32_t* ports, const uint32_t* payload,
                                   void* const* tokens, dk_demi_sgarray_t* out, uint32_t* frame_idx, uint32_t cap,
                                   uint32_t* nout) {
    if (!nout) return EINVAL;
    *nout = 0;
    if (n == 0) return 0;
    if (!frames || !off || !meta || !src_ip || !ports || !payload || (cap && !out)) return EINVAL;
    uint32_t k = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t v = meta[i] & 0xFFu;
        if (v != DK_V_OK_UDP) continue;  // TCP pops come from the connection's receive queue: dk_tcp_into_sgarrays
        if (k == cap) {
            *nout = k;
            return ENOSPC;
        }
        dk_demi_sgarray_t& s = out[k];
        memset(&s, 0, sizeof s);  // sga_addr: mem::zeroed() unless the pop carries an address
        const uint8_t* f = frames + off[i];
        s.sga_buf = tokens ? tokens[i] : const_cast<uint8_t*>(f);
        s.sga_numsegs = 1;
        s.sga_segs[0].sgaseg_buf = const_cast<uint8_t*>(f + (payload[i] & 0xFFFFu));
        s.sga_segs[0].sgaseg_len = payload[i] >> 16;
        // socketaddrv4_to_sockaddr (pal/mod.rs:154-160) of the datagram's remote address
        struct sockaddr_in a;
        memset(&a, 0, sizeof a);
        a.sin_family = AF_INET;
        a.sin_port = htons((uint16_t)(ports[i] & 0xFFFFu));  // src port (host order in the results)
        a.sin_addr.s_addr = src_ip[i];                       // already network order (frame bytes)
        memcpy(&s.sga_addr, &a, sizeof a);
        if (frame_idx) frame_idx[k] = i;
        k++;
    }
    *nout = k;
    return 0;
}

extern "C" int dk_tcp_into_sgarrays(const uint8_t* frames, const uint32_t* off, uint32_t n, const dk_tcp_view* deliv,
                                    uint32_t count, void* const* tokens, dk_demi_sgarray_t* out, uint32_t cap,
                                    uint32_t* nout) {
    if (!nout) return EINVAL;
    *nout = 0;
    if (count == 0) return 0;
    if (!deliv || (cap && !out)) return EINVAL;
    for (uint32_t k = 0; k < count; k++) {
        const dk_tcp_view& v = deliv[k];
        if (v.ref != DK_TCP_REF_EOF && (v.ref >= n || !frames || !off)) return EINVAL;
    }
    for (uint32_t k = 0; k < count; k++) {
        if (k == cap) {
            *nout = k;
            return ENOSPC;
        }
        const dk_tcp_view& v = deliv[k];
        dk_demi_sgarray_t& s = out[k];
        memset(&s, 0, sizeof s);  // sga_addr: TCP pops carry none (mem::zeroed(), runtime/memory/mod.rs:52)
        s.sga_numsegs = 1;
        if (v.ref != DK_TCP_REF_EOF) {
            const uint8_t* f = frames + off[v.ref];
            s.sga_buf = tokens ? tokens[v.ref] : const_cast<uint8_t*>(f);
            s.sga_segs[0].sgaseg_buf = const_cast<uint8_t*>(f + v.off);
            s.sga_segs[0].sgaseg_len = v.len;
        }
    }
    *nout = count;
    return 0;
}
