// tcp_kernels.hip — established-state TCP receive processing on the GPU (include/dk_tcp.h).
//
// The reference queues each delivered segment on its socket (tcp/socket.rs:308-314, ctrlblk.rs:345-347) and
// ControlBlock::poll runs process_packet on them one at a time (ctrlblk.rs:350-440). Connections are independent;
// within one, order matters (RCV.NXT, the out-of-order store). For a whole dk_rx batch:
//   1. dk_tcp_key_kernel: frame -> key (its connection, for delivered TCP segments of a connection in the table; else
//      nconns) and value (its index); per-connection segment counts; default outputs;
//   2. an exclusive scan of the counts (each connection's range) and a stable radix sort of (key, index) over the key's
//      bits (hipCUB / rocPRIM): each connection's segments, contiguous, in arrival order;
//   3. dk_tcp_gather_kernel: the sorted segments' {seq, ack, meta, payload} into one contiguous array;
//   4. dk_tcp_walk_kernel: one lane per connection runs its segments through the state machine in order, kBatch
//      segments' fields loaded together. The walk is the only sequential part (latency-bound, lanes = connections);
//      everything else is a pass over the batch.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cerrno>

#include "../../include/dk_tcp.h"

namespace dk_tcp {
namespace {

constexpr uint32_t kBlock = 256;
constexpr uint32_t kBatch = 8;  // segments whose fields a walker lane loads together

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
    uint32_t* vals;
    uint32_t* skeys;
    uint32_t* svals;
    uint32_t* counts;
    uint32_t* seg_start;
    uint4* seg;  // sorted {seq, ack, meta, payload}
    dk_tcp_out out;
};

__global__ __launch_bounds__(kBlock) void dk_tcp_key_kernel(Params P) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= P.n) return;
    uint32_t key = P.nconns;
    if ((P.meta[i] & 0xFFu) == DK_V_OK_TCP) {
        const uint32_t f = P.flow_id[i];
        if (f < P.nconns && P.conns[f].state != DK_TCP_NONE) {
            key = f;
            atomicAdd(P.counts + f, 1u);
        }
    }
    P.keys[i] = key;
    P.vals[i] = i;
    P.out.action[i] = DK_TCP_SKIP;
    const uint32_t pay = P.payload[i];
    P.out.view[i] = dk_tcp_view{i, pay & 0xFFFFu, pay >> 16};
}

__global__ __launch_bounds__(kBlock) void dk_tcp_gather_kernel(Params P) {
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= P.n || P.skeys[p] >= P.nconns) return;
    const uint32_t i = P.svals[p];
    P.seg[p] = make_uint4(P.seq[i], P.ack[i], P.meta[i], P.payload[i]);
}

// One connection's scalar receive state, in registers during the walk (the store's entries stay in global memory).
struct Walk {
    uint32_t state, rn, reader, bufsz, snd, fin_pending, fin_seq, nooo;
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

__device__ void ooo_remove(dk_tcp_conn* s, Walk& w, uint32_t at) {
    for (uint32_t k = at; k + 1 < w.nooo; k++) {
        s->ooo_start[k] = s->ooo_start[k + 1];
        s->ooo[k] = s->ooo[k + 1];
    }
    w.nooo--;
}

// store_out_of_order_segment (ctrlblk.rs:844-941) on the fixed arrays.
__device__ __noinline__ uint32_t ooo_store(dk_tcp_conn* s, Walk& w, uint32_t new_start, uint32_t new_end,
                                           dk_tcp_view buf) {
    uint32_t at = w.nooo;
    bool again = true;
    while (again) {
        again = false;
        at = w.nooo;
        for (uint32_t i = 0; i < w.nooo; i++) {
            const uint32_t ss = s->ooo_start[i], se = ss + (s->ooo[i].len - 1);
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
    for (uint32_t k = min(w.nooo, DK_TCP_OOO_MAX - 1); k > at; k--) {
        s->ooo_start[k] = s->ooo_start[k - 1];
        s->ooo[k] = s->ooo[k - 1];
    }
    s->ooo_start[at] = new_start;
    s->ooo[at] = buf;
    w.nooo = min(w.nooo + 1, DK_TCP_OOO_MAX);
    return DK_TCP_STORED;
}

// receive_data (ctrlblk.rs:951-1001): true if a stored FIN is now in order.
__device__ __noinline__ bool receive_data(dk_tcp_conn* s, Walk& w, dk_tcp_view buf, Out& o) {
    uint32_t recv_next = w.rn + buf.len;
    o.push(buf, w);
    while (w.nooo > 0 && s->ooo_start[0] == recv_next) {
        const dk_tcp_view t = s->ooo[0];
        ooo_remove(s, w, 0);
        recv_next += t.len;
        o.push(t, w);
    }
    return w.fin_pending && w.fin_seq == recv_next;
}

// process_packet (ctrlblk.rs:403-440) for segment g = {seq, ack, meta, payload} of frame i.
__device__ __noinline__ uint32_t process(dk_tcp_conn* s, Walk& w, uint4 g, uint32_t i, Out& o, dk_tcp_view& view) {
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

__global__ __launch_bounds__(kBlock) void dk_tcp_walk_kernel(Params P) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= P.nconns) return;
    dk_tcp_conn* s = P.conns + c;
    const uint32_t k0 = P.seg_start[c], cnt = P.counts[c];
    const uint32_t d0 = k0 + DK_TCP_DELIV_EXTRA * c;
    P.out.deliv_start[c] = d0;
    Walk w{s->state, s->receive_next, s->reader_next, s->buffer_size, s->send_next, s->fin_pending, s->fin_seq,
           min(s->ooo_count, DK_TCP_OOO_MAX)};
    Out o{P.out.deliv + d0, 0, cnt + DK_TCP_DELIV_EXTRA};
    for (uint32_t k = 0; k < cnt; k += kBatch) {
        uint4 g[kBatch];
        uint32_t idx[kBatch];
#pragma unroll
        for (uint32_t j = 0; j < kBatch; j++) {
            if (k + j < cnt) {
                g[j] = P.seg[k0 + k + j];
                idx[j] = P.svals[k0 + k + j];
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < kBatch; j++) {
            if (k + j >= cnt) break;
            if (w.state != DK_TCP_ESTABLISHED) {
                P.out.action[idx[j]] = DK_TCP_UNPROCESSED;
                continue;
            }
            dk_tcp_view v;
            P.out.action[idx[j]] = (uint8_t)process(s, w, g[j], idx[j], o, v);
            P.out.view[idx[j]] = v;
        }
    }
    s->state = w.state;
    s->receive_next = w.rn;
    s->fin_pending = w.fin_pending;
    s->fin_seq = w.fin_seq;
    s->ooo_count = w.nooo;
    for (uint32_t k = w.nooo; k < DK_TCP_OOO_MAX; k++) {
        s->ooo_start[k] = 0;
        s->ooo[k] = dk_tcp_view{0, 0, 0};
    }
    P.out.deliv_count[c] = o.n;
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

struct dk_tcp_ctx {
    int device = 0;
    uint32_t *keys = nullptr, *vals = nullptr, *skeys = nullptr, *svals = nullptr;
    size_t keys_cap = 0, vals_cap = 0, skeys_cap = 0, svals_cap = 0;
    uint4* seg = nullptr;
    size_t seg_cap = 0;
    uint32_t *counts = nullptr, *seg_start = nullptr;
    size_t counts_cap = 0, start_cap = 0;
    uint8_t* temp = nullptr;
    size_t temp_cap = 0;
};

extern "C" {

int dk_tcp_ctx_create(int32_t device, dk_tcp_ctx** out) {
    if (!out) return EINVAL;
    *out = nullptr;
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || device < 0 || device >= nd) return EINVAL;
    dk_tcp_ctx* t = new dk_tcp_ctx();
    t->device = device;
    *out = t;
    return 0;
}

void dk_tcp_ctx_destroy(dk_tcp_ctx* t) {
    if (!t) return;
    dk_tcp::DeviceGuard g(t->device);
    for (void* p : {(void*)t->keys, (void*)t->vals, (void*)t->skeys, (void*)t->svals, (void*)t->seg, (void*)t->counts,
                    (void*)t->seg_start, (void*)t->temp})
        if (p) (void)hipFree(p);
    delete t;
}

int dk_tcp_rx_process(dk_tcp_ctx* t, const dk_rx_results* rx, uint32_t n, dk_tcp_conn* conns, uint32_t nconns,
                      const dk_tcp_out* out, void* stream) {
    using namespace dk_tcp;
    if (!t || !rx || !out) return EINVAL;
    if (n && (!rx->meta || !rx->flow_id || !rx->payload || !rx->tcp_seq || !rx->tcp_ack || !out->action || !out->view))
        return EINVAL;
    if (nconns && (!conns || !out->deliv || !out->deliv_start || !out->deliv_count)) return EINVAL;
    if (n > 0x7FFFFFFFu || nconns > 0x7FFFFFFFu ||
        (uint64_t)n + (uint64_t)DK_TCP_DELIV_EXTRA * nconns > 0xFFFFFFFFull)
        return EINVAL;
    if (n == 0 && nconns == 0) return 0;
    DeviceGuard g(t->device);
    const hipStream_t s = (hipStream_t)stream;
    int rc = 0;
    if ((rc = grow(t->keys, t->keys_cap, n)) || (rc = grow(t->vals, t->vals_cap, n)) ||
        (rc = grow(t->skeys, t->skeys_cap, n)) || (rc = grow(t->svals, t->svals_cap, n)) ||
        (rc = grow(t->seg, t->seg_cap, n)) || (rc = grow(t->counts, t->counts_cap, nconns)) ||
        (rc = grow(t->seg_start, t->start_cap, nconns)))
        return rc;
    int bits = 1;
    while (bits < 32 && (1ull << bits) <= nconns) bits++;  // keys are 0 .. nconns
    size_t sort_bytes = 0, scan_bytes = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, t->keys, t->skeys, t->vals, t->svals, (int)n, 0, bits,
                                           s) != hipSuccess ||
        hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, t->counts, t->seg_start, (int)nconns, s) != hipSuccess)
        return EINVAL;
    if ((rc = grow(t->temp, t->temp_cap, std::max(sort_bytes, scan_bytes)))) return rc;

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
    P.vals = t->vals;
    P.skeys = t->skeys;
    P.svals = t->svals;
    P.counts = t->counts;
    P.seg_start = t->seg_start;
    P.seg = t->seg;
    P.out = *out;
    if (nconns && hipMemsetAsync(t->counts, 0, nconns * sizeof(uint32_t), s) != hipSuccess) return EINVAL;
    const dim3 gn((n + kBlock - 1) / kBlock), gc((nconns + kBlock - 1) / kBlock);
    if (n) hipLaunchKernelGGL(dk_tcp_key_kernel, gn, dim3(kBlock), 0, s, P);
    if (nconns) {
        size_t b = t->temp_cap;
        if (hipcub::DeviceScan::ExclusiveSum(t->temp, b, t->counts, t->seg_start, (int)nconns, s) != hipSuccess)
            return EINVAL;
    }
    if (n) {
        size_t b = t->temp_cap;
        if (hipcub::DeviceRadixSort::SortPairs(t->temp, b, t->keys, t->skeys, t->vals, t->svals, (int)n, 0, bits, s) !=
            hipSuccess)
            return EINVAL;
        hipLaunchKernelGGL(dk_tcp_gather_kernel, gn, dim3(kBlock), 0, s, P);
    }
    if (nconns) hipLaunchKernelGGL(dk_tcp_walk_kernel, gc, dim3(kBlock), 0, s, P);
    return hipGetLastError() == hipSuccess ? 0 : EINVAL;
}

}  // extern "C"
