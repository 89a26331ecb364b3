// TEST INFRASTRUCTURE ONLY: driver for the ASan/UBSan build of the oracle (oracle/Makefile: dk_oracle_asan).
// Reads a batch file and writes the result arrays, so tests can run the restatement under host sanitizers.
//   input:  u32 n | u64 blob_len | u32 local_ip | u32 tcp_offload | u32 udp_offload | u32 nflows |
//           flows[nflows] (dk_flow) | off[n] (u32) | len[n] (u16) | blob[blob_len]
//   output: meta, src_ip, dst_ip, ports, payload, flow_id, tcp_seq, tcp_ack, tcp_win (u32[n] each),
//           flow_counts (u64[max(nflows,1)]), verdict_counts (u64[DK_V_COUNT])
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/dk_rx.h"

extern "C" {
struct dko_peer;
dko_peer* dko_peer_new(uint32_t local_ipv4, int tcp_offload, int udp_offload);
void dko_peer_free(dko_peer* p);
int dko_peer_set_flows(dko_peer* p, const dk_flow* flows, uint32_t n);
void dko_process(const dko_peer* p, const uint8_t* frames, uint64_t frames_bytes, const uint32_t* off,
                 const uint16_t* len, uint32_t n, uint32_t* meta, uint32_t* src, uint32_t* dst, uint32_t* ports,
                 uint32_t* payload, uint32_t* flow, uint32_t* seq, uint32_t* ack, uint32_t* win,
                 uint64_t* flow_counts, uint64_t* verdict_counts, dk_tcp_opts* opts);
}

template <class T>
static void rd(FILE* f, T* p, size_t n) {
    if (n && fread(p, sizeof(T), n, f) != n) {
        fprintf(stderr, "short read\n");
        exit(2);
    }
}

int main(int argc, char** argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: %s in.bin out.bin\n", argv[0]);
        return 2;
    }
    FILE* in = fopen(argv[1], "rb");
    if (!in) return 2;
    uint32_t n, lip, to, uo, nf;
    uint64_t blob_len;
    rd(in, &n, 1);
    rd(in, &blob_len, 1);
    rd(in, &lip, 1);
    rd(in, &to, 1);
    rd(in, &uo, 1);
    rd(in, &nf, 1);
    std::vector<dk_flow> flows(nf);
    rd(in, flows.data(), nf);
    std::vector<uint32_t> off(n);
    std::vector<uint16_t> len(n);
    rd(in, off.data(), n);
    rd(in, len.data(), n);
    // Exactly blob_len bytes on the heap: ASan flags any read past the blob.
    uint8_t* blob = (uint8_t*)malloc(blob_len ? blob_len : 1);
    rd(in, blob, blob_len);
    fclose(in);
    dko_peer* p = dko_peer_new(lip, (int)to, (int)uo);
    if (dko_peer_set_flows(p, flows.data(), nf)) return 3;
    std::vector<uint32_t> a[9];
    for (auto& v : a) v.assign(n, 0);
    std::vector<uint64_t> fc(nf ? nf : 1, 0), vc(DK_V_COUNT, 0);
    std::vector<dk_tcp_opts> opts(n ? n : 1);
    dko_process(p, blob, blob_len, off.data(), len.data(), n, a[0].data(), a[1].data(), a[2].data(), a[3].data(),
                a[4].data(), a[5].data(), a[6].data(), a[7].data(), a[8].data(), fc.data(), vc.data(), opts.data());
    FILE* out = fopen(argv[2], "wb");
    if (!out) return 2;
    for (auto& v : a) fwrite(v.data(), 4, n, out);
    fwrite(fc.data(), 8, fc.size(), out);
    fwrite(vc.data(), 8, vc.size(), out);
    fclose(out);
    dko_peer_free(p);
    free(blob);
    return 0;
}
