/* dk_demi.h — the demi_pop side of the drop-in: delivered frames of a dk_rx batch as Demikernel scatter-gather arrays.
 *
 * The receive path replaces the stack below the socket queues; what the application sees is unchanged. A popped
 * buffer reaches the application as a demi_sgarray_t built by MemoryRuntime::into_sgarray
 * (src/rust/runtime/memory/mod.rs:38-54: one segment over the stripped DemiBuffer, sga_buf = the buffer's token,
 * sga_addr zeroed), and NetworkLibOS::pack_result (src/rust/demikernel/libos/network/libos.rs:495-499) sets sga_addr
 * from the popped address when the queue returns one — UDP pops return the remote (src_ip, sport)
 * (udp/peer.rs:167 queues it with the datagram), TCP pops return none. The stripped buffer is the dk_rx payload
 * window: frame base + payload offset, payload length (what DemiBuffer::adjust/trim leave, demibuffer.rs:515-590).
 *
 * The types below have exactly the layout of include/demi/types.h:38-68 (packed; 12 and 40 bytes, the sizes
 * tests/c/sizes.c:48-68 asserts), so a LibOS can pass its own demi_sgarray_t storage.
 *
 * Host-side, no GPU work: it reads results the caller has copied back (or mapped) and never touches frame bytes.
 */
#ifndef DK_DEMI_H
#define DK_DEMI_H

#include <netinet/in.h>
#include <stdint.h>

#include "dk_rx.h"
#include "dk_tcp.h"

#ifdef __cplusplus
extern "C" {
#endif

#define DK_DEMI_SGARRAY_MAXSIZE 1 /* DEMI_SGARRAY_MAXSIZE, include/demi/types.h:28 */

typedef struct __attribute__((__packed__)) dk_demi_sgaseg {
    void* sgaseg_buf;    /* payload bytes */
    uint32_t sgaseg_len; /* payload length */
} dk_demi_sgaseg_t;

typedef struct __attribute__((__packed__)) dk_demi_sgarray {
    void* sga_buf;        /* buffer token (the reference: the DemiBuffer's raw pointer, demi_sgafree's argument) */
    uint32_t sga_numsegs; /* 1 */
    dk_demi_sgaseg_t sga_segs[DK_DEMI_SGARRAY_MAXSIZE];
    struct sockaddr_in sga_addr; /* UDP: remote address (AF_INET, network-order port and address); TCP: zero */
} dk_demi_sgarray_t;

/* UDP pops: builds the scatter-gather arrays demi_pop would hand out for the delivered datagrams (verdict
 * DK_V_OK_UDP) of a batch, in frame order (UdpPeer::receive queues each datagram whole, udp/peer.rs:167). Delivered
 * TCP frames (DK_V_OK_TCP) are skipped: a TCP pop returns what the connection's ControlBlock pushed to its receive
 * queue after the in-window checks and reordering, not frames — use dk_tcp_into_sgarrays on dk_tcp_rx_process's
 * output for those. Inputs are host-resident: the frame blob base (host or mapped pointer;
 * only addresses are formed), the batch's u32 offsets, and the dk_rx result words meta, src_ip, ports and payload
 * of n frames. tokens (nullable): per-frame buffer tokens for sga_buf (e.g. the mbuf each frame came in); NULL puts
 * the frame's own address there. Writes at most cap arrays to out and, when frame_idx is not NULL, the frame index
 * of each; *nout = number written. Returns 0, EINVAL (NULL required pointer), or ENOSPC when more than cap frames
 * were delivered (out holds the first cap; *nout = cap). */
int dk_rx_into_sgarrays(const uint8_t* frames, const uint32_t* off, uint32_t n, const uint32_t* meta,
                        const uint32_t* src_ip, const uint32_t* ports, const uint32_t* payload,
                        void* const* tokens, dk_demi_sgarray_t* out, uint32_t* frame_idx, uint32_t cap,
                        uint32_t* nout);

/* TCP pops: the buffers one dk_tcp_rx_process call pushed to ONE connection's receive queue (its dk_tcp_out.deliv
 * entries deliv[deliv_start[c] .. + deliv_count[c]), copied to host), in queue order, one demi_sgarray_t each — what
 * ControlBlock::pop(None) (tcp/established/ctrlblk.rs:823, Receiver::pop :113-130) returns buffer by buffer, packed by
 * into_sgarray: one segment of view.len bytes at frame view.ref's base (frames + off[view.ref]) + view.off, sga_buf =
 * tokens[view.ref] (NULL tokens: the frame's address), sga_addr zero (TCP pops carry no address). The EOF buffer
 * (view.ref == DK_TCP_REF_EOF: process_remote_close's DemiBuffer::new(0), ctrlblk.rs:1008) is one zero-length segment
 * with sga_buf and sgaseg_buf NULL. View refs index this batch's frames (0 .. n). Writes at most cap arrays;
 * *nout = number written. Returns 0, EINVAL (NULL required pointer, ref >= n) or ENOSPC (out holds the first cap). */
int dk_tcp_into_sgarrays(const uint8_t* frames, const uint32_t* off, uint32_t n, const dk_tcp_view* deliv,
                         uint32_t count, void* const* tokens, dk_demi_sgarray_t* out, uint32_t cap, uint32_t* nout);

#ifdef __cplusplus
}
#endif

#endif /* DK_DEMI_H */
