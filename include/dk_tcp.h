/*
 * dk_tcp.h — established-state TCP receive processing on the GPU: the sequence-space checks
 * and per-connection in-order delivery that ControlBlock::poll runs on every segment TcpPeer::receive queued for an
 * established socket (tcp/socket.rs:308-314 -> tcp/established/ctrlblk.rs:345-440), for a whole dk_rx batch at once.
 *
 * Per segment, in arrival order within each connection (paths relative to /root/reference/src/rust/inetstack/
 * protocols/layer4/tcp/):
 *   check_segment_in_window   established/ctrlblk.rs:447-567  duplicate / out-of-window drops, front and end trims
 *   check_rst, check_syn      :570-604
 *   process_ack               :607-650   only the ack_num <= SND.NXT test (the send side is not modelled)
 *   process_data              :652-695   in order -> receive_data (:951-1001, also recovers stored segments),
 *                                        else the out-of-order store (:836-941, MAX_OUT_OF_ORDER_SIZE_FRAMES = 16)
 *   process_remote_close      :1003-1024 FIN: EOF buffer, RCV.NXT + 1, the connection stops processing
 * SeqNumber comparisons are sequence_number.rs:76-101 (sign of the wrapping difference). Reference quirks are kept:
 * the end-overlap adjust of the out-of-order store is one byte short (ctrlblk.rs:916), a front-overlapping segment is
 * inserted at the back of the store (ctrlblk.rs:891-899 leave action_index at the end), a FIN-only in-order segment
 * pushes an empty buffer before the EOF buffer (ctrlblk.rs:693 + :1008).
 * Not modelled: the delayed-ACK timer and the ACKs segments trigger, the sender (SND.UNA, RTO, congestion control),
 * states other than ESTABLISHED (FIN-WAIT-1/2 etc.).
 *
 * Conventions as dk_rx.h: 0 or a positive errno; device pointers; asynchronous on the caller's stream. A context holds
 * one set of scratch buffers: calls on one context are serialised — a call on another stream than the previous call
 * first waits (on the device) for the previous call's work — so use one context per stream for concurrent batches.
 * The engine picks its per-connection walk from the batch (one lane per connection; one wave per connection at
 * >= 8 segments per connection; at >= 1,024 segments per connection and <= 256 connections the scan walk: windows
 * precomputed across the chip, 64 windows per wave scan per connection, the rest in parallel); the diagnostic
 * dk_diag_tcp_set_walk (dk_diag.h) forces one (relay: 8 waves per connection passing its state window to window).
 * The environment is never read. Results are identical.
 */
#ifndef DK_TCP_H
#define DK_TCP_H

#include <stdint.h>

#include "dk_rx.h"

#ifdef __cplusplus
extern "C" {
#endif

#define DK_TCP_OOO_MAX 16u          /* MAX_OUT_OF_ORDER_SIZE_FRAMES (ctrlblk.rs:53)                              */
#define DK_TCP_DELIV_EXTRA 18u      /* delivery slots per connection beyond its segment count (stored + 2 EOF)   */
#define DK_TCP_REF_EOF 0xFFFFFFFFu  /* dk_tcp_view.ref of the empty EOF buffer process_remote_close pushes       */

enum dk_tcp_state {
    DK_TCP_NONE = 0,        /* not a connection: its frames are left alone (DK_TCP_SKIP)                          */
    DK_TCP_ESTABLISHED = 1,
    DK_TCP_CLOSED = 2       /* after RST or FIN: ControlBlock::poll has returned (ctrlblk.rs:381-396)             */
};

/* A DemiBuffer view: `len` bytes at byte `off` of frame `ref` (the frame's index in the dk_rx batch it came in, or
 * whatever the caller keeps in state carried between batches; DK_TCP_REF_EOF for the EOF buffer). */
typedef struct dk_tcp_view {
    uint32_t ref;
    uint32_t off;
    uint32_t len;
} dk_tcp_view;

/* Receive side of one connection's ControlBlock (ctrlblk.rs:145-220), indexed by the flow_id dk_rx gives its frames. */
typedef struct dk_tcp_conn {
    uint32_t state;         /* enum dk_tcp_state                                                                   */
    uint32_t receive_next;  /* RCV.NXT, Receiver::receive_next (ctrlblk.rs:98)                                     */
    uint32_t reader_next;   /* Receiver::reader_next (ctrlblk.rs:95); window = buffer_size - (RCV.NXT - reader_next) */
    uint32_t buffer_size;   /* receive_buffer_size_frames (ctrlblk.rs:191)                                         */
    uint32_t send_next;     /* SND.NXT, for process_ack's ack_num <= SND.NXT (ctrlblk.rs:623-633)                  */
    uint32_t fin_pending;   /* receive_out_of_order_fin is Some (ctrlblk.rs:220)                                   */
    uint32_t fin_seq;
    uint32_t ooo_count;     /* receive_out_of_order_frames (ctrlblk.rs:208), in store order; entries past the count
                               are zero                                                                            */
    uint32_t ooo_start[DK_TCP_OOO_MAX];
    dk_tcp_view ooo[DK_TCP_OOO_MAX];
} dk_tcp_conn;              /* 288 bytes */

enum dk_tcp_action {
    DK_TCP_SKIP = 0,           /* not a delivered TCP segment of a connection in the table                        */
    DK_TCP_DELIVERED = 1,      /* in order: pushed to the receive queue (with any stored segments it unblocked)   */
    DK_TCP_STORED = 2,         /* out of order: kept for later (data and/or FIN)                                  */
    DK_TCP_STORE_DUP = 3,      /* out of order, inside stored data: dropped (ctrlblk.rs:903-908)                  */
    DK_TCP_NO_DATA = 4,        /* acceptable, no data and no FIN                                                  */
    DK_TCP_FIN = 5,            /* FIN reached in order: EOF pushed, connection closes (ECONNRESET, :1003-1024)    */
    DK_TCP_DUPLICATE = 6,      /* entirely old (ctrlblk.rs:495-504)                              EBADMSG          */
    DK_TCP_OUT_OF_WINDOW = 7,  /* starts at or beyond the window end (ctrlblk.rs:525-535)        EBADMSG          */
    DK_TCP_RST = 8,            /* reset (ctrlblk.rs:570-583): connection closes                  ECONNRESET       */
    DK_TCP_SYN = 9,            /* in-window SYN (ctrlblk.rs:586-604)                             EBADMSG          */
    DK_TCP_NO_ACK = 10,        /* ACK bit clear (ctrlblk.rs:608-613)                             EBADMSG          */
    DK_TCP_ACK_UNSENT = 11,    /* acknowledges beyond SND.NXT (ctrlblk.rs:640-647)               EBADMSG          */
    DK_TCP_UNPROCESSED = 12    /* queued behind the close: never processed (ctrlblk.rs:355-363)                   */
};

/* Outputs of one call (device arrays). action, view: [n], per frame of the batch; view = the segment's data after
 * check_segment_in_window's adjust/trim (the payload as dk_rx gave it for frames that are dropped before or never
 * processed). deliv: the buffers pushed to each connection's receive queue, in order: connection c's are
 * deliv[deliv_start[c] .. deliv_start[c] + deliv_count[c]), where the engine sets deliv_start[c] = (segments of
 * connections < c) + DK_TCP_DELIV_EXTRA * c; deliv must hold n + DK_TCP_DELIV_EXTRA * nconns entries. */
typedef struct dk_tcp_out {
    uint8_t* action;
    dk_tcp_view* view;
    dk_tcp_view* deliv;
    uint32_t* deliv_start;  /* [nconns] */
    uint32_t* deliv_count;  /* [nconns] */
} dk_tcp_out;

typedef struct dk_tcp_ctx dk_tcp_ctx;

/* Scratch (sort buffers) for dk_tcp_rx_process on `device`. Returns 0 or EINVAL. */
int dk_tcp_ctx_create(int32_t device, dk_tcp_ctx** out);
void dk_tcp_ctx_destroy(dk_tcp_ctx* ctx);

/* Run the TCP segments of one dk_rx_process batch through their connections: rx = that call's device results (meta,
 * flow_id, payload, tcp_seq and tcp_ack are required), conns[0 .. nconns) = the connections by flow_id (device,
 * 16-byte aligned as hipMalloc returns it, updated in place). Asynchronous on `stream`. Returns 0, EINVAL (also for a
 * misaligned conns) or ENOMEM. */
int dk_tcp_rx_process(dk_tcp_ctx* ctx, const dk_rx_results* rx, uint32_t n, dk_tcp_conn* conns, uint32_t nconns,
                      const dk_tcp_out* out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DK_TCP_H */
