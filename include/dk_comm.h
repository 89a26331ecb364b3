/*
 * dk_comm.h — RCCL communicator bootstrap for packet-sharded receive across the GPUs of a node.
 *
 * The receive path shards by packet: every GPU runs dk_rx_process on its own frames with a replica of the socket
 * table, and the only exchange is the sum of the per-flow / per-verdict counters (dk_rx_flow_counts_allreduce in
 * dk_rx.h, one grouped ncclAllReduce over RCCL / xGMI). The reference has no counterpart: it is one single-threaded
 * LibOS per process (demikernel/bindings.rs:33-35) with no drop counters (layer2/mod.rs:62 "TODO: Collect dropped packet
 * statistics"); the per-flow key being summed is its SocketId (layer4/tcp/peer.rs:241-251).
 *
 * These calls only wrap the image's librccl so a LibOS can build communicators without a Python or torch process
 * group: rank 0 creates the id, ships its DK_COMM_ID_BYTES bytes to the other ranks by any channel, and every rank
 * joins. Communicators are opaque `void*` (an ncclComm_t). Conventions as dk_rx.h: 0 or a positive errno (EINVAL bad
 * argument, EIO any RCCL failure).
 */
#ifndef DK_COMM_H
#define DK_COMM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DK_COMM_ID_BYTES 128 /* NCCL_UNIQUE_ID_BYTES */

/* ncclGetUniqueId: the bootstrap id of a new communicator (rank 0 calls it). */
int dk_comm_unique_id(uint8_t id[DK_COMM_ID_BYTES]);

/* ncclCommInitRank on `device`: blocks until all nranks ranks have joined with the same id. */
int dk_comm_init_rank(void** comm, int32_t nranks, const uint8_t id[DK_COMM_ID_BYTES], int32_t rank, int32_t device);

/* ncclCommInitAll: ndev communicators of one process, comms[k] on devices[k] (single-process tests and tools). */
int dk_comm_init_all(void** comms, int32_t ndev, const int32_t* devices);

/* ncclCommCount. */
int dk_comm_count(void* comm, int32_t* nranks);

/* ncclCommDestroy. */
int dk_comm_destroy(void* comm);

#ifdef __cplusplus
}
#endif

#endif /* DK_COMM_H */
