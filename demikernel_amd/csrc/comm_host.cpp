// comm_host.cpp — the receive path's one collective (dk_rx_flow_counts_allreduce, include/dk_rx.h) and the RCCL
// communicator bootstrap of include/dk_comm.h. Links the image's librccl (RCCL over xGMI between the GPUs of a node).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cerrno>
#include <cstring>

#include "../../include/dk_comm.h"
#include "rx_common.h"

static_assert(DK_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "dk_comm.h id size");

namespace {
int rc_of(ncclResult_t r) { return r == ncclSuccess ? 0 : (r == ncclInvalidArgument || r == ncclInvalidUsage) ? EINVAL : EIO; }
}  // namespace

extern "C" {

int dk_comm_unique_id(uint8_t id[DK_COMM_ID_BYTES]) {
    if (!id) return EINVAL;
    ncclUniqueId u;
    const int rc = rc_of(ncclGetUniqueId(&u));
    if (rc == 0) memcpy(id, u.internal, DK_COMM_ID_BYTES);
    return rc;
}

int dk_comm_init_rank(void** comm, int32_t nranks, const uint8_t id[DK_COMM_ID_BYTES], int32_t rank, int32_t device) {
    if (!comm || !id || nranks < 1 || rank < 0 || rank >= nranks) return EINVAL;
    *comm = nullptr;
    int prev = -1;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess) return EINVAL;
    ncclUniqueId u;
    memcpy(u.internal, id, DK_COMM_ID_BYTES);
    ncclComm_t c = nullptr;
    const int rc = rc_of(ncclCommInitRank(&c, nranks, u, rank));
    if (prev >= 0) (void)hipSetDevice(prev);
    if (rc == 0) *comm = c;
    return rc;
}

int dk_comm_init_all(void** comms, int32_t ndev, const int32_t* devices) {
    if (!comms || ndev < 1 || !devices) return EINVAL;
    static_assert(sizeof(ncclComm_t) == sizeof(void*), "opaque handle");
    return rc_of(ncclCommInitAll(reinterpret_cast<ncclComm_t*>(comms), ndev, devices));
}

int dk_comm_count(void* comm, int32_t* nranks) {
    if (!comm || !nranks) return EINVAL;
    int n = 0;
    const int rc = rc_of(ncclCommCount(static_cast<ncclComm_t>(comm), &n));
    *nranks = n;
    return rc;
}

int dk_comm_destroy(void* comm) {
    if (!comm) return EINVAL;
    return rc_of(ncclCommDestroy(static_cast<ncclComm_t>(comm)));
}

namespace {
int counts_allreduce(dk_rx_ctx* ctx, const dk_rx_results* res, uint64_t* flow_out, uint64_t* verdict_out,
                     void* nccl_comm, void* stream) {
    if (!ctx || !res || !nccl_comm) return EINVAL;
    const uint32_t nflows = dk_rx_flow_table_size(ctx);
    const ncclComm_t comm = static_cast<ncclComm_t>(nccl_comm);
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const bool flows = res->flow_counts && nflows, verdicts = res->verdict_counts != nullptr;
    if ((flows && !flow_out) || (verdicts && !verdict_out)) return EINVAL;
    if (!flows && !verdicts) return 0;
    int rc = rc_of(ncclGroupStart());
    if (rc) return rc;
    if (flows) rc = rc_of(ncclAllReduce(res->flow_counts, flow_out, nflows, ncclUint64, ncclSum, comm, s));
    if (rc == 0 && verdicts)
        rc = rc_of(ncclAllReduce(res->verdict_counts, verdict_out, DK_V_COUNT, ncclUint64, ncclSum, comm, s));
    const int rc2 = rc_of(ncclGroupEnd());
    return rc ? rc : rc2;
}
}  // namespace

int dk_rx_flow_counts_allreduce(dk_rx_ctx* ctx, const dk_rx_results* res, void* nccl_comm, void* stream) {
    return res ? counts_allreduce(ctx, res, res->flow_counts, res->verdict_counts, nccl_comm, stream) : EINVAL;
}

int dk_rx_flow_counts_allreduce_to(dk_rx_ctx* ctx, const dk_rx_results* res, uint64_t* flow_out,
                                   uint64_t* verdict_out, void* nccl_comm, void* stream) {
    return counts_allreduce(ctx, res, flow_out, verdict_out, nccl_comm, stream);
}

}  // extern "C"
