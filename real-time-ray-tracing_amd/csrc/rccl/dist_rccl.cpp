// dist_rccl.cpp — include/rtx_dist_rccl.h: the rtd_comm of include/rtx_dist.h over RCCL (built as
// lib/librtx_rccl.so so that librtx.so itself does not depend on librccl).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include "rtx_dist_rccl.h"

namespace {

ncclComm_t as_comm(void* p) { return (ncclComm_t)p; }

int all_gather(void* arg, const void* send, void* recv, size_t bytes, void* stream) {
    return ncclAllGather(send, recv, bytes, ncclUint8, as_comm(arg), (hipStream_t)stream) == ncclSuccess ? 0 : 1;
}

int all_reduce_sum_i32(void* arg, int32_t* buf, size_t count, void* stream) {
    return ncclAllReduce(buf, buf, count, ncclInt32, ncclSum, as_comm(arg), (hipStream_t)stream) == ncclSuccess ? 0 : 1;
}

int all_to_allv(void* arg, const void* send, const size_t* send_bytes, const size_t* send_offsets, void* recv,
                const size_t* recv_bytes, const size_t* recv_offsets, void* stream) {
    ncclComm_t c = as_comm(arg);
    int world = 0;
    if (ncclCommCount(c, &world) != ncclSuccess) return 1;
    hipStream_t s = (hipStream_t)stream;
    if (ncclGroupStart() != ncclSuccess) return 1;
    ncclResult_t e = ncclSuccess;
    for (int r = 0; r < world && e == ncclSuccess; ++r) {
        if (send_bytes[r]) e = ncclSend((const char*)send + send_offsets[r], send_bytes[r], ncclUint8, r, c, s);
        if (e == ncclSuccess && recv_bytes[r])
            e = ncclRecv((char*)recv + recv_offsets[r], recv_bytes[r], ncclUint8, r, c, s);
    }
    const ncclResult_t g = ncclGroupEnd();
    return e == ncclSuccess && g == ncclSuccess ? 0 : 1;
}

}  // namespace

extern "C" {

int rtd_rccl_get_unique_id(void* id128) {
    if (!id128) return RT_ERR_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return RT_ERR_HIP;
    memcpy(id128, &id, sizeof(id));
    return RT_OK;
}

int rtd_rccl_comm_init(int world, int rank, const void* id128, void** nccl_comm) {
    if (!id128 || !nccl_comm || world < 1 || rank < 0 || rank >= world) return RT_ERR_ARG;
    ncclUniqueId id;
    memcpy(&id, id128, sizeof(id));
    ncclComm_t c = nullptr;
    if (ncclCommInitRank(&c, world, id, rank) != ncclSuccess) return RT_ERR_HIP;
    *nccl_comm = c;
    return RT_OK;
}

void rtd_rccl_comm_destroy(void* nccl_comm) {
    if (nccl_comm) ncclCommDestroy(as_comm(nccl_comm));
}

int rtd_comm_rccl(void* nccl_comm, rtd_comm* out) {
    if (!nccl_comm || !out) return RT_ERR_ARG;
    memset(out, 0, sizeof(*out));
    out->arg = nccl_comm;
    out->all_gather = all_gather;
    out->all_reduce_sum_i32 = all_reduce_sum_i32;
    out->all_to_allv = all_to_allv;
    return RT_OK;
}

}  // extern "C"
