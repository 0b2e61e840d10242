/* rtx_dist_rccl.h — an RCCL communicator for include/rtx_dist.h (lib/librtx_rccl.so, links librccl).
 * A host without a communicator of its own creates one per rank and plugs it into rtd_create:
 *
 *     char id[128];  if (rank == 0) rtd_rccl_get_unique_id(id);  ... broadcast id out of band ...
 *     void* nc;  rtd_rccl_comm_init(world, rank, id, &nc);     // after hipSetDevice(local rank)
 *     rtd_comm comm;  rtd_comm_rccl(nc, &comm);
 *     rtd_create(W, H, world, rank, &comm, &s);  rtd_attach(s, ctx);
 *
 * The collectives run on the stream the renderer passes (the denoise's): ncclAllGather,
 * ncclAllReduce(ncclSum, int32), and the all-to-allv as grouped ncclSend / ncclRecv — one message
 * per peer over its own xGMI link on an 8-GPU MI355X node.  Status codes: 0 / RT_ERR_*. */
#ifndef RTX_DIST_RCCL_H
#define RTX_DIST_RCCL_H

#include "rtx_dist.h"

#ifdef __cplusplus
extern "C" {
#endif

int rtd_rccl_get_unique_id(void* id128);
int rtd_rccl_comm_init(int world, int rank, const void* id128, void** nccl_comm);
void rtd_rccl_comm_destroy(void* nccl_comm);
/* fills `out` with RCCL collectives over nccl_comm (an ncclComm_t); copy2d / alloc / release stay
 * NULL (the library's HIP defaults) */
int rtd_comm_rccl(void* nccl_comm, rtd_comm* out);

#ifdef __cplusplus
}
#endif

#endif /* RTX_DIST_RCCL_H */
