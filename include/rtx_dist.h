/* rtx_dist.h — the multi-GPU screen split for hosts that are not Python: the C-ABI
 * counterpart of rtx/dist.py (StripGather + StripDenoise), in librtx.so, over a communicator the
 * host plugs in (RCCL on a real node: ncclAllGather / ncclAllReduce / grouped ncclSend+ncclRecv;
 * INTEGRATION.md §3 shows the adapter).
 *
 * The reference renders on one GPU (RayTracer::draw, kernel.cu:259-398); this is the layer a
 * multi-GPU host adds around the same draw call.  One process per GPU; every rank creates its
 * context with [render] stripCount = world, stripIndex = rank, then
 *
 *     rtd_create(W, H, world, rank, &comm, &s);
 *     rtd_attach(s, ctx);              // binds full-frame buffers, installs rtd_hook (3 stages)
 *     for (;;) rt_draw_device(ctx, target, pitch, 0);   // or rt_draw / rt_path_trace + rt_denoise_post
 *
 * Per frame the renderer then calls the hook three times on the stream the denoise runs on:
 *   RT_HOOK_GBUFFERS   before the denoise: every rank's path-traced 16-row blocks of the five
 *                      G-buffers to the ranks whose denoise reads them (all-to-all of the rows
 *                      rt_info.gbufferRowBegin/End names per rank; the whole frame = all-gather when
 *                      the denoise is not strip-local),
 *   RT_HOOK_HISTOGRAM  the 64-bin histogram all-reduce (strip-local denoise only),
 *   RT_HOOK_ROWS       the accumulation / history / RGBA8 rows of every rank's strip, all-gathered,
 * so every rank ends the frame holding the single-GPU frame bit for bit (RGBA8, final HDR, state).
 *
 * Layout (the renderer's own rules, bvh_kernels.h): 16-row trace blocks dealt round-robin (block b
 * belongs to rank b mod world), full-frame G-buffers padded to ceil(ceil(H/16)/world)*world*16 rows,
 * contiguous 64-row denoise strips, 5 tiles of G-buffer halo.  Status codes are RT_OK / RT_ERR_*.
 */
#ifndef RTX_DIST_H
#define RTX_DIST_H

#include <stddef.h>
#include <stdint.h>

#include "rtx_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The communicator.  Collectives are enqueued on `stream` (a hipStream_t) and return 0 on success.
 * Buffers are the library's staging memory (alloc) and the bound device buffers. */
typedef struct rtd_comm {
    void* arg;
    /* every rank's `bytes` of send, rank-major into recv (world * bytes) */
    int (*all_gather)(void* arg, const void* send, void* recv, size_t bytes, void* stream);
    /* in-place sum over the ranks of `count` int32 */
    int (*all_reduce_sum_i32)(void* arg, int32_t* buf, size_t count, void* stream);
    /* send_bytes[r] bytes at send + send_offsets[r] to rank r; recv_bytes[r] bytes from rank r at
     * recv + recv_offsets[r] (entries for this rank are 0) */
    int (*all_to_allv)(void* arg, const void* send, const size_t* send_bytes, const size_t* send_offsets, void* recv,
                       const size_t* recv_bytes, const size_t* recv_offsets, void* stream);
    /* rank-local copy of `height` rows of `width` bytes; NULL: hipMemcpy2DAsync on the stream */
    int (*copy2d)(void* arg, void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t height,
                  void* stream);
    /* staging memory; NULL: hipMalloc / hipFree */
    void* (*alloc)(void* arg, size_t bytes);
    void (*release)(void* arg, void* p);
} rtd_comm;

typedef struct rtd_strips rtd_strips;

int rtd_create(int width, int height, int world, int rank, const rtd_comm* comm, rtd_strips** out);
void rtd_destroy(rtd_strips* s); /* frees staging and attached buffers (after the context is destroyed) */
const char* rtd_last_error(const rtd_strips* s);

/* layout queries */
int rtd_denoise_rows(const rtd_strips* s, int rank, int32_t* begin, int32_t* end);  /* strip-local denoise rows */
int rtd_gbuffer_rows(const rtd_strips* s, int rank, int32_t* begin, int32_t* end);  /* rows that denoise reads */
size_t rtd_gbuffer_bytes(const rtd_strips* s, int name);  /* padded full-frame bytes of a G-buffer (RT_BUF_*) */
/* bytes this rank receives per frame: stage RT_HOOK_GBUFFERS (strip_local 1: strip exchange, 0: the
 * whole frame), RT_HOOK_ROWS, RT_HOOK_HISTOGRAM */
size_t rtd_recv_bytes(const rtd_strips* s, int stage, int strip_local);

/* The exchanges on caller buffers (full-frame, row-major, padded G-buffers as rtd_gbuffer_bytes). */
typedef struct rtd_gbuffers {
    void* color;   /* RT_BUF_RENDER_COLOR, 8 B/px */
    void* normal;  /* RT_BUF_NORMAL, 8 */
    void* albedo;  /* RT_BUF_ALBEDO, 8 */
    void* depth;   /* RT_BUF_DEPTH, 2 */
    void* motion;  /* RT_BUF_MOTION, 4 */
} rtd_gbuffers;
int rtd_exchange_gbuffers(rtd_strips* s, const rtd_gbuffers* g, int strip_local, void* stream);
int rtd_exchange_histogram(rtd_strips* s, int32_t* histogram, void* stream);
/* this rank's denoise rows of the accumulation (8 B/px), history (8 B/px) and RGBA8 (4 B/px) buffers
 * to every rank */
int rtd_exchange_rows(rtd_strips* s, void* accum, void* history, void* rgba, void* stream);

/* Allocate (hipMalloc) and bind (rt_bind_buffer) the full-frame buffers the exchanges move — the
 * G-buffers of all RT_GBUFFER_SETS G-buffer sets, accumulation, both history buffers, histogram, RGBA8 — and
 * install rtd_hook for RT_HOOK_GBUFFERS, RT_HOOK_HISTOGRAM and RT_HOOK_ROWS (rt_set_hook_stages).
 * ctx must be an inited context of this rank's strip (stripCount = world, stripIndex = rank).
 * On failure the buffers bound before the failing step stay bound to ctx and are owned by s: the
 * context must then not render again — destroy it (rt_destroy), then the strips (rtd_destroy). */
int rtd_attach(rtd_strips* s, rt_context* ctx);
/* the rt_collective_fn rtd_attach installs (arg = the rtd_strips) */
int rtd_hook(void* arg, int stage, void* stream, const rt_strip_exchange* x);

#ifdef __cplusplus
}
#endif

#endif /* RTX_DIST_H */
