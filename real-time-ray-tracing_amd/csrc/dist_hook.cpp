// dist_hook.cpp — include/rtx_dist.h: the multi-GPU screen split behind a C ABI, the counterpart of
// rtx/dist.py (StripGather.exchange / .gather, StripDenoise.exchange_histogram / .exchange_rows) for
// hosts that are not Python, over a communicator the host plugs in (RCCL on a node).
//
// Every data movement is a 2-D copy: a rank's 16-row blocks of one G-buffer are every world-th block
// of the full-frame buffer, i.e. rows of `block bytes` at a pitch of world blocks, so packing the
// blocks one peer needs is one strided copy per G-buffer (not one per block), and a rank's denoise
// strip of each exchanged buffer is one copy of contiguous rows.
#include <hip/hip_runtime.h>
#include <string.h>

#include <string>
#include <vector>

#include "bvh_kernels.h"
#include "rtx_dist.h"

namespace {

// the five path-trace G-buffers and their bytes per pixel, in rtx/dist.py's GBUFFERS order
constexpr int kGb = 5;
constexpr int kGbName[kGb] = {RT_BUF_RENDER_COLOR, RT_BUF_NORMAL, RT_BUF_ALBEDO, RT_BUF_DEPTH, RT_BUF_MOTION};
constexpr size_t kGbBpp[kGb] = {8, 8, 8, 2, 4};
constexpr int kSets = RT_GBUFFER_SETS;  // G-buffer sets of a pipelined context (rt_set_post_stream)

struct Range { uint32_t lo, hi; };

}  // namespace

struct rtd_strips {
    int W = 0, H = 0, N = 1, me = 0;
    rtd_comm comm{};
    std::string err;
    uint32_t rounds = 0;          // 16-row blocks per rank (padded): block b = round * N + owner
    std::vector<Range> dnRows;    // denoise strip per rank
    std::vector<Range> gbRows;    // G-buffer rows per rank's strip-local denoise
    uint32_t maxRows = 0;         // largest denoise strip
    // staging
    void* xsend = nullptr;
    void* xrecv = nullptr;
    size_t xsendCap = 0, xrecvCap = 0;
    void* rsend = nullptr;
    void* rrecv = nullptr;
    // attached buffers (rtd_attach)
    rt_context* ctx = nullptr;
    void* gb[kSets][kGb] = {};
    void* accum = nullptr;
    void* history[2] = {};
    void* rgba = nullptr;
    int32_t* histogram = nullptr;
    std::vector<void*> owned;     // hipMalloc'd by rtd_attach

    size_t blk(int g) const { return (size_t)kRowBlock * W * kGbBpp[g]; }
    size_t row_bytes() const { return (size_t)W * (8 + 8 + 4); }
};

namespace {

int fail(rtd_strips* s, const std::string& what) {
    s->err = what;
    return RT_ERR_STATE;
}

void* stage_alloc(rtd_strips* s, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (s->comm.alloc) return s->comm.alloc(s->comm.arg, bytes);
    void* p = nullptr;
    return hipMalloc(&p, bytes) == hipSuccess ? p : nullptr;
}

void stage_free(rtd_strips* s, void* p) {
    if (!p) return;
    if (s->comm.release) s->comm.release(s->comm.arg, p);
    else (void)hipFree(p);
}

int copy2d(rtd_strips* s, void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t height,
           void* stream) {
    if (width == 0 || height == 0) return 0;
    if (s->comm.copy2d) return s->comm.copy2d(s->comm.arg, dst, dpitch, src, spitch, width, height, stream);
    return hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyDeviceToDevice, (hipStream_t)stream) ==
                   hipSuccess
               ? 0
               : 1;
}

// [j0, j1): the rounds j whose block b = j * N + owner intersects rows [lo, hi) (rtx/dist.py _rounds_in)
void rounds_in(const rtd_strips* s, Range rows, int owner, uint32_t& j0, uint32_t& j1) {
    j0 = 0;
    while (j0 < s->rounds && ((j0 * s->N + owner) + 1) * kRowBlock <= rows.lo) ++j0;
    j1 = j0;
    while (j1 < s->rounds && (j1 * s->N + owner) * kRowBlock < rows.hi) ++j1;
}

// per peer: the rounds this rank sends it and the rounds it receives from it
struct Plan {
    std::vector<uint32_t> s0, s1, r0, r1;
    std::vector<size_t> sb, so, rb, ro;
    size_t sendTotal = 0, recvTotal = 0;
};

Plan make_plan(const rtd_strips* s, int strip_local) {
    Plan p;
    const int N = s->N;
    p.s0.assign(N, 0); p.s1.assign(N, 0); p.r0.assign(N, 0); p.r1.assign(N, 0);
    p.sb.assign(N, 0); p.so.assign(N, 0); p.rb.assign(N, 0); p.ro.assign(N, 0);
    size_t blkAll = 0;
    for (int g = 0; g < kGb; ++g) blkAll += s->blk(g);
    const Range whole = {0, (uint32_t)s->H};
    for (int r = 0; r < N; ++r) {
        if (r == s->me) continue;
        rounds_in(s, strip_local ? s->gbRows[r] : whole, s->me, p.s0[r], p.s1[r]);
        rounds_in(s, strip_local ? s->gbRows[s->me] : whole, r, p.r0[r], p.r1[r]);
        p.sb[r] = (p.s1[r] - p.s0[r]) * blkAll;
        p.rb[r] = (p.r1[r] - p.r0[r]) * blkAll;
    }
    for (int r = 0; r < N; ++r) {
        p.so[r] = p.sendTotal;
        p.sendTotal += p.sb[r];
        p.ro[r] = p.recvTotal;
        p.recvTotal += p.rb[r];
    }
    return p;
}

}  // namespace

extern "C" {

int rtd_create(int width, int height, int world, int rank, const rtd_comm* comm, rtd_strips** out) {
    if (!out) return RT_ERR_ARG;
    *out = nullptr;
    if (width <= 0 || height <= 0 || world < 1 || rank < 0 || rank >= world || !comm || !comm->all_gather ||
        !comm->all_reduce_sum_i32 || !comm->all_to_allv || ((comm->alloc == nullptr) != (comm->release == nullptr)))
        return RT_ERR_ARG;
    rtd_strips* s = new rtd_strips();
    s->W = width;
    s->H = height;
    s->N = world;
    s->me = rank;
    s->comm = *comm;
    const uint32_t blocks = ((uint32_t)height + kRowBlock - 1) / kRowBlock;
    s->rounds = (blocks + world - 1) / world;
    for (int r = 0; r < world; ++r) {
        uint32_t a = 0, b = (uint32_t)height, lo = 0, hi = (uint32_t)height;
        if (world > 1 && !denoise_rows((uint32_t)height, (uint32_t)world, (uint32_t)r, a, b)) {
            delete s;
            return RT_ERR_ARG;  // fewer 64-row denoise blocks than ranks
        }
        gbuffer_rows((uint32_t)height, a, b, lo, hi);
        s->dnRows.push_back({a, b});
        s->gbRows.push_back({lo, hi});
        if (b - a > s->maxRows) s->maxRows = b - a;
    }
    const Plan a = make_plan(s, 0);  // the whole-frame exchange moves the most
    s->xsendCap = a.sendTotal;
    s->xrecvCap = a.recvTotal;
    s->xsend = stage_alloc(s, s->xsendCap);
    s->xrecv = stage_alloc(s, s->xrecvCap);
    s->rsend = stage_alloc(s, (size_t)s->maxRows * s->row_bytes());
    s->rrecv = stage_alloc(s, (size_t)world * s->maxRows * s->row_bytes());
    if (!s->xsend || !s->xrecv || !s->rsend || !s->rrecv) {
        rtd_destroy(s);
        return RT_ERR_HIP;
    }
    *out = s;
    return RT_OK;
}

void rtd_destroy(rtd_strips* s) {
    if (!s) return;
    for (void* p : {s->xsend, s->xrecv, s->rsend, s->rrecv}) stage_free(s, p);
    for (void* p : s->owned) (void)hipFree(p);
    delete s;
}

const char* rtd_last_error(const rtd_strips* s) { return s ? s->err.c_str() : "null rtd_strips"; }

int rtd_denoise_rows(const rtd_strips* s, int rank, int32_t* begin, int32_t* end) {
    if (!s || rank < 0 || rank >= s->N || !begin || !end) return RT_ERR_ARG;
    *begin = (int32_t)s->dnRows[rank].lo;
    *end = (int32_t)s->dnRows[rank].hi;
    return RT_OK;
}

int rtd_gbuffer_rows(const rtd_strips* s, int rank, int32_t* begin, int32_t* end) {
    if (!s || rank < 0 || rank >= s->N || !begin || !end) return RT_ERR_ARG;
    *begin = (int32_t)s->gbRows[rank].lo;
    *end = (int32_t)s->gbRows[rank].hi;
    return RT_OK;
}

size_t rtd_gbuffer_bytes(const rtd_strips* s, int name) {
    if (!s) return 0;
    for (int g = 0; g < kGb; ++g)
        if (kGbName[g] == name) return (size_t)s->rounds * s->N * s->blk(g);
    return 0;
}

size_t rtd_recv_bytes(const rtd_strips* s, int stage, int strip_local) {
    if (!s || s->N < 2) return 0;
    switch (stage) {
        case RT_HOOK_GBUFFERS: return make_plan(s, strip_local).recvTotal;
        case RT_HOOK_ROWS: return (size_t)(s->N - 1) * s->maxRows * s->row_bytes();
        case RT_HOOK_HISTOGRAM: return 256;
        default: return 0;
    }
}

// StripGather.exchange (strip_local) / .gather (whole frame) on caller buffers
int rtd_exchange_gbuffers(rtd_strips* s, const rtd_gbuffers* g, int strip_local, void* stream) {
    if (!s || !g) return RT_ERR_ARG;
    if (s->N < 2) return RT_OK;
    void* const buf[kGb] = {g->color, g->normal, g->albedo, g->depth, g->motion};
    for (void* b : buf)
        if (!b) return RT_ERR_ARG;
    const Plan p = make_plan(s, strip_local);
    char* send = (char*)s->xsend;
    char* recv = (char*)s->xrecv;
    const size_t pitch = (size_t)s->N;  // in blocks
    for (int r = 0; r < s->N; ++r) {  // per peer: every G-buffer's blocks of rounds [s0, s1)
        size_t o = p.so[r];
        const uint32_t n = p.s1[r] - p.s0[r];
        for (int k = 0; k < kGb && n; ++k) {
            const size_t b = s->blk(k);
            const char* src = (const char*)buf[k] + ((size_t)p.s0[r] * s->N + s->me) * b;
            if (copy2d(s, send + o, b, src, pitch * b, b, n, stream)) return fail(s, "copy (G-buffer pack) failed");
            o += n * b;
        }
    }
    if (s->comm.all_to_allv(s->comm.arg, send, p.sb.data(), p.so.data(), recv, p.rb.data(), p.ro.data(), stream))
        return fail(s, "all_to_allv (G-buffers) failed");
    for (int r = 0; r < s->N; ++r) {
        size_t o = p.ro[r];
        const uint32_t n = p.r1[r] - p.r0[r];
        for (int k = 0; k < kGb && n; ++k) {
            const size_t b = s->blk(k);
            char* dst = (char*)buf[k] + ((size_t)p.r0[r] * s->N + r) * b;
            if (copy2d(s, dst, pitch * b, recv + o, b, b, n, stream)) return fail(s, "copy (G-buffer unpack) failed");
            o += n * b;
        }
    }
    return RT_OK;
}

// StripDenoise.exchange_histogram
int rtd_exchange_histogram(rtd_strips* s, int32_t* histogram, void* stream) {
    if (!s || !histogram) return RT_ERR_ARG;
    if (s->N < 2) return RT_OK;
    return s->comm.all_reduce_sum_i32(s->comm.arg, histogram, 64, stream) ? fail(s, "all_reduce (histogram) failed")
                                                                          : RT_OK;
}

// StripDenoise.exchange_rows: rows [a, b) of accumulation | history | RGBA8 packed per row
int rtd_exchange_rows(rtd_strips* s, void* accum, void* history, void* rgba, void* stream) {
    if (!s || !accum || !history || !rgba) return RT_ERR_ARG;
    if (s->N < 2) return RT_OK;
    const size_t W = (size_t)s->W, rb = s->row_bytes();
    const Range mine = s->dnRows[s->me];
    const size_t n = mine.hi - mine.lo;
    char* send = (char*)s->rsend;
    char* recv = (char*)s->rrecv;
    void* const buf[3] = {accum, history, rgba};
    const size_t bpp[3] = {8, 8, 4}, col[3] = {0, W * 8, W * 16};
    for (int k = 0; k < 3; ++k)
        if (copy2d(s, send + col[k], rb, (const char*)buf[k] + mine.lo * W * bpp[k], W * bpp[k], W * bpp[k], n, stream))
            return fail(s, "copy (rows pack) failed");
    const size_t slot = (size_t)s->maxRows * rb;
    if (s->comm.all_gather(s->comm.arg, send, recv, slot, stream)) return fail(s, "all_gather (rows) failed");
    for (int r = 0; r < s->N; ++r) {
        if (r == s->me) continue;
        const Range q = s->dnRows[r];
        for (int k = 0; k < 3; ++k)
            if (copy2d(s, (char*)buf[k] + q.lo * W * bpp[k], W * bpp[k], recv + r * slot + col[k], rb, W * bpp[k],
                       q.hi - q.lo, stream))
                return fail(s, "copy (rows unpack) failed");
    }
    return RT_OK;
}

int rtd_hook(void* arg, int stage, void* stream, const rt_strip_exchange* x) {
    rtd_strips* s = (rtd_strips*)arg;
    if (!s || !x || !s->ctx) return RT_ERR_ARG;
    switch (stage) {
        case RT_HOOK_GBUFFERS: {
            if (x->gbufferSet < 0 || x->gbufferSet >= kSets) return fail(s, "hook: G-buffer set out of range");
            void* const* b = s->gb[x->gbufferSet];
            const rtd_gbuffers g = {b[0], b[1], b[2], b[3], b[4]};
            return rtd_exchange_gbuffers(s, &g, x->stripLocal, stream);
        }
        case RT_HOOK_HISTOGRAM: return rtd_exchange_histogram(s, s->histogram, stream);
        case RT_HOOK_ROWS:
            if ((uint32_t)x->rowBegin != s->dnRows[s->me].lo || (uint32_t)x->rowEnd != s->dnRows[s->me].hi)
                return fail(s, "hook: renderer and host disagree on the strip");
            if (x->historySet < 0 || x->historySet > 1) return fail(s, "hook: history set out of range");
            return rtd_exchange_rows(s, s->accum, s->history[x->historySet], s->rgba, stream);
        default: return fail(s, "hook: unknown stage");
    }
}

int rtd_attach(rtd_strips* s, rt_context* ctx) {
    if (!s || !ctx) return RT_ERR_ARG;
    rt_info info;
    int rc = rt_get_info(ctx, &info);
    if (rc != RT_OK) return rc;
    if (info.renderWidth != s->W || info.renderHeight != s->H || info.screenWidth != s->W ||
        info.screenHeight != s->H)
        return fail(s, "rtd_attach: the context's render and screen size must be the strips' size");
    int32_t a = 0, b = 0;
    rtd_denoise_rows(s, s->me, &a, &b);
    if (s->N > 1 && (info.denoiseRowBegin != a || info.denoiseRowEnd != b))
        return fail(s, "rtd_attach: the context is not this rank's strip (stripCount / stripIndex)");
    auto alloc = [&](size_t bytes, void** p) -> int {
        if (hipMalloc(p, bytes) != hipSuccess) return fail(s, "rtd_attach: hipMalloc failed");
        s->owned.push_back(*p);
        return hipMemset(*p, 0, bytes) == hipSuccess ? RT_OK : fail(s, "rtd_attach: hipMemset failed");
    };
    for (int k = 0; k < kSets; ++k)
        for (int g = 0; g < kGb; ++g) {
            const size_t bytes = rtd_gbuffer_bytes(s, kGbName[g]);
            if ((rc = alloc(bytes, &s->gb[k][g])) != RT_OK) return rc;
            if ((rc = rt_bind_buffer(ctx, kGbName[g] | (k << 8), s->gb[k][g], bytes)) != RT_OK) return rc;
        }
    const size_t P = (size_t)s->W * s->H;
    if ((rc = alloc(P * 8, &s->accum)) != RT_OK || (rc = alloc(P * 8, &s->history[0])) != RT_OK ||
        (rc = alloc(P * 8, &s->history[1])) != RT_OK || (rc = alloc(P * 4, &s->rgba)) != RT_OK ||
        (rc = alloc(256, (void**)&s->histogram)) != RT_OK)
        return rc;
    if ((rc = rt_bind_buffer(ctx, RT_BUF_ACCUMULATION, s->accum, P * 8)) != RT_OK ||
        (rc = rt_bind_buffer(ctx, RT_BUF_HISTORY_COLOR, s->history[0], P * 8)) != RT_OK ||
        (rc = rt_bind_buffer(ctx, RT_BUF_HISTORY_COLOR | RT_BUF_SET1, s->history[1], P * 8)) != RT_OK ||
        (rc = rt_bind_buffer(ctx, RT_BUF_RGBA8, s->rgba, P * 4)) != RT_OK ||
        (rc = rt_bind_buffer(ctx, RT_BUF_HISTOGRAM, s->histogram, 256)) != RT_OK)
        return rc;
    s->ctx = ctx;
    if (s->N < 2) return RT_OK;
    if ((rc = rt_set_collective_hook(ctx, rtd_hook, s)) != RT_OK) return rc;
    return rt_set_hook_stages(ctx, (1u << RT_HOOK_GBUFFERS) | (1u << RT_HOOK_HISTOGRAM) | (1u << RT_HOOK_ROWS));
}

}  // extern "C"
