// frame.cpp — the per-frame part of RayTracer::draw (kernel.cu:259-398) behind the C-ABI:
// sky/sun regeneration, the path tracer, G-buffer access.  Denoise and post-processing
// stages are dispatched from here as they land.
//
//   sun direction       UpdateFrame (kernel.cu:119-123), rotate3f (linearMath.h:650-716)
//   UpdateSkyState      sky.cuh:124-146 (host, float + rtmath, like the reference's host code)
//   sky regeneration    kernel.cu:286-307
//   PathTrace launch    kernel.cu:330-350; HistoryCamera::Setup kernel.cu:133-136, 357
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <fstream>
#include <utility>
#include <vector>

#include "context.h"
#include "rtmath.h"

namespace {

constexpr float kPi = 3.1415926535897932384626422832795028841971f;
constexpr float kTwoPi = 6.2831853071795864769252867665590057683943f;
constexpr float kPiOver180 = 0.01745329251f;

// ---- host vector helpers with the device rounding policy (one rounding per op, fma only
// where the reference's TwoProd/InnerProduct use it)
struct V3 { float x, y, z; };
V3 v3(float x, float y, float z) { return V3{x, y, z}; }
V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
V3 operator*(float s, V3 a) { return v3(a.x * s, a.y * s, a.z * s); }
V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
float dop(float a, float b, float c, float d) {
    const float cd = c * d;
    const float err = fmaf(-c, d, cd);
    const float dp = fmaf(a, b, -cd);
    return dp + err;
}
float inner3(float a, float b, float c, float d, float e, float f) {
    const float ef = e * f, efe = fmaf(e, f, -ef);
    const float cd = c * d, cde = fmaf(c, d, -cd);
    const float s2 = cd + ef, dl2 = s2 - cd, s2e = (cd - (s2 - dl2)) + (ef - dl2);
    const float tpv = s2, tpe = cde + (efe + s2e);
    const float ab = a * b, abe = fmaf(a, b, -ab);
    const float s1 = ab + tpv, dl1 = s1 - ab, s1e = (ab - (s1 - dl1)) + (tpv - dl1);
    return s1 + (abe + (tpe + s1e));
}
float dot(V3 a, V3 b) { return inner3(a.x, b.x, a.y, b.y, a.z, b.z); }
V3 cross(V3 a, V3 b) { return v3(dop(a.y, b.z, a.z, b.y), dop(a.z, b.x, a.x, b.z), dop(a.x, b.y, a.y, b.x)); }
V3 normalize(V3 v) {
    const float n = sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    return v3(v.x / n, v.y / n, v.z / n);
}

struct Quat { V3 v; float w; };
Quat qmul(const Quat& p, const Quat& q) { return Quat{p.w * q.v + q.w * p.v + cross(p.v, q.v), p.w * q.w - dot(p.v, q.v)}; }

// sunDir = rotate3f(axis, angle, cross(up, axis)).normalized()
V3 sun_direction(float timeOfDay, float sunAxisAngle) {
    const V3 axis = normalize(v3(0.0f, rt_cosf(sunAxisAngle * kPiOver180), rt_sinf(sunAxisAngle * kPiOver180)));
    const float angle = fmodf(timeOfDay * kPi, kTwoPi);
    const V3 v = cross(v3(0.0f, 1.0f, 0.0f), axis);
    const Quat q{normalize(axis) * rt_sinf(angle / 2), rt_cosf(angle / 2)};
    const Quat r = qmul(qmul(q, Quat{v, 0.0f}), Quat{-q.v, q.w});
    return normalize(r.v);
}

float fitting(const float* m, float s, int i) {  // GetFittingData (sky.cuh:90-99)
    return (rt_powf(1.0f - s, 5.0f) * m[i] + 5.0f * rt_powf(1.0f - s, 4.0f) * s * m[i + 9] +
            10.0f * rt_powf(1.0f - s, 3.0f) * rt_powf(s, 2.0f) * m[i + 18] +
            10.0f * rt_powf(1.0f - s, 2.0f) * rt_powf(s, 3.0f) * m[i + 27] +
            5.0f * (1.0f - s) * rt_powf(s, 4.0f) * m[i + 36] + rt_powf(s, 5.0f) * m[i + 45]);
}
float fitting2(const float* m, float s) {  // GetFittingData2 (sky.cuh:102-111)
    return (rt_powf(1.0f - s, 5.0f) * m[0] + 5.0f * rt_powf(1.0f - s, 4.0f) * s * m[1] +
            10.0f * rt_powf(1.0f - s, 3.0f) * rt_powf(s, 2.0f) * m[2] +
            10.0f * rt_powf(1.0f - s, 2.0f) * rt_powf(s, 3.0f) * m[3] + 5.0f * (1.0f - s) * rt_powf(s, 4.0f) * m[4] +
            rt_powf(s, 5.0f) * m[5]);
}

struct SkyTablesHost {
    std::vector<float> skyDataSets, skyDataSetsRad, solar, limb, cieX, cieY, cieZ;
};
SkyTablesHost g_tables;  // immutable after the first successful load

bool load_sky_tables(const std::string& path, SkyTablesHost& t, std::string& err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) { err = "cannot read " + path; return false; }
    uint32_t count = 0;
    f.read((char*)&count, 4);
    if (count != 7) { err = "bad sky table file " + path; return false; }
    uint32_t len[7];
    f.read((char*)len, sizeof(len));
    const uint32_t expect[7] = {540, 60, 1800, 60, 10, 10, 10};
    std::vector<float>* dst[7] = {&t.skyDataSets, &t.skyDataSetsRad, &t.solar, &t.limb, &t.cieX, &t.cieY, &t.cieZ};
    for (int i = 0; i < 7; ++i) {
        if (len[i] != expect[i]) { err = "bad sky table sizes in " + path; return false; }
        dst[i]->resize(len[i]);
        f.read((char*)dst[i]->data(), len[i] * 4);
    }
    if (!f) { err = "truncated " + path; return false; }
    return true;
}

bool sky_params_equal(const rt_sky_params& a, const rt_sky_params& b) {
    return a.timeOfDay == b.timeOfDay && a.sunAxisAngle == b.sunAxisAngle && a.skyScalar == b.skyScalar &&
           a.sunScalar == b.sunScalar && a.sunAngle == b.sunAngle;
}

// kernel.cu:286-307 — regenerate when asked to, or when the sky parameters changed
int update_sky(rt_context* ctx) {
    FrameResources& fr = ctx->fr;
    rt_sky_params& sp = ctx->params.sky;
    const V3 sunDir = sun_direction(sp.timeOfDay, sp.sunAxisAngle);
    fr.sunDir[0] = sunDir.x; fr.sunDir[1] = sunDir.y; fr.sunDir[2] = sunDir.z;
    if (fr.skyValid && !sp.needRegenerate && sky_params_equal(sp, fr.lastSky)) return RT_OK;
    if (fr.spec.valid) HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->specDone, 0));  // they read the sky
    if (ctx->postStream) {  // frame pipelining: nothing may read the sky while it is rewritten
        const int rc = sync_streams(ctx, false);
        if (rc != RT_OK) return rc;
    }
    sp.sunScalar = sp.sunScalar > 0.00001f ? sp.sunScalar : 0.00001f;
    sp.skyScalar = sp.skyScalar > 0.00001f ? sp.skyScalar : 0.00001f;
    sp.sunAngle = sp.sunAngle > 0.51f ? sp.sunAngle : 0.51f;
    SkyGenParams p;
    memcpy(p.sunDir, fr.sunDir, 12);
    p.skyScalar = sp.skyScalar;
    p.sunScalar = sp.sunScalar;
    p.sunAngle = sp.sunAngle;
    const float elevation = rt_acosf(sunDir.y);
    const float se = rt_powf(elevation / (kPi / 2.0f), (1.0f / 3.0f));
    for (int ch = 0; ch < 10; ++ch) {
        for (int i = 0; i < 9; ++i) p.st.configs[ch * 9 + i] = fitting(g_tables.skyDataSets.data() + ch * 54, se, i);
        p.st.radiances[ch] = fitting2(g_tables.skyDataSetsRad.data() + ch * 6, se);
    }
    const float sunRadius = sp.sunAngle * kPi / 180.0f / 2.0f;
    p.cosThetaMax = rt_cosf(sunRadius);
    p.solar = fr.solar;
    p.limb = fr.limb;
    p.cie = fr.cie;
    p.skyBuffer = fr.sky;
    p.skyPdf = fr.skyPdf;
    p.skyCdf = fr.skyCdf;
    p.sunBuffer = fr.sun;
    p.sunPdf = fr.sunPdf;
    p.sunCdf = fr.sunCdf;
    p.scanSums = fr.scanSums;
    p.skyTree = fr.skyTree;
    p.sunTree = fr.sunTree;
    p.lightSel = fr.lightSel;
    HIP_TRY(ctx, rtk_launch_sky(&p, ctx->stream));
    if (ctx->postStream) HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // before the side stream's camera rays
    fr.sunArea = rt_powf(rt_tanf(sunRadius), 2.0f) * kPi;
    fr.cosThetaMax = p.cosThetaMax;
    fr.skyValid = true;
    sp.needRegenerate = 0;
    fr.lastSky = sp;
    return RT_OK;
}

// LocalizeSample(sunDir) (sampler / sky.cuh): u = cross(n, w), v = cross(n, u) with the
// reference's fma-based DiffOfProducts cross, exactly as the device evaluates it
float dop_host(float a, float b, float c, float d) {
    const float cd = c * d;
    const float err = fmaf(-c, d, cd);
    const float dp = fmaf(a, b, -cd);
    return dp + err;
}
void sun_frame(const float n[3], float t[3], float b[3]) {
    float w[3] = {1.0f, 0.0f, 0.0f};
    if (fabsf(n[0]) > 0.707f) { w[0] = 0.0f; w[1] = 1.0f; }
    auto cross = [](const float* a, const float* c, float* r) {
        r[0] = dop_host(a[1], c[2], a[2], c[1]);
        r[1] = dop_host(a[2], c[0], a[0], c[2]);
        r[2] = dop_host(a[0], c[1], a[1], c[0]);
    };
    cross(n, w, t);
    cross(n, t, b);
}

HistCamera hist_of(const HostCamera& c) {
    HistCamera h;
    memcpy(h.pos, c.pos, 12);
    memcpy(h.left, c.left, 12);
    memcpy(h.up, c.up, 12);
    memcpy(h.dir, c.dir, 12);
    return h;
}

}  // namespace

// point the G-buffer views at set fr.gbSet
void select_gbuffers(FrameResources& fr) {
    const int k = fr.gbSet;
    if (fr.renderColor == fr.color) fr.renderColor = fr.gColor[k];
    fr.color = fr.gColor[k];
    fr.normal = fr.gNormal[k];
    fr.albedo = fr.gAlbedo[k];
    fr.depth = fr.gDepth[k];
    fr.motion = fr.gMotion[k];
}

// the denoise/post chain of one frame on stream s: phase 0, the histogram exchange, phase 1, the
// rows exchange (the exchanges only for a strip-local denoise, through the caller's hook)
// Whether this context's next denoise is strip-local (multi-GPU: a collective hook, and none of
// the passes that read the whole frame), and its rows [a, b) (the whole frame otherwise).
bool strip_local_denoise(const rt_context* ctx, uint32_t& a, uint32_t& b) {
    const rt_render_pass_settings& ps = ctx->params.pass;
    const uint32_t H = (uint32_t)ctx->renderH;
    a = 0;
    b = H;
    // TemporalFilter2 on: its output (the exchanged history buffer) is then the frame's final HDR
    const bool strip = ctx->stripCount > 1 && ctx->hook != nullptr && !ps.enableNoiseLevelVisualize &&
                       !(ps.enablePostProcess && (ps.enableBloomEffect || ps.enableLensFlare)) &&
                       ps.enableTemporalDenoising2 && ctx->screenW == ctx->renderW && ctx->screenH == ctx->renderH;
    uint32_t sa = 0, sb = H;
    if (!strip || !denoise_rows(H, (uint32_t)ctx->stripCount, (uint32_t)ctx->stripIndex, sa, sb)) return false;
    a = sa;
    b = sb;
    return true;
}

int run_denoise(rt_context* ctx, DenoisePostParams& p, hipStream_t s) {
    rt_strip_exchange x{p.frameNum, (int32_t)p.rowA, (int32_t)p.rowB, p.histOutSet, p.gbSet, p.stripLocal};
    // the G-buffer rows this rank's denoise reads, from the ranks that traced them (opt-in stage:
    // rtx/dist.py's FramePipeline moves them itself, rtx_dist.h's rtd_hook through this call)
    if (ctx->stripCount > 1 && ctx->hook && (ctx->hookStages & (1u << RT_HOOK_GBUFFERS)) &&
        ctx->hook(ctx->hookArg, RT_HOOK_GBUFFERS, (void*)s, &x) != 0) {
        ctx->err = "collective hook failed (G-buffers)";
        return RT_ERR_STATE;
    }
    if (p.marks)  // every marked pair recorded once up front: a kernel this frame does not launch reads 0 ms
        for (int k = 0; k < 2 * kDnKernels; ++k)
            if (p.marks[k]) HIP_TRY(ctx, hipEventRecord(p.marks[k], s));
    // taken when the denoise is issued (a deferred one runs after the earlier frames' swaps)
    p.tileParity = ctx->fr.tileParity;
    p.accum = ctx->fr.accum;
    p.accumAlt = ctx->fr.accumAlt;
    HIP_TRY(ctx, rtk_denoise_phase(&p, s, 0));
    if (p.listUsed) {  // the list chain wrote the other accumulation buffer; the next list frame
        ctx->fr.tileParity ^= 1;  // appends under the other counters
        if (ctx->fr.accumBound || p.stripLocal) {
            // the caller's buffer (a strip-local rank exchanges its rows of it) gets the rows this
            // chain finished — a strip-local rank's own rows, which the rows exchange gathers; the
            // halo rows the later passes read come from accumAlt (their `alt`) — once TemporalFilter,
            // the last reader of the previous frame's accumulation, is done
            const size_t r0 = p.stripLocal ? p.rowA : 0, r1 = p.stripLocal ? p.rowB : p.H;
            HIP_TRY(ctx, hipMemcpyAsync(p.accum + r0 * p.W, p.accumAlt + r0 * p.W, (r1 - r0) * p.W * 8,
                                        hipMemcpyDeviceToDevice, s));
        } else {
            std::swap(ctx->fr.accum, ctx->fr.accumAlt);
        }
    }
    // the histogram is recomputed only with the post chain on; summing a stale one again would
    // multiply it by the rank count every frame
    if (p.stripLocal && p.postProcess && ctx->hook(ctx->hookArg, RT_HOOK_HISTOGRAM, (void*)s, &x) != 0) {
        ctx->err = "collective hook failed (histogram)";
        return RT_ERR_STATE;
    }
    HIP_TRY(ctx, rtk_denoise_phase(&p, s, 1));
    if (!p.stripLocal) return RT_OK;
    if (ctx->hook(ctx->hookArg, RT_HOOK_ROWS, (void*)s, &x) != 0) {
        ctx->err = "collective hook failed (rows)";
        return RT_ERR_STATE;
    }
    // whole-frame outputs exist only after the exchange: the HDR copy of the final colour (the
    // exchanged history buffer) and the caller's draw target (k_scale_post wrote this rank's rows
    // into the exchanged RGBA8 buffer)
    const size_t W = p.W, H = p.H;
    if (p.hdrOut) HIP_TRY(ctx, rtk_hdr_out(p.finalColor, p.hdrOut, W * H, s));
    if (p.rgbaTarget)
        HIP_TRY(ctx, hipMemcpy2DAsync(p.rgbaTarget, (size_t)p.rgbaTargetPitch * 4, p.rgba, (size_t)p.Ws * 4,
                                      (size_t)p.Ws * 4, (size_t)p.Hs, hipMemcpyDeviceToDevice, s));
    return RT_OK;
}

// enqueue a deferred rt_denoise_post on the post stream (frame pipelining)
int issue_pending_post(rt_context* ctx) {
    if (!ctx->postPending) return RT_OK;
    ctx->postPending = false;
    const int set = ctx->postPendingSet;
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->postStream, ctx->ptDone[set], 0));
    if (ctx->postGather) HIP_TRY(ctx, hipStreamWaitEvent(ctx->postStream, ctx->gatherDone[set], 0));
    if (int rc = run_denoise(ctx, ctx->postParams, ctx->postStream)) return rc;
    HIP_TRY(ctx, hipEventRecord(ctx->postDone[set], ctx->postStream));
    ctx->fr.renderColor = ctx->postParams.finalColor;  // the launcher's buffer plan names them
    ctx->fr.scaledColor = ctx->postParams.finalScaled;
    return RT_OK;
}

namespace {
// PtLaunchHook of a pipelined frame: after kernel `overlapAfter` the previous frame's denoise
// is issued (it then runs beside the trace stages' latency-bound tails), and after kernel
// `cameraAfter` the gate event the next frame's camera rays wait for is recorded
// the previous frame's deferred denoise, behind everything enqueued so far on the context stream
hipError_t issue_overlapped_post(rt_context* ctx) {
    hipError_t e = hipEventRecord(ctx->overlapEv, ctx->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(ctx->postStream, ctx->overlapEv, 0);
    if (e == hipSuccess && issue_pending_post(ctx) != RT_OK) e = hipErrorUnknown;
    return e;
}

hipError_t overlap_hook(void* arg, int kernel) {
    rt_context* ctx = (rt_context*)arg;
    hipError_t e = hipSuccess;
    if (kernel == ctx->overlapAfter && ctx->postPending) e = issue_overlapped_post(ctx);
    if (e == hipSuccess && kernel == ctx->cameraAfter) {
        e = hipEventRecord(ctx->cameraGate, ctx->stream);
        ctx->cameraGated = e == hipSuccess;
    }
    return e;
}
}  // namespace

// wait for the context stream and, when set, the post stream.  `report`: return a kernel's failure
// report (RT_ERR_DEVICE) — rt_sync, the draws, the reads and rt_build_bvh do; the setters that only
// need the streams idle (stream / hook / buffer / texture changes) pass false and do their work, the
// report then waiting for the next reporting call.
int sync_streams(rt_context* ctx, bool report) {
    if (ctx->postStream) {
        const int rc = issue_pending_post(ctx);
        if (rc != RT_OK) return rc;
    }
    if (ctx->sideStream) HIP_TRY(ctx, hipStreamSynchronize(ctx->sideStream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->postStream) HIP_TRY(ctx, hipStreamSynchronize(ctx->postStream));
    poll_q3(ctx);
    // camera rays a synchronous draw traced ahead are kept only up to the next draw: any call that
    // waits for the streams (a read, a setter, a mode change) drops them
    FrameResources& fr = ctx->fr;
    if (fr.spec.valid) {
        fr.spec.valid = false;
        fr.syncZeroed[fr.spec.block] = false;
        fr.specCounts = 2;
    }
    if (fr.specCounts) {  // the ray counts of launches ahead: the used ones into the frame's
        HIP_TRY(ctx, rtk_fold_ray_counts(fr.specCounts == 1 ? fr.rayCounter : nullptr, fr.specRayCounter, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        fr.specCounts = 0;
    }
    return report ? check_device_status(ctx) : RT_OK;
}

// The end of a synchronous draw: its frame is complete (kernel.cu:393-397) once the context stream
// is idle; the next frame's camera rays traced ahead may still run on the side stream
static int sync_draw(rt_context* ctx) {
    if (!ctx->fr.spec.valid) return sync_streams(ctx);
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    poll_q3(ctx);
    return check_device_status(ctx);
}

// The last serial frame's queue-3 length (rt_path_trace's chain choice), if k_pt_resolve has
// stored it: the pinned word pairs the length with the tag of the frame that asked for it, so a
// host that never syncs still picks it up at its next path trace, without waiting.
void poll_q3(rt_context* ctx) {
    FrameResources& fr = ctx->fr;
    if (!fr.q3Pending) return;
    const unsigned long long v = __atomic_load_n(fr.q3Host, __ATOMIC_ACQUIRE);
    if ((uint32_t)(v >> 32) != fr.q3Tag) return;
    fr.lastQ3 = (uint32_t)v;
    fr.q3Pending = false;
}

// Failures the kernels reported into the pinned status words (rt_device.h report_status): the
// LBVH's TLAS workgroup timed out waiting for a batch's publication.  The error is reported once,
// and the launch counters of both LBVH sets are re-armed (a batch that never published left its
// set's counter one short).  Called after the streams are idle (sync_streams) or before a build.
int check_device_status(rt_context* ctx) {
    const uint32_t missing = __atomic_load_n(&ctx->status[kStatusTlasTimeout], __ATOMIC_ACQUIRE);
    if (!missing) return RT_OK;
    const uint32_t build = __atomic_load_n(&ctx->status[kStatusTlasTimeoutBuild], __ATOMIC_ACQUIRE);
    if (ctx->sideStream) HIP_TRY(ctx, hipStreamSynchronize(ctx->sideStream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    for (const BvhBufs& b : ctx->bvh)
        if (b.counter) HIP_TRY(ctx, hipMemset(b.counter, 0, 64));
    __atomic_store_n(&ctx->status[kStatusTlasTimeout], 0u, __ATOMIC_RELEASE);
    __atomic_store_n(&ctx->status[kStatusTlasTimeoutBuild], 0u, __ATOMIC_RELEASE);
    ctx->err = "LBVH build: the TLAS workgroup timed out waiting for " + std::to_string(missing) +
               " batch publication(s) (last in build " + std::to_string(build) +
               "); the TLAS of that build (and the frames traced on it) may be wrong";
    return RT_ERR_DEVICE;
}

// UpdateFrame's timer (kernel.cu:67-71): the frame time rt_draw already took, the fixed one
// (rt_set_delta_time) or the wall clock since the previous call.  The 75-fps limiter's busy wait
// (timer.h) is frame pacing for a window and is not reproduced.
float frame_delta(rt_context* ctx) {
    FrameResources& fr = ctx->fr;
    if (fr.drawDt >= 0.0f) {
        const float d = fr.drawDt;
        fr.drawDt = -1.0f;
        return d;
    }
    if (ctx->deltaMs > 0.0f) return ctx->deltaMs;
    const double now = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    const float dt = fr.lastDrawTime < 0 ? 1000.0f / 60.0f : (float)((now - fr.lastDrawTime) * 1000.0);
    fr.lastDrawTime = now;
    return dt;
}

// UpdateFrame's dynamic resolution (kernel.cu:77-100): outside the targetFps +-2 band the width
// scales by sqrt(target / frame time), snaps to a multiple of 16, clamps to [minWidth, maxWidth]
// and the height follows at 16:9.  Every render-size buffer was allocated at the initial (max)
// size; a height past maxHeight (a config whose max is not 16:9) is clamped to it so it fits.
void update_dynamic_resolution(rt_context* ctx, float dt) {
    if (!(dt > 0.0f)) return;
    const float hi = 1000.0f / (ctx->targetFps - 2), lo = 1000.0f / (ctx->targetFps + 2);
    int w = ctx->renderW;
    if (hi < dt || lo > dt) {
        const float ratio = sqrtf((1000.0f / ctx->targetFps) / dt);
        w = (int)((float)w * ratio);
    }
    w = w + ((w % 16 < 8) ? (-w % 16) : (16 - w % 16));
    w = w < ctx->minWidth ? ctx->minWidth : w > ctx->maxWidth ? ctx->maxWidth : w;
    int h = (w / 16) * 9;
    if (h > ctx->maxHeight) h = ctx->maxHeight;
    ctx->renderW = w;
    ctx->renderH = h;
    ctx->stripRows = h;
}

int rt_frame_init(rt_context* ctx) {
    FrameResources& fr = ctx->fr;
    std::string err;
    if (g_tables.solar.empty()) {
        SkyTablesHost t;
        if (!load_sky_tables(rt_data_dir() + "/sky_tables.bin", t, err)) { ctx->err = err; return RT_ERR_IO; }
        g_tables = std::move(t);
    }
    int rc;
#define ALLOC(p, bytes) if ((rc = dalloc(ctx, &(p), (bytes))) != RT_OK) return rc
    ALLOC(fr.solar, 1800 * 4);
    ALLOC(fr.limb, 60 * 4);
    ALLOC(fr.cie, 30 * 4);
    ALLOC(fr.sky, (size_t)kSkySize * 16);
    ALLOC(fr.skyPdf, (size_t)kSkySize * 4);
    ALLOC(fr.skyCdf, (size_t)kSkySize * 4);
    ALLOC(fr.sun, (size_t)kSunSize * 16);
    ALLOC(fr.sunPdf, (size_t)kSunSize * 4);
    ALLOC(fr.sunCdf, (size_t)kSunSize * 4);
    ALLOC(fr.scanSums, 512 * 4);
    ALLOC(fr.skyTree, (size_t)kSkyTreeNodes * 4);
    ALLOC(fr.sunTree, (size_t)kSunTreeNodes * 4);
    ALLOC(fr.lightSel, 16);
    ALLOC(fr.texAlbedo, (size_t)kTexTexels * 8);
    ALLOC(fr.texNormal, (size_t)kTexTexels * 8);
    ALLOC(fr.texHeight, (size_t)kTexTexels * 2);
    HIP_TRY(ctx, hipMemset(fr.texHeight, 0, (size_t)kTexTexels * 2));
    const size_t P = (size_t)ctx->renderW * ctx->renderH;
    ALLOC(fr.color, P * 8);
    ALLOC(fr.normal, P * 8);
    ALLOC(fr.albedo, P * 8);
    ALLOC(fr.depth, P * 2);
    ALLOC(fr.motion, P * 4);
    fr.gColor[0] = fr.color;
    fr.gNormal[0] = fr.normal;
    fr.gAlbedo[0] = fr.albedo;
    fr.gDepth[0] = fr.depth;
    fr.gMotion[0] = fr.motion;
    ALLOC(fr.rays, P * 4);
    ALLOC(fr.ptStats, P * 16);
    ALLOC(fr.rayCounter, (size_t)kRayCounterSlots * kRayCounterStride * 8);
    {  // wavefront workspace: one entry per traced sample of the strip
        const size_t cap = (size_t)ctx->renderW * ctx->stripRows * ctx->spp;
        if (cap >= (1ull << 31)) { ctx->err = "strip x spp too large for the path-trace queues"; return RT_ERR_ARG; }
        PtWorkspace& ws = fr.ws;
        ws.cap = (uint32_t)cap;
        ALLOC(ws.hit0Rec, cap * 16);
        ALLOC(ws.hit0Err, cap * 4);
        for (PtQueue* q : {&ws.q3, &ws.q4}) {
            ALLOC(q->rayO, cap * 16);
            ALLOC(q->rayD, cap * 16);
            ALLOC(q->st0, cap * 16);
            ALLOC(q->st1, cap * 16);
            ALLOC(q->st2, cap * 16);
        }
        ALLOC(ws.hitRec, cap * 16);
        ALLOC(ws.hitErr, cap * 4);
        ALLOC(ws.pathL, cap * 16);
        ALLOC(ws.pending, (size_t)ctx->renderW * ctx->stripRows * 4);
        ALLOC(ws.surface, (size_t)ctx->renderW * ctx->stripRows * 4);
        ALLOC(fr.camCount[0], kWsCounterWords * 4);
        ALLOC(fr.syncCount[1], kWsCounterWords * 4);
        ALLOC(fr.syncCount[2], kWsCounterWords * 4);
        fr.syncCount[0] = fr.camCount[0];
        fr.camQ3[0] = ws.q3;
        fr.camQ4[0] = ws.q4;
        fr.camHitRec[0] = ws.hitRec;
        fr.camHitErr[0] = ws.hitErr;
        fr.camPathL[0] = ws.pathL;
        fr.camPending[0] = ws.pending;
        fr.camHit0Rec[0] = ws.hit0Rec;
        fr.camHit0Err[0] = ws.hit0Err;
        fr.camSurface[0] = ws.surface;
        ws.counters = fr.camCount[0];
        ws.fetch = ws.counters + 64;
        int dev = 0, cus = 0;
        HIP_TRY(ctx, hipGetDevice(&dev));
        HIP_TRY(ctx, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        const int perCu = rtk_trace_queue_blocks_per_cu();
        if (cus <= 0) cus = 256;
        // grid of the persistent shade / resume kernels: 5 workgroups per CU (measured)
        ws.persistBlocks = (uint32_t)(cus * 5);
        ws.cus = (uint32_t)cus;
        ws.shadeBlocksPerCu = (uint32_t)(ctx->tune.shadeBlocksPerCu > 0 ? ctx->tune.shadeBlocksPerCu : 0);
        // the queue tracers run below their residency (5 workgroups per CU at 32 KiB of LDS
        // stack each): queue 3 at 3 per CU, queue 4 at 1, so a bounce queue holds
        // more rays than lanes, lanes refill as rays finish, and the CUs keep room for the
        // denoise and next-frame waves beside the traversal tail (measured: DESIGN.md §7)
        int tracePerCu = perCu >= 3 ? 3 : (perCu > 0 ? perCu : 1), trace4PerCu = 1;
        const rt_context::Tuning& tn = ctx->tune;  // [tuning] tracePerCu / trace4PerCu (A/B aids)
        if (tn.tracePerCu > 0 && tn.tracePerCu <= perCu) tracePerCu = tn.tracePerCu;
        if (tn.trace4PerCu > 0 && tn.trace4PerCu <= perCu) trace4PerCu = tn.trace4PerCu;
        ws.traceBlocks = (uint32_t)(cus * tracePerCu);
        // one GPU: a short queue 3 (below kTrace3Short rays, the default view's 323 k) is traced by
        // 2 workgroups per CU, which leaves the next frame's camera waves more room (1.091 -> 1.081
        // ms/frame, four repeats); a long one (the terrain view) keeps all of them (2 per CU there:
        // 4.14 -> 4.44 ms); strip ranks keep 3 (at 2 ranks 0.710 vs 0.727 ms, equal at 4 and 8)
        ws.trace3ShortBlocks = ctx->stripCount == 1 && tn.trace3ShortPerCu > 0 ? (uint32_t)(cus * tn.trace3ShortPerCu) : 0u;
        ws.chain = (uint32_t)tn.chain;  // [tuning] chain = "off" | "serial" | "always" (default serial)
        ws.trace4Blocks = (uint32_t)(cus * trace4PerCu);
    }
    ALLOC(fr.colorB, P * 8);
    ALLOC(fr.accum, P * 8);
    ALLOC(fr.accumAlt, P * 8);  // the list chain's other accumulation buffer (denoise.hip active-tile lists)
    ALLOC(fr.histBuf[0], P * 8);
    ALLOC(fr.histBuf[1], P * 8);
    ALLOC(fr.histDepth, P * 2);
    const size_t W = (size_t)ctx->renderW, H = (size_t)ctx->renderH;
    const size_t W4 = (W + 3) / 4, H4 = (H + 3) / 4, W16 = (W4 + 3) / 4, H16 = (H4 + 3) / 4;
    ALLOC(fr.noise8, ((W + 7) / 8) * ((H + 7) / 8) * 2);
    ALLOC(fr.noise16, ((W + 15) / 16) * ((H + 15) / 16) * 2);
    ALLOC(fr.chainCounter, 4);
    HIP_TRY(ctx, hipMemset(fr.chainCounter, 0, 4));
    {  // active-tile lists (denoise.hip): 2 x 2 x 16 counters 128 B apart, then 2 x 16 partitions of entries
        fr.tileCap = (uint32_t)(((W + 15) / 16) * ((H + 15) / 16));
        const size_t words = 2 * 2 * 16 * 32 + 2 * 16 * (size_t)(fr.tileCap / 16 + 1);
        ALLOC(fr.tileList, words * 4);
        HIP_TRY(ctx, hipMemset(fr.tileList, 0, words * 4));
    }
    ALLOC(fr.c4, W4 * H4 * 8);
    ALLOC(fr.c16, W16 * H16 * 8);
    ALLOC(fr.c64, ((W16 + 3) / 4) * ((H16 + 3) / 4) * 8);
    ALLOC(fr.bloom4, W4 * H4 * 8);
    ALLOC(fr.bloom16, W16 * H16 * 8);
    ALLOC(fr.histogram, 256);
    ALLOC(fr.exposure, 16);
    const size_t Ps = (size_t)ctx->screenW * ctx->screenH;
    ALLOC(fr.scaledA, Ps * 8);
    ALLOC(fr.scaledB, Ps * 8);
    ALLOC(fr.rgba, Ps * 4);
    fr.outRgba = fr.rgba;
    fr.outPitch = (uint32_t)ctx->screenW;
    ALLOC(fr.hdr, P * 16);
#undef ALLOC
    HIP_TRY(ctx, hipMemcpy(fr.solar, g_tables.solar.data(), 1800 * 4, hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemcpy(fr.limb, g_tables.limb.data(), 60 * 4, hipMemcpyHostToDevice));
    std::vector<float> cie(30);
    memcpy(cie.data(), g_tables.cieX.data(), 40);
    memcpy(cie.data() + 10, g_tables.cieY.data(), 40);
    memcpy(cie.data() + 20, g_tables.cieZ.data(), 40);
    HIP_TRY(ctx, hipMemcpy(fr.cie, cie.data(), 30 * 4, hipMemcpyHostToDevice));
    // soil texture pair (synthetic stand-in for the missing blobs, scene_gen.h): level 0 uploaded,
    // the mip chain built by MipmapGen on the device, as init.cu:524-580 does for the PNGs
    {
        rtscene::TexturePair t;
        rtscene::make_textures(t);
        if (t.albedoAo.size() != (size_t)kTexTexels * 4) { ctx->err = "texture chain size mismatch"; return RT_ERR_STATE; }
        int rc2;
        if ((rc2 = rt_upload_texture(ctx, RT_TEX_SOIL_ALBEDO_AO, t.albedoAo.data(), kTexSize, kTexSize, 4)) != RT_OK ||
            (rc2 = rt_upload_texture(ctx, RT_TEX_SOIL_NORMAL_ROUGHNESS, t.normalRough.data(), kTexSize, kTexSize, 4)) != RT_OK)
            return rc2;
    }
    HIP_TRY(ctx, hipMemset(fr.color, 0, P * 8));
    HIP_TRY(ctx, hipMemset(fr.normal, 0, P * 8));
    HIP_TRY(ctx, hipMemset(fr.albedo, 0, P * 8));
    HIP_TRY(ctx, hipMemset(fr.depth, 0, P * 2));
    HIP_TRY(ctx, hipMemset(fr.motion, 0, P * 4));
    HIP_TRY(ctx, hipMemset(fr.rays, 0, P * 4));
    HIP_TRY(ctx, hipMemset(fr.ptStats, 0, P * 16));
    HIP_TRY(ctx, hipMemset(fr.rayCounter, 0, (size_t)kRayCounterSlots * kRayCounterStride * 8));
    HIP_TRY(ctx, hipMemset(fr.colorB, 0, P * 8));
    HIP_TRY(ctx, hipMemset(fr.accum, 0, P * 8));
    HIP_TRY(ctx, hipMemset(fr.histBuf[0], 0, P * 8));
    HIP_TRY(ctx, hipMemset(fr.histBuf[1], 0, P * 8));
    HIP_TRY(ctx, hipMemset(fr.histDepth, 0, P * 2));
    HIP_TRY(ctx, hipMemset(fr.histogram, 0, 256));
    const float exposure0[4] = {1.0f, 1.0f, 1.0f, 1.0f};  // init.cu:331-333
    HIP_TRY(ctx, hipMemcpy(fr.exposure, exposure0, 16, hipMemcpyHostToDevice));
    fr.renderColor = fr.color;
    fr.scaledColor = fr.scaledB;
    fr.ready = true;
    return RT_OK;
}

extern "C" {

// init.cu:524-580 for one texture of the atlas: its 16-bit level 0 (stbi_load_16 output, rows of
// width * channels ushorts) to the device, then GenerateMipmap (mipgen.cu:148-178) on the device
int rt_upload_texture(rt_context* ctx, int which, const uint16_t* texels, int width, int height, int channels) {
    if (!ctx || !texels) return RT_ERR_ARG;
    FrameResources& fr = ctx->fr;
    if (!fr.texAlbedo) { ctx->err = "rt_upload_texture before rt_init"; return RT_ERR_STATE; }
    uint16_t* chain = nullptr;
    int want = 4;
    switch (which) {
        case RT_TEX_SOIL_ALBEDO_AO: chain = (uint16_t*)fr.texAlbedo; break;
        case RT_TEX_SOIL_NORMAL_ROUGHNESS: chain = (uint16_t*)fr.texNormal; break;
        case RT_TEX_SOIL_HEIGHT: chain = fr.texHeight; want = 1; break;
        default: ctx->err = "rt_upload_texture: unknown texture"; return RT_ERR_ARG;
    }
    // the atlas is BUFFER_2D_1024x1024 with 11 levels (init.cu:526-528, texture.h:14-17), asserted there
    if (width != kTexSize || height != kTexSize || channels != want) {
        ctx->err = "rt_upload_texture: the soil textures are 1024 x 1024, 4 channels (height: 1)";
        return RT_ERR_ARG;
    }
    if (ctx->inited) {  // frames in flight may be sampling the old chain
        const int rc = sync_streams(ctx, false);
        if (rc != RT_OK) return rc;
    }
    HIP_TRY(ctx, hipMemcpyAsync(chain, texels, (size_t)width * height * channels * 2, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, rtk_launch_mipgen(chain, kTexSize, kTexLevels, channels, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

namespace {
// workspace slot k (1 .. kGbSets - 1): the camera outputs, and with `queues` the bounce queues with
// their hit records (slot 0 is fr.ws's own buffers); allocated once, full size
int alloc_ws_slot(rt_context* ctx, int k, bool queues) {
    FrameResources& fr = ctx->fr;
    int rc = RT_OK;
#define ALLOC(p, bytes) if (!(p) && (rc = dalloc(ctx, &(p), (bytes))) != RT_OK) return rc
    const size_t cap = fr.ws.cap, strip = (size_t)ctx->allocW * ctx->allocStripRows;
    ALLOC(fr.camHit0Rec[k], cap * 16);
    ALLOC(fr.camHit0Err[k], cap * 4);
    ALLOC(fr.camSurface[k], strip * 4);
    ALLOC(fr.camCount[k], kWsCounterWords * 4);
    if (queues) {
        for (PtQueue* q : {&fr.camQ3[k], &fr.camQ4[k]}) {
            ALLOC(q->rayO, cap * 16);
            ALLOC(q->rayD, cap * 16);
            ALLOC(q->st0, cap * 16);
            ALLOC(q->st1, cap * 16);
            ALLOC(q->st2, cap * 16);
        }
        ALLOC(fr.camHitRec[k], cap * 16);
        ALLOC(fr.camHitErr[k], cap * 4);
        ALLOC(fr.camPathL[k], cap * 16);
        ALLOC(fr.camPending[k], strip * 4);
    }
#undef ALLOC
    return rc;
}

// The launch parameters of frame `frame_num`'s path trace into G-buffer / camera-output set g, with
// that set's counter block (the serial frames' block, the stream plan and the bookkeeping are
// rt_path_trace's).  Zero-filled first, so that two calls with the same state compare equal byte
// for byte (the synchronous draws' camera rays traced ahead, launch_spec_camera).  Returns the
// bounce-queue slot.
int fill_pt_params(const rt_context* ctx, int frame_num, int with_detail, const HostCamera& hc, int g,
                   PathTraceParams& p) {
    const FrameResources& fr = ctx->fr;
    memset(&p, 0, sizeof p);
    p.cam = rt_trace_camera(hc);
    p.tanHalfFov[0] = hc.tanHalfFov[0];
    p.tanHalfFov[1] = hc.tanHalfFov[1];
    p.res[0] = hc.res[0];
    p.res[1] = hc.res[1];
    p.halfRes[0] = hc.res[0] / 2;
    p.halfRes[1] = hc.res[1] / 2;
    p.hist = fr.hist;
    p.width = (uint32_t)ctx->renderW;
    p.height = (uint32_t)ctx->renderH;
    p.y0 = (uint32_t)ctx->stripY0;
    p.rows = (uint32_t)ctx->stripRows;
    p.nStrips = (uint32_t)ctx->stripCount;
    p.strip = (uint32_t)ctx->stripIndex;
    p.frameNum = frame_num;
    p.spp = (uint32_t)ctx->spp;
    p.invSpp = (ctx->spp & (ctx->spp - 1)) == 0 ? 1.0f / (float)ctx->spp : 0.0f;  // exact for a power of two
    p.materialOverride = ctx->materialOverride;
    p.triCount = ctx->mesh.triCount;
    p.bluenoise = ctx->dBlueNoise;
    p.triPos = ctx->dTriPos;
    p.triNrm = ctx->dTriNrm;
    p.nodes = ctx->dNodes;
    p.tlasNodes = ctx->dTlasNodes;
    p.texAlbedo = fr.texAlbedo;
    p.texNormal = fr.texNormal;
    p.skyBuffer = fr.sky;
    p.sunBuffer = fr.sun;
    p.skyCdf = fr.skyCdf;
    p.sunCdf = fr.sunCdf;
    p.skyTree = fr.skyTree;
    p.sunTree = fr.sunTree;
    p.lightSel = fr.lightSel;
    memcpy(p.sunDir, fr.sunDir, 12);
    p.cosThetaMax = fr.cosThetaMax;
    p.oneMinusCosThetaMax = 1.0f - fr.cosThetaMax;
    sun_frame(fr.sunDir, p.sunT, p.sunB);
    p.colorOut = fr.gColor[g];
    p.normalOut = fr.gNormal[g];
    p.albedoOut = fr.gAlbedo[g];
    p.depthOut = fr.gDepth[g];
    p.motionOut = fr.gMotion[g];
    p.raysOut = with_detail ? fr.rays : nullptr;
    p.statsOut = with_detail ? fr.ptStats : nullptr;
    p.rayCounter = fr.rayCounter;
    p.ws = fr.ws;
    p.ws.hit0Rec = fr.camHit0Rec[g];
    p.ws.hit0Err = fr.camHit0Err[g];
    p.ws.surface = fr.camSurface[g];
    p.ws.counters = fr.camCount[g];
    p.ws.fetch = p.ws.counters + 64;
    const int qs = fr.camQ3[g].rayO ? g : 0;  // bounce-queue slot: per set when allocated (shadeOnSide)
    p.ws.q3 = fr.camQ3[qs];
    p.ws.q4 = fr.camQ4[qs];
    p.ws.hitRec = fr.camHitRec[qs];
    p.ws.hitErr = fr.camHitErr[qs];
    p.ws.pathL = fr.camPathL[qs];
    p.ws.pending = fr.camPending[qs];
    {  // material table (init.cu:215-251): only mirror / glass ids make steps 1-2 trace
        const int m = ctx->materialOverride;
        p.ws.glossy = m >= 0 && (m == 1 || m == 5 || m >= 10);
        p.ws.microfacet = m == 4;  // mat_type: only id 4 is MICROFACET, the reference table uses 3 / 6
    }
    return qs;
}

// Synchronous draws trace the next frame's camera rays ahead (launch_spec_camera): one GPU, no
// post stream, the G-buffer sets the context's own, [tuning] syncSpec
bool spec_on(const rt_context* ctx) {
    return ctx->tune.syncSpec && ctx->fr.specReady && !ctx->postStream && ctx->stripCount == 1 && !ctx->fr.gbBound;
}

// whether the camera and shade kernels launched with `a` wrote what ones launched with `b` would:
// the same parameters but for those they do not read (or that only select the later kernels)
bool spec_matches(const PathTraceParams& a, const PathTraceParams& b) {
    PathTraceParams x = a, y = b;
    for (PathTraceParams* q : {&x, &y}) {
        q->rayCounter = nullptr;  // the launches ahead count into specRayCounter
        // they read the LBVH set of the frame that launched them, the next frame reads the other:
        // the geometry is fixed after rt_init, so both hold the same build (tests/test_gpu_bvh.py)
        q->nodes = q->tlasNodes = nullptr;
        q->triPos = nullptr;
        q->triNrm = nullptr;
        q->ws.traceBlocks = 0;
        q->ws.shadeBlocksPerCu = 0;  // the shade's grid (dynamic claims: the same result on any grid)
        q->ws.countersZeroed = 0;
        q->ws.chain = 0;
        q->ws.q3HostOut = nullptr;
        q->ws.q3Tag = 0;
    }
    return memcmp(&x, &y, sizeof x) == 0;
}

// PtLaunchHook of a synchronous frame whose successor's camera rays are traced ahead: after
// kernel tune.specAfter (1 = shade) the gate they wait for
hipError_t spec_hook(void* arg, int kernel) {
    rt_context* ctx = (rt_context*)arg;
    return kernel == ctx->tune.specAfter ? hipEventRecord(ctx->specGate, ctx->stream) : hipSuccess;
}

}  // namespace

int rt_path_trace(rt_context* ctx, int frame_num, int with_detail) {
    if (!ctx || frame_num < 1) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_path_trace before rt_init"; return RT_ERR_STATE; }
    FrameResources& fr = ctx->fr;
    if (ctx->postStream) {  // frame pipelining: trace into the set no denoise still reads
        fr.gbSet = (fr.gbSet + 1) % kGbSets;
        select_gbuffers(fr);
        if (fr.setInFlight[fr.gbSet]) HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->postDone[fr.gbSet], 0));
    } else if (spec_on(ctx)) {  // synchronous frames alternate two sets: the next one's camera rays go ahead
        fr.gbSet ^= 1;
        select_gbuffers(fr);
    }
    int rc = update_sky(ctx);
    if (rc != RT_OK) return rc;
    HostCamera hc;
    rt_camera_update(ctx->camera, ctx->renderW, ctx->renderH, hc);
    if (frame_num == 1 || !fr.histValid) fr.hist = hist_of(hc);  // kernel.cu:133-136
    const int g = fr.gbSet;  // camera-output slot = G-buffer set
    PathTraceParams p;
    const int qs = fill_pt_params(ctx, frame_num, with_detail, hc, g, p);
    if (!ctx->postStream) {  // serial frames: the counter block the resolve before last zeroed
        const int b = fr.syncIdx;
        p.ws.counters = fr.syncCount[b];
        p.ws.countersZeroed = fr.syncZeroed[b] ? 1 : 0;
        p.ws.zeroNext = fr.syncCount[(b + 2) % 3];
        p.ws.fetch = p.ws.counters + 64;
        fr.syncZeroed[b] = fr.syncZeroed[(b + 2) % 3] = false;  // until this frame's resolve is enqueued
    }
    fr.lastCounters = p.ws.counters;
    fr.lastSlot = qs;
    // the fused bounce chain shortens a serial frame; pipelined frames keep the four lean kernels,
    // beside which the next frame's camera waves fit (k_pt_chain's 168 VGPRs at 3 waves/SIMD leave
    // them no room); on ranks of 8 strips too, since the queue tracers' refill-free tail loops
    // (0.436 vs 0.450 ms per rank frame)
    // ... and only while queue 3 is short: a long queue (the terrain view's 3.85 M rays) runs the
    // four kernels faster serially too (4.64 against 5.11 ms per synchronous terrain draw).  The
    // length is that of the last serial frame a host sync completed (q3Host, stored by the frame's
    // resolve kernel, read in sync_streams: a fixed schedule, no event on the stream).
    poll_q3(ctx);
    p.ws.chain = fr.ws.chain == 2 || (fr.ws.chain == 1 && !ctx->postStream && fr.lastQ3 < kChainMaxQ3);
    if (spec_on(ctx)) {  // beside the next frame's camera rays
        if (ctx->tune.specChain >= 0) p.ws.chain = ctx->tune.specChain != 0;  // A/B aid
        // fewer bounce-chain / queue-3 workgroups per CU leave the camera waves room beside them
        // (synchronous draw 0.985 -> 0.972 ms at 2 per CU against 3)
        if (ctx->tune.specTracePerCu > 0) p.ws.traceBlocks = fr.ws.cus * (uint32_t)ctx->tune.specTracePerCu;
    }
    fr.lastChain = p.ws.chain && !p.ws.glossy && !p.ws.microfacet;  // as rtk_launch_pt_rest decides
    if (with_detail) {  // per-pixel counters: everything in order on the context stream
        if (ctx->postStream && (rc = sync_streams(ctx)) != RT_OK) return rc;
        HIP_TRY(ctx, hipMemsetAsync(fr.rays, 0, (size_t)ctx->renderW * ctx->renderH * 4, ctx->stream));
        HIP_TRY(ctx, hipMemsetAsync(fr.ptStats, 0, (size_t)ctx->renderW * ctx->renderH * 16, ctx->stream));
    }
    // Frame pipelining: the camera rays go to the side stream behind this frame's LBVH build,
    // so they run beside the previous frame's trace tails; they wait only for the readers of
    // this slot's G-buffers (the denoise of frame f-2) and camera outputs (shade of frame f-2).
    const bool side = ctx->postStream && !with_detail;
    hipStream_t cs = side ? ctx->sideStream : ctx->stream;
    p.ws.shadeClaim = !ctx->postStream;  // dynamic batch claims in synchronous frames (pathtrace.hip)
    if (side) {
        if (fr.setInFlight[g]) HIP_TRY(ctx, hipStreamWaitEvent(cs, ctx->postDone[g], 0));
        if (fr.camInFlight[g]) HIP_TRY(ctx, hipStreamWaitEvent(cs, ctx->restDone[g], 0));
        if (ctx->cameraGated) HIP_TRY(ctx, hipStreamWaitEvent(cs, ctx->cameraGate, 0));
    } else if ((rc = wait_bvh(ctx)) != RT_OK) {
        return rc;
    }
    // rt_frame_marks_begin: this path trace's kernels are bracketed by events (caller's timed frames)
    hipEvent_t* const savedMarks = ctx->ptMarks;
    const bool ringSlot = !ctx->ptMarks && ctx->markNext < ctx->markFrames;
    if (ringSlot) ctx->ptMarks = ctx->markRing.data() + (size_t)(ctx->markNext++) * 2 * kFrameKernels;
    ctx->dnMarks = ctx->ptMarks ? ctx->ptMarks + 2 * kPtKernels : nullptr;  // for this frame's rt_denoise_post
    struct MarksReset {  // every return path leaves ptMarks as it found it
        rt_context* c;
        hipEvent_t* m;
        ~MarksReset() { c->ptMarks = m; }
    } marksReset{ctx, savedMarks};
    if (ringSlot)  // the slot's denoise pairs, recorded once here: a frame no rt_denoise_post follows
        for (int k = 2 * kPtKernels; k < 2 * kFrameKernels; ++k)  // reads 0 ms for them
            if (ctx->ptMarks[k]) HIP_TRY(ctx, hipEventRecord(ctx->ptMarks[k], cs));
    // the camera rays traced ahead by the previous synchronous draw: used when this launch would
    // write what they wrote, dropped otherwise; either way nothing after them runs before they end
    bool reuse = false, reuseShade = false;
    if (fr.spec.valid) {
        fr.spec.valid = false;
        HIP_TRY(ctx, hipStreamWaitEvent(cs, ctx->specDone, 0));
        reuse = !side && spec_matches(p, fr.spec.p);
        reuseShade = reuse && fr.spec.shade;
        if (!reuse) p.ws.countersZeroed = 0;  // their counts are in the block: the launcher clears it
        fr.specCounts = reuse ? 1 : 2;  // folded into the frame's (or cleared) ahead of the next ones
    }
    if (reuse) {
        for (int k = 0; k < (reuseShade ? 4 : 2) && ctx->ptMarks; ++k)  // zero-length slots for the marks
            if (ctx->ptMarks[k]) HIP_TRY(ctx, hipEventRecord(ctx->ptMarks[k], cs));
    } else {
        HIP_TRY(ctx, rtk_launch_pt_camera(&p, cs, ctx->ptMarks));
    }
    // the shade kernel follows on the side stream, so it runs beside the previous frame's queue
    // tracers instead of after them (its bounce queues are this set's own, camQ3[g] ..)
    const bool shadeSide = side && ctx->shadeOnSide && qs == g;
    if (shadeSide) HIP_TRY(ctx, rtk_launch_pt_shade(&p, cs, ctx->ptMarks));
    if (side) {
        HIP_TRY(ctx, hipEventRecord(ctx->camDone[g], cs));
        // overlapAfter 0: the previous frame's denoise waits only for that frame's path trace
        // (everything on the context stream so far), not for this frame's camera rays and shade
        if (ctx->overlapAfter == 0 && ctx->postPending) HIP_TRY(ctx, issue_overlapped_post(ctx));
        HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->camDone[g], 0));
    }
    PtLaunchHook hook{overlap_hook, ctx};
    const bool askQ3 = !side && !fr.q3Pending;  // serial frames: queue 3's length for the next chain choice
    if (askQ3) {
        if (!fr.q3Host) {
            HIP_TRY(ctx, hipHostMalloc((void**)&fr.q3Host, sizeof(unsigned long long), hipHostMallocDefault));
            *fr.q3Host = 0ull;
        }
        p.ws.q3HostOut = fr.q3Host;  // stored by k_pt_resolve (no copy on the stream)
        p.ws.q3Tag = ++fr.q3Tag;
    }
    PtLaunchHook shook{spec_hook, ctx};
    if (shadeSide) HIP_TRY(ctx, rtk_launch_pt_rest_after_shade(&p, ctx->stream, ctx->ptMarks, &hook));
    else if (reuseShade) HIP_TRY(ctx, rtk_launch_pt_rest_after_shade(&p, ctx->stream, ctx->ptMarks, &shook));
    else {
        const PtLaunchHook* h = ctx->postStream ? &hook : spec_on(ctx) && !with_detail ? &shook : nullptr;
        HIP_TRY(ctx, rtk_launch_pt_rest(&p, ctx->stream, ctx->ptMarks, h));
    }
    // pending only once the launches that store it are enqueued: a failed launch leaves the next
    // serial frame to ask again instead of freezing the chain choice
    if (askQ3) fr.q3Pending = true;
    if (!ctx->postStream) {  // block b + 2 is zeroed by this frame's resolve, enqueued above
        const int b = fr.syncIdx;
        fr.syncZeroed[(b + 2) % 3] = true;
        fr.syncIdx = (b + 1) % 3;
    }
    if (ctx->postPending && (rc = issue_pending_post(ctx)) != RT_OK) return rc;
    if (ctx->postStream) {
        HIP_TRY(ctx, hipEventRecord(ctx->restDone[g], ctx->stream));
        fr.camInFlight[g] = true;
        HIP_TRY(ctx, hipEventRecord(ctx->bvhFree[ctx->bvhSet], ctx->stream));
        ctx->bvhInFlight[ctx->bvhSet] = true;
    }
    fr.renderColor = fr.color;
    fr.hist = hist_of(hc);  // HistoryCamera::Setup after PathTrace (kernel.cu:357)
    fr.histValid = true;
    ctx->lastFrame = frame_num;
    return RT_OK;
}

int rt_get_ray_count(rt_context* ctx, uint64_t* rays, int reset) {
    if (!ctx || !rays) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_get_ray_count before rt_init"; return RT_ERR_STATE; }
    if (int rc = sync_streams(ctx)) return rc;  // the side stream's camera and shade kernels add rays too
    std::vector<unsigned long long> part((size_t)kRayCounterSlots * kRayCounterStride);
    const size_t bytes = part.size() * 8;
    HIP_TRY(ctx, hipMemcpy(part.data(), ctx->fr.rayCounter, bytes, hipMemcpyDeviceToHost));
    unsigned long long v = 0;
    for (int k = 0; k < kRayCounterSlots; ++k) v += part[(size_t)k * kRayCounterStride];
    *rays = v;
    if (reset) HIP_TRY(ctx, hipMemset(ctx->fr.rayCounter, 0, bytes));
    return RT_OK;
}

// TemporalSpatialDenoising + PostProcessing + CopyToOutput for the frame just path traced
int rt_denoise_post(rt_context* ctx, int frame_num, int with_hdr) {
    if (!ctx || frame_num < 1) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_denoise_post before rt_init"; return RT_ERR_STATE; }
    const rt_render_pass_settings& ps = ctx->params.pass;
    if (ps.enablePostProcess && ps.enableToneMapping &&
        (ctx->params.post.toneMappingType < 0 || ctx->params.post.toneMappingType > 3)) {
        ctx->err = "toneMappingType must be 0 (Uncharted), 1 (ACES1), 2 (ACES2) or 3 (Reinhard)";
        return RT_ERR_ARG;
    }
    FrameResources& fr = ctx->fr;
    DenoisePostParams p;
    p.W = (uint32_t)ctx->renderW;
    p.H = (uint32_t)ctx->renderH;
    p.Ws = (uint32_t)ctx->screenW;
    p.Hs = (uint32_t)ctx->screenH;
    p.frameNum = frame_num;
    p.histW = (uint32_t)ctx->histW;
    p.histH = (uint32_t)ctx->histH;
    p.deltaTime = frame_delta(ctx);
    p.temporal = ps.enableTemporalDenoising;
    p.localSpatial = ps.enableLocalSpatialFilter;
    p.visualize = ps.enableNoiseLevelVisualize;
    p.wideSpatial = ps.enableWideSpatialFilter;
    p.temporal2 = ps.enableTemporalDenoising2;
    p.postProcess = ps.enablePostProcess;
    p.downScale = ps.enableDownScalePasses;
    p.histogramOn = ps.enableHistogram;
    p.autoExposure = ps.enableAutoExposure;
    p.sharpen = ps.enableSharpening;
    p.tonemap = ps.enableToneMapping;
    p.gain = ctx->params.post.gain;
    p.fixedExposure = ctx->params.post.exposure;
    p.maxWhite = ctx->params.post.maxWhite;
    p.gamma = ctx->params.post.gamma;
    p.dn = ctx->params.denoise;
    {  // the depth weights' divisors as reciprocals (rtmath.h rt_div_rcp), where that is exact
        const float sig[3] = {p.dn.temporal_denoise_sigma_depth, p.dn.local_denoise_sigma_depth,
                              p.dn.large_denoise_sigma_depth};
        p.rcpDepthOk = 0;
        for (int k = 0; k < 3; ++k) {
            volatile float d = sig[k];  // the IEEE reciprocal, as the oracle's check computes it
            p.rcpDepth[k] = 1.0f / d;
            if (rt_div_rcp_ok(sig[k])) p.rcpDepthOk |= 1 << k;
        }
    }
    p.colorA = fr.color;
    p.colorB = fr.colorB;
    p.normal = fr.normal;
    p.albedo = fr.albedo;
    p.depth = fr.depth;
    p.motion = fr.motion;
    p.accum = fr.accum;
    p.histColor = fr.histBuf[fr.histIdx];
    p.histColorOut = fr.histBuf[fr.histIdx ^ 1];
    p.histOutSet = fr.histIdx ^ 1;
    p.gbSet = fr.gbSet;
    p.ty0 = 0;
    p.ty1 = (int)((p.H + 15) / 16);
    {  // multi-GPU strip-local denoise: only with a collective hook, and for the passes it covers
        uint32_t a = 0, b = p.H;
        p.stripLocal = strip_local_denoise(ctx, a, b) ? 1 : 0;
        // the list passes at two threads per pixel ([tuning] dnSplit: 0 never, 1 synchronous frames
        // only, 2 always): in pipelined frames their 512-thread workgroups wait for room beside the
        // next frame's camera and shade waves (A/B in DESIGN.md §4.2)
        p.listSplit = ctx->tune.dnSplit == 2 || (ctx->tune.dnSplit == 1 && !ctx->postStream) ? 1 : 0;
        p.listFold = ctx->tune.dnFold ? 1 : 0;
        p.rowA = a;
        p.rowB = b;
    }
    p.histDepth = fr.histDepth;
    p.noise8 = fr.noise8;
    p.noise16 = fr.noise16;
    p.chainCounter = fr.chainCounter;
    p.tileList = fr.tileList;
    p.tileCap = fr.tileCap;
    p.tileParity = fr.tileParity;
    p.listUsed = 0;
    p.exposureDone = 0;
    p.histDepthInTemporal = 0;
    p.c4 = fr.c4;
    p.c16 = fr.c16;
    p.c64 = fr.c64;
    p.histogram = fr.histogram;
    p.exposure = fr.exposure;
    p.scaledA = fr.scaledA;
    p.scaledB = fr.scaledB;
    // rt_draw_device: the caller's device target; a strip-local denoise writes its rows into the
    // exchanged buffer instead and copies the whole frame to the target after the rows exchange
    p.rgbaTarget = (p.stripLocal && fr.drawTarget) ? fr.drawTarget : nullptr;
    p.rgbaTargetPitch = fr.drawTarget ? fr.drawPitch : 0u;
    p.rgba = (fr.drawTarget && !p.stripLocal) ? fr.drawTarget : fr.rgba;
    p.rgbaPitch = (fr.drawTarget && !p.stripLocal) ? fr.drawPitch : (uint32_t)ctx->screenW;
    fr.outRgba = fr.drawTarget ? fr.drawTarget : fr.rgba;
    fr.outPitch = fr.drawTarget ? fr.drawPitch : (uint32_t)ctx->screenW;
    p.bluenoise = ctx->dBlueNoise;
    p.hdrOut = with_hdr ? fr.hdr : nullptr;
    p.marks = ctx->dnMarks;  // the frame's denoise marks (rt_frame_marks_begin / rt_time_frame_kernels)
    ctx->dnMarks = nullptr;
    p.bloom = ps.enablePostProcess && ps.enableBloomEffect;
    p.toneMappingType = ctx->params.post.toneMappingType;
    p.bloom4 = fr.bloom4;
    p.bloom16 = fr.bloom16;
    p.lensFlare = 0;
    p.sunPos[0] = p.sunPos[1] = 0.0f;
    p.sunUv[0] = p.sunUv[1] = 0;
    if (ps.enablePostProcess && ps.enableLensFlare) {
        // UpdateFrame's sunPos / sunUv (kernel.cu:126-127): Camera::WorldToScreenSpace(pos + sunDir)
        HostCamera hc;
        rt_camera_update(ctx->camera, ctx->renderW, ctx->renderH, hc);
        const V3 pos = v3(hc.pos[0], hc.pos[1], hc.pos[2]);
        const V3 sd = v3(fr.sunDir[0], fr.sunDir[1], fr.sunDir[2]);
        const V3 w = pos + sd;
        const V3 d = v3(w.x - pos.x, w.y - pos.y, w.z - pos.z);
        const V3 vs = v3(dot(v3(hc.left[0], hc.left[1], hc.left[2]), d), dot(v3(hc.up[0], hc.up[1], hc.up[2]), d),
                         dot(v3(hc.dir[0], hc.dir[1], hc.dir[2]), d));
        const float sx = vs.x / vs.z, sy = vs.y / vs.z;
        const float nx = sx / hc.tanHalfFov[0], ny = sy / hc.tanHalfFov[1];
        float px = 0.5f - nx * 0.5f, py = 0.5f - ny * 0.5f;
        const int ux = (int)floorf(px * (float)ctx->renderW), uy = (int)floorf(py * (float)ctx->renderH);
        // PostProcessing's predicate (postprocessing.cu:90)
        if (px > 0 && px < 1 && py > 0 && py < 1 && sd.y > -0.0f &&
            dot(sd, v3(hc.dir[0], hc.dir[1], hc.dir[2])) > 0) {
            px -= 0.5f;
            py -= 0.5f;
            px *= (float)ctx->renderW / (float)ctx->renderH;
            p.lensFlare = 1;
            p.sunPos[0] = px;
            p.sunPos[1] = py;
            p.sunUv[0] = ux;
            p.sunUv[1] = uy;
        }
    }
    if (ctx->postStream) {
        // deferred: enqueued behind the next path trace's first kernels (overlap_hook) or at the
        // next host read; it waits for everything enqueued so far on the context stream (this
        // frame's path trace and any G-buffer gathers)
        int rc = issue_pending_post(ctx);
        if (rc != RT_OK) return rc;
        HIP_TRY(ctx, hipEventRecord(ctx->ptDone[fr.gbSet], ctx->stream));
        ctx->postGather = ctx->gatherOn;
        if (ctx->postGather) HIP_TRY(ctx, hipEventRecord(ctx->gatherDone[fr.gbSet], ctx->gatherStream));
        ctx->postParams = p;
        ctx->postPendingSet = fr.gbSet;
        ctx->postPending = true;
        fr.setInFlight[fr.gbSet] = true;
    } else {
        if (ctx->gatherOn) {
            HIP_TRY(ctx, hipEventRecord(ctx->gatherDone[0], ctx->gatherStream));
            HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->gatherDone[0], 0));
        }
        if (int rc = run_denoise(ctx, p, ctx->stream)) return rc;
        fr.renderColor = p.finalColor;
        fr.scaledColor = p.finalScaled;
    }
    if (p.temporal2) fr.histIdx ^= 1;
    ctx->histW = ctx->renderW;  // the history buffers now hold this frame's size
    ctx->histH = ctx->renderH;
    return RT_OK;
}

// the last frame's RGBA8 (screen size) into tightly packed host memory; waits for the frame
int copy_rgba_out(rt_context* ctx, void* dst) {
    if (int rc = sync_streams(ctx)) return rc;
    const FrameResources& fr = ctx->fr;
    const size_t row = (size_t)ctx->screenW * 4;
    HIP_TRY(ctx, hipMemcpy2D(dst, row, fr.outRgba, (size_t)fr.outPitch * 4, row, (size_t)ctx->screenH,
                             hipMemcpyDeviceToHost));
    return RT_OK;
}

namespace {
// Synchronous draws: the next frame's LBVH rebuild (BuildBvhLevel1/2, one per frame as in the
// reference) goes into the other set on the side stream, where it runs beside this frame's
// denoise instead of ahead of the next frame's path trace.  The geometry is fixed after rt_init,
// so the build depends on nothing this frame computes; the other set was last read by the
// previous frame, which has finished.
int prebuild_next_bvh(rt_context* ctx) {
    int rc;
    if ((rc = ensure_bvh_pair(ctx)) != RT_OK) return rc;
    const int cur = ctx->bvhSet;
    bvh_select(ctx, cur ^ 1);
    hipStream_t keep = ctx->stream;  // no post stream: rt_build_bvh builds on ctx->stream
    ctx->stream = ctx->sideStream;
    rc = rt_build_bvh(ctx);
    ctx->stream = keep;
    if (rc == RT_OK) {
        if (hipEventRecord(ctx->buildDone[cur ^ 1], ctx->sideStream) != hipSuccess) {
            ctx->err = "hipEventRecord (LBVH prebuild)";
            rc = RT_ERR_HIP;
        }
        ctx->buildOnSide[cur ^ 1] = true;
    }
    bvh_select(ctx, cur);
    ctx->bvhPrebuilt = rc == RT_OK;
    return rc;
}

// Set 1's G-buffers and camera outputs and the events of the synchronous draws' camera rays traced
// ahead (allocated at full size, once)
int ensure_sync_spec(rt_context* ctx) {
    FrameResources& fr = ctx->fr;
    int rc;
    const size_t P = (size_t)ctx->allocW * ctx->allocH;
#define ALLOC(p, bytes) if (!(p) && (rc = dalloc(ctx, &(p), (bytes))) != RT_OK) return rc
    ALLOC(fr.gColor[1], P * 8);
    ALLOC(fr.gNormal[1], P * 8);
    ALLOC(fr.gAlbedo[1], P * 8);
    ALLOC(fr.gDepth[1], P * 2);
    ALLOC(fr.gMotion[1], P * 4);
#undef ALLOC
    if ((rc = alloc_ws_slot(ctx, 1, true)) != RT_OK) return rc;  // with bounce queues: the shade goes ahead too
    if (!fr.specRayCounter) {  // zero between uses (rtk_fold_ray_counts)
        if ((rc = dalloc(ctx, &fr.specRayCounter, (size_t)kRayCounterSlots * kRayCounterStride * 8)) != RT_OK) return rc;
        HIP_TRY(ctx, hipMemset(fr.specRayCounter, 0, (size_t)kRayCounterSlots * kRayCounterStride * 8));
    }
    for (hipEvent_t* e : {&ctx->specGate, &ctx->specDone})
        if (!*e) HIP_TRY(ctx, hipEventCreateWithFlags(e, hipEventDisableTiming));
    fr.specReady = true;
    return RT_OK;
}

// Synchronous draws: the next frame's camera rays, traced ahead on the side stream after this
// frame's shade kernel (spec_hook) and ahead of the next frame's LBVH build (prebuild_next_bvh), on
// this frame's LBVH, into the other G-buffer set and the next counter block, with the camera, sky
// and frame number as they are now.
// They then run beside this frame's bounces and denoise instead of at the head of the next draw.
// The next rt_path_trace uses them only when its own launch parameters equal these (spec_matches:
// a host that moves the camera, changes the sky, the size or the frame number between the draws
// gets them traced again), and any call that waits for the streams drops them, so no draw's output
// depends on this.
int launch_spec_camera(rt_context* ctx) {
    FrameResources& fr = ctx->fr;
    if (!ctx->tune.syncSpec || ctx->postStream || ctx->stripCount != 1 || fr.gbBound) return RT_OK;
    int rc;
    if (!fr.specReady && (rc = ensure_sync_spec(ctx)) != RT_OK) return rc;
    HostCamera hc;
    rt_camera_update(ctx->camera, ctx->renderW, ctx->renderH, hc);
    PathTraceParams p;  // on this frame's LBVH set (spec_matches)
    fill_pt_params(ctx, ctx->nextFrame, 0, hc, fr.gbSet ^ 1, p);
    const int b = fr.syncIdx;
    p.ws.counters = fr.syncCount[b];
    p.ws.countersZeroed = fr.syncZeroed[b] ? 1 : 0;
    p.ws.zeroNext = fr.syncCount[(b + 2) % 3];
    p.ws.fetch = p.ws.counters + 64;
    p.ws.shadeClaim = 1;  // as rt_path_trace sets it for synchronous frames
    p.rayCounter = fr.specRayCounter;
    if (fr.specCounts) {  // the last launches' ray counts: into the frame's if they were used, then cleared
        HIP_TRY(ctx, rtk_fold_ray_counts(fr.specCounts == 1 ? fr.rayCounter : nullptr, fr.specRayCounter, ctx->sideStream));
        fr.specCounts = 0;
    }
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->sideStream, ctx->specGate, 0));
    HIP_TRY(ctx, rtk_launch_pt_camera(&p, ctx->sideStream, nullptr));
    // then the next frame's shade kernel, which runs beside this frame's denoise (synchronous draw
    // 0.969 -> 0.945 ms, the terrain view 3.70 -> 3.33 ms), on 2 workgroups per CU so that the
    // denoise passes' workgroups fit beside it (0.942 -> 0.935 ms)
    const bool shade = ctx->tune.specShade == 2 || (ctx->tune.specShade == 1 && !fr.lastChain);
    if (shade) {
        if (ctx->tune.specShadePerCu > 0) p.ws.shadeBlocksPerCu = (uint32_t)ctx->tune.specShadePerCu;
        HIP_TRY(ctx, rtk_launch_pt_shade(&p, ctx->sideStream, nullptr));
    }
    HIP_TRY(ctx, hipEventRecord(ctx->specDone, ctx->sideStream));
    fr.syncZeroed[b] = false;
    fr.spec.valid = true;
    fr.spec.shade = shade;
    fr.spec.block = b;
    fr.spec.p = p;
    return RT_OK;
}

// UpdateFrame (kernel.cu:61-137) + BuildBvhLevel1/2 + PathTrace + TemporalSpatialDenoising +
// PostProcessing + CopyToOutput of one frame, enqueued (draw, kernel.cu:259-398); the RGBA8 image
// goes to `target` (pitch in pixels) or, when NULL, to the context's own buffer
int enqueue_frame(rt_context* ctx, uint32_t* target, uint32_t pitch, bool hdr) {
    const int frame = ctx->nextFrame++;
    int rc;
    ctx->fr.drawDt = -1.0f;
    const float dt = frame_delta(ctx);  // UpdateFrame's timer, read once per frame
    if (ctx->useDynamicResolution && frame > 1 && ctx->fullFrame) update_dynamic_resolution(ctx, dt);
    rt_input_control_update(ctx, dt);  // UpdateFrame's InputControlUpdate (kernel.cu:117)
    ctx->fr.drawDt = dt;
    if (ctx->bvhPrebuilt && !ctx->postStream) {  // built beside the previous synchronous frame
        ctx->bvhPrebuilt = false;
        bvh_select(ctx, ctx->bvhSet ^ 1);  // the path trace waits for its build (wait_bvh)
    } else if ((rc = rt_build_bvh(ctx)) != RT_OK) {
        return rc;
    }
    if ((rc = rt_path_trace(ctx, frame, 0)) != RT_OK) return rc;
    // the next frame's camera rays first on the side stream, then its LBVH (which only its bounces read)
    if (!ctx->postStream && (rc = launch_spec_camera(ctx)) != RT_OK) return rc;
    if (!ctx->postStream && (rc = prebuild_next_bvh(ctx)) != RT_OK) return rc;
    ctx->fr.drawTarget = target;
    ctx->fr.drawPitch = pitch;
    rc = rt_denoise_post(ctx, frame, hdr ? 1 : 0);
    ctx->fr.drawTarget = nullptr;
    return rc;
}
}  // namespace

// RayTracer::draw (kernel.cu:259-398) with host outputs: BVH rebuild, path trace, denoise, post,
// output, then the copies to the caller's host buffers
int rt_draw(rt_context* ctx, uint8_t* rgba8_out, float* hdr_out) {
    if (!ctx) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_draw before rt_init"; return RT_ERR_STATE; }
    int rc;
    if ((rc = enqueue_frame(ctx, nullptr, 0, hdr_out != nullptr)) != RT_OK) return rc;
    if ((rc = sync_draw(ctx)) != RT_OK) return rc;
    if (rgba8_out && (rc = copy_rgba_out(ctx, rgba8_out)) != RT_OK) return rc;
    if (hdr_out)
        HIP_TRY(ctx, hipMemcpy(hdr_out, ctx->fr.hdr, (size_t)ctx->renderW * ctx->renderH * 16, hipMemcpyDeviceToHost));
    return RT_OK;
}

// RayTracer::draw(SurfObj* renderTarget) (kernel.cu:259, CopyToOutput kernel.cu:26-59): the frame's
// RGBA8 image is written straight into caller-owned device memory.  RT_DRAW_ASYNC returns once the
// frame is enqueued and runs the frame pipeline (an internal post stream unless the caller set one).
int rt_draw_device(rt_context* ctx, void* rgba8_device, size_t pitch_bytes, int flags) {
    if (!ctx || !rgba8_device) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_draw_device before rt_init"; return RT_ERR_STATE; }
    const size_t row = (size_t)ctx->screenW * 4;
    if (pitch_bytes == 0) pitch_bytes = row;
    if (pitch_bytes < row || pitch_bytes % 4 != 0 || ((uintptr_t)rgba8_device & 3u) != 0) {
        ctx->err = "rt_draw_device: pitch must be >= screen width * 4 and a multiple of 4, target 4-byte aligned";
        return RT_ERR_ARG;
    }
    if ((flags & ~RT_DRAW_ASYNC) != 0) { ctx->err = "rt_draw_device: unknown flags"; return RT_ERR_ARG; }
    int rc;
    if ((flags & RT_DRAW_ASYNC) && !ctx->postStream) {  // pipelined frames on an internal low-priority stream
        if (!ctx->ownPostStream && (rc = rt_create_stream(ctx, &ctx->ownPostStream, false)) != RT_OK) return rc;
        if ((rc = rt_set_post_stream(ctx, ctx->ownPostStream)) != RT_OK) return rc;
    }
    if ((rc = enqueue_frame(ctx, (uint32_t*)rgba8_device, (uint32_t)(pitch_bytes / 4), false)) != RT_OK) return rc;
    if (!(flags & RT_DRAW_ASYNC)) return sync_draw(ctx);  // draw ends with a device sync (kernel.cu:393-397)
    return RT_OK;
}

int rt_set_stream(rt_context* ctx, void* stream) {
    if (!ctx) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_set_stream before rt_init"; return RT_ERR_STATE; }
    int rc = sync_streams(ctx, false);
    if (rc != RT_OK) return rc;
    ctx->stream = stream == RT_OWN_STREAM ? ctx->ownStream : (hipStream_t)stream;  // NULL: the null stream
    return RT_OK;
}

int rt_set_collective_hook(rt_context* ctx, rt_collective_fn fn, void* arg) {
    if (!ctx) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_set_collective_hook before rt_init"; return RT_ERR_STATE; }
    int rc = sync_streams(ctx, false);
    if (rc != RT_OK) return rc;
    ctx->hook = fn;
    ctx->hookArg = arg;
    return RT_OK;
}

int rt_set_hook_stages(rt_context* ctx, uint32_t stage_mask) {
    if (!ctx || (stage_mask & ~7u) != 0) return RT_ERR_ARG;
    // HISTOGRAM and ROWS are what make a strip-local denoise equal one GPU's: a mask without them
    // would leave each rank with its own exposure and stale peer rows, so it is refused
    const uint32_t need = (1u << RT_HOOK_HISTOGRAM) | (1u << RT_HOOK_ROWS);
    if ((stage_mask & need) != need) {
        ctx->err = "rt_set_hook_stages: HISTOGRAM and ROWS are mandatory; the mask only opts into GBUFFERS";
        return RT_ERR_ARG;
    }
    ctx->hookStages = stage_mask;
    return RT_OK;
}

int rt_set_gather_stream(rt_context* ctx, void* stream) {
    if (!ctx) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_set_gather_stream before rt_init"; return RT_ERR_STATE; }
    int rc = sync_streams(ctx, false);
    if (rc != RT_OK) return rc;
    for (int k = 0; k < kGbSets; ++k)
        if (!ctx->gatherDone[k]) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->gatherDone[k], hipEventDisableTiming));
    ctx->gatherOn = stream != RT_STREAM_OFF;  // NULL is the null stream, as in rt_set_stream
    ctx->gatherStream = ctx->gatherOn ? (hipStream_t)stream : nullptr;
    return RT_OK;
}

// The second LBVH set, the side stream and the build events: frame f+1's build beside frame f
// (pipelined frames, and the prebuild of synchronous draws)
int ensure_bvh_pair(rt_context* ctx) {
    int rc;
#define ALLOC(p, bytes) if (!(p) && (rc = dalloc(ctx, &(p), (bytes))) != RT_OK) return rc
    {
        const size_t NP = ctx->mesh.triCountPadded, B = ctx->B;
        BvhBufs& b = ctx->bvh[1];
        if (!b.nodes) {  // the record arena (traverse.h), as in rt_init
            ALLOC(b.nodes, arena_bytes(B, NP));
            HIP_TRY(ctx, hipMemset(b.nodes, 0, arena_bytes(B, NP)));
            b.tlasNodes = (char*)b.nodes + B * 1024 * 64;
            b.triPos = (float4*)((char*)b.nodes + (B * 1024 + B) * 64);
        }
        ALLOC(b.triNrm, NP * 48);
        ALLOC(b.aabbs, NP * 24);
        ALLOC(b.batchScene, B * 24);
        ALLOC(b.morton, B * 4096);
        ALLOC(b.reorder, B * 4096);
        ALLOC(b.tlasAabbs, B * 24);
        ALLOC(b.tlasScene, 24);
        ALLOC(b.tlasMorton, 4096);
        ALLOC(b.tlasReorder, 4096);
        if (!b.counter) {
            ALLOC(b.counter, 64);
            HIP_TRY(ctx, hipMemset(b.counter, 0, 64));
        }
    }
#undef ALLOC
    // lowest priority: it should fill what the trace chain leaves idle
    if (!ctx->sideStream && (rc = rt_create_stream(ctx, &ctx->sideStream, false)) != RT_OK) return rc;
    for (hipEvent_t* e : {&ctx->buildDone[0], &ctx->buildDone[1], &ctx->bvhFree[0], &ctx->bvhFree[1]})
        if (!*e) HIP_TRY(ctx, hipEventCreateWithFlags(e, hipEventDisableTiming));
    return RT_OK;
}

int rt_set_post_stream(rt_context* ctx, void* stream) {
    if (!ctx) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_set_post_stream before rt_init"; return RT_ERR_STATE; }
    int rc = sync_streams(ctx, false);
    if (rc != RT_OK) return rc;
    FrameResources& fr = ctx->fr;
    for (int k = 0; k < kGbSets; ++k) fr.setInFlight[k] = false;
    fr.syncZeroed[0] = fr.syncZeroed[1] = fr.syncZeroed[2] = false;  // pipelined frames use (and dirty) camCount[0] too
    if (!stream) {
        ctx->postStream = nullptr;
        return RT_OK;
    }
    // sized for the largest frame: with dynamic resolution the current size may be smaller and
    // grow back later
    const size_t P = (size_t)ctx->allocW * ctx->allocH;
#define ALLOC(p, bytes) if (!(p) && (rc = dalloc(ctx, &(p), (bytes))) != RT_OK) return rc
    for (int k = 1; k < kGbSets; ++k) {  // further G-buffer sets and camera-output slots
        ALLOC(fr.gColor[k], P * 8);
        ALLOC(fr.gNormal[k], P * 8);
        ALLOC(fr.gAlbedo[k], P * 8);
        ALLOC(fr.gDepth[k], P * 2);
        ALLOC(fr.gMotion[k], P * 4);
        if ((rc = alloc_ws_slot(ctx, k, false)) != RT_OK) return rc;
    }
    // the shade kernel runs on the side stream, with bounce queues per set ([tuning] shadeOnSide:
    // A/B aid); measured: one GPU 1.025 -> 0.970 ms/frame, one rank's share at
    // 2 / 4 / 8 ranks 0.648 -> 0.650 / 0.495 -> 0.482 / 0.453 -> 0.411 ms
    ctx->shadeOnSide = ctx->tune.shadeOnSide;
    for (int k = 1; ctx->shadeOnSide && k < kGbSets; ++k)
        if ((rc = alloc_ws_slot(ctx, k, true)) != RT_OK) return rc;
#undef ALLOC
    if ((rc = ensure_bvh_pair(ctx)) != RT_OK) return rc;
    for (int k = 0; k < kGbSets; ++k) {
        if (!ctx->camDone[k]) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->camDone[k], hipEventDisableTiming));
        if (!ctx->restDone[k]) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->restDone[k], hipEventDisableTiming));
        fr.camInFlight[k] = false;
    }
    ctx->bvhInFlight[0] = ctx->bvhInFlight[1] = false;
    ctx->buildOnSide[0] = ctx->buildOnSide[1] = false;
    for (int k = 0; k < kGbSets; ++k) {
        if (!ctx->ptDone[k]) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->ptDone[k], hipEventDisableTiming));
        if (!ctx->postDone[k]) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->postDone[k], hipEventDisableTiming));
    }
    if (!ctx->overlapEv) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->overlapEv, hipEventDisableTiming));
    if (!ctx->cameraGate) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->cameraGate, hipEventDisableTiming));
    ctx->cameraGated = false;
    // the next frame's camera rays: ungated on one GPU (they run beside this frame's shade and
    // queue-3 traversal), after this frame's trace<3> on two GPUs and its resume<3> on four, where
    // a rank's tails are shorter, and after its shade on eight (measured per N: DESIGN.md §7)
    ctx->cameraAfter = ctx->stripCount == 1 ? 0 : ctx->stripCount == 2 ? 2 : ctx->stripCount < 8 ? 3 : 1;
    if (ctx->tune.overlapAfter >= 0) ctx->overlapAfter = ctx->tune.overlapAfter;  // [tuning] A/B aids
    if (ctx->tune.cameraAfter >= 0) ctx->cameraAfter = ctx->tune.cameraAfter;
    ctx->postStream = (hipStream_t)stream;
    return RT_OK;
}

int rt_bind_buffer(rt_context* ctx, int name, void* device_ptr, size_t bytes) {
    if (!ctx || !device_ptr) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_bind_buffer before rt_init"; return RT_ERR_STATE; }
    const int set = (name >> 8) & 3;  // RT_BUF_SET1 / RT_BUF_SET2 / RT_BUF_SET3
    name &= 0xFF;
    if (set >= kGbSets) { ctx->err = "rt_bind_buffer: no such G-buffer set"; return RT_ERR_ARG; }
    const size_t need = rt_alloc_bytes(ctx, name);  // later frames may be larger than the current one
    if (need == 0 || bytes < need) { ctx->err = "rt_bind_buffer: unknown buffer or too small"; return RT_ERR_ARG; }
    if (((uintptr_t)device_ptr & 15u) != 0) { ctx->err = "rt_bind_buffer: pointer must be 16-byte aligned"; return RT_ERR_ARG; }
    int rc = sync_streams(ctx, false);
    if (rc != RT_OK) return rc;
    FrameResources& fr = ctx->fr;
    switch (name) {
        case RT_BUF_RENDER_COLOR: fr.gColor[set] = (uint2*)device_ptr; break;
        case RT_BUF_NORMAL: fr.gNormal[set] = (uint2*)device_ptr; break;
        case RT_BUF_ALBEDO: fr.gAlbedo[set] = (uint2*)device_ptr; break;
        case RT_BUF_DEPTH: fr.gDepth[set] = (uint16_t*)device_ptr; break;
        case RT_BUF_MOTION: fr.gMotion[set] = (uint32_t*)device_ptr; break;
        // the strip-local denoise's exchanged buffers (set 0 only, except the history pair 0 / 1);
        // the new memory takes over the old contents (a frame-persistent state)
        case RT_BUF_ACCUMULATION:
        case RT_BUF_HISTORY_COLOR:
        case RT_BUF_HISTOGRAM:
        case RT_BUF_RGBA8: {
            if (set > (name == RT_BUF_HISTORY_COLOR ? 1 : 0)) { ctx->err = "rt_bind_buffer: no such set"; return RT_ERR_ARG; }
            void** slot = name == RT_BUF_ACCUMULATION ? (void**)&fr.accum
                          : name == RT_BUF_HISTORY_COLOR ? (void**)&fr.histBuf[set]
                          : name == RT_BUF_HISTOGRAM ? (void**)&fr.histogram : (void**)&fr.rgba;
            HIP_TRY(ctx, hipMemcpy(device_ptr, *slot, need, hipMemcpyDeviceToDevice));
            if (name == RT_BUF_RGBA8 && fr.outRgba == fr.rgba) fr.outRgba = (uint32_t*)device_ptr;
            // a caller-owned accumulation buffer stays the accumulation buffer: the list chain
            // writes the internal one and copies its rows back instead of swapping the two
            if (name == RT_BUF_ACCUMULATION) fr.accumBound = true;
            *slot = device_ptr;
            return RT_OK;
        }
        default: ctx->err = "rt_bind_buffer: this buffer cannot be bound"; return RT_ERR_ARG;
    }
    fr.gbBound = true;  // synchronous frames then stay in their set (no camera rays traced ahead)
    if (set == fr.gbSet) select_gbuffers(fr);
    return RT_OK;
}

// bytes a render-size buffer has at the allocation (maximum) size
size_t rt_alloc_bytes(const rt_context* ctx, int name) {
    const size_t P = (size_t)ctx->allocW * ctx->allocH;
    switch (name) {
        case RT_BUF_RENDER_COLOR: case RT_BUF_NORMAL: case RT_BUF_ALBEDO: case RT_BUF_ACCUMULATION:
        case RT_BUF_HISTORY_COLOR: return P * 8;
        case RT_BUF_HISTOGRAM: return 256;
        case RT_BUF_RGBA8: return (size_t)ctx->screenW * ctx->screenH * 4;
        case RT_BUF_DEPTH: return P * 2;
        case RT_BUF_MOTION: return P * 4;
        default: return 0;
    }
}

size_t rt_buffer_bytes(const rt_context* ctx, int name) {
    if (!ctx) return 0;
    const size_t P = (size_t)ctx->renderW * ctx->renderH;
    switch (name) {
        case RT_BUF_RENDER_COLOR: case RT_BUF_NORMAL: case RT_BUF_ALBEDO: case RT_BUF_ACCUMULATION:
        case RT_BUF_HISTORY_COLOR: return P * 8;
        case RT_BUF_SCALED_COLOR: return (size_t)ctx->screenW * ctx->screenH * 8;
        case RT_BUF_DEPTH: case RT_BUF_HISTORY_DEPTH: return P * 2;
        case RT_BUF_NOISE_LEVEL: return (size_t)((ctx->renderW + 7) / 8) * ((ctx->renderH + 7) / 8) * 2;
        case RT_BUF_NOISE_LEVEL16: return (size_t)((ctx->renderW + 15) / 16) * ((ctx->renderH + 15) / 16) * 2;
        case RT_BUF_MOTION: return P * 4;
        case RT_BUF_SKY: return (size_t)kSkySize * 16;
        case RT_BUF_SUN: return (size_t)kSunSize * 16;
        case RT_BUF_HISTOGRAM: return 256;
        case RT_BUF_RGBA8: return (size_t)ctx->screenW * ctx->screenH * 4;
        default: return 0;
    }
}

int rt_get_buffer(const rt_context* cctx, int name, void* dst, size_t bytes) {
    rt_context* ctx = const_cast<rt_context*>(cctx);
    if (!ctx || !dst) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_get_buffer before rt_init"; return RT_ERR_STATE; }
    if (int rc = sync_streams(ctx)) return rc;  // also issues a deferred denoise (buffer plan)
    const FrameResources& fr = ctx->fr;
    const void* src = nullptr;
    switch (name) {
        case RT_BUF_RENDER_COLOR: src = fr.renderColor; break;
        case RT_BUF_ACCUMULATION: src = fr.accum; break;
        case RT_BUF_HISTORY_COLOR: src = fr.histBuf[fr.histIdx]; break;
        case RT_BUF_HISTORY_DEPTH: src = fr.histDepth; break;
        case RT_BUF_SCALED_COLOR: src = fr.scaledColor; break;
        case RT_BUF_NOISE_LEVEL: src = fr.noise8; break;
        case RT_BUF_NOISE_LEVEL16: src = fr.noise16; break;
        case RT_BUF_NORMAL: src = fr.normal; break;
        case RT_BUF_ALBEDO: src = fr.albedo; break;
        case RT_BUF_DEPTH: src = fr.depth; break;
        case RT_BUF_MOTION: src = fr.motion; break;
        case RT_BUF_SKY: src = fr.sky; break;
        case RT_BUF_SUN: src = fr.sun; break;
        case RT_BUF_HISTOGRAM: src = fr.histogram; break;
        case RT_BUF_RGBA8:
            if (bytes < rt_buffer_bytes(ctx, name)) { ctx->err = "destination too small"; return RT_ERR_ARG; }
            return copy_rgba_out(ctx, dst);
        default: ctx->err = "buffer not available in this revision"; return RT_ERR_ARG;
    }
    const size_t need = rt_buffer_bytes(ctx, name);
    if (bytes < need) { ctx->err = "destination too small"; return RT_ERR_ARG; }
    if (int rc = sync_streams(ctx)) return rc;
    HIP_TRY(ctx, hipMemcpy(dst, src, need, hipMemcpyDeviceToHost));
    return RT_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- camera file I/O, image dumps
namespace {
// Camera (kernel.cuh:78-100), __align__(16): the reference's on-disk record
struct CameraRecord {
    float pos[3], pitch;
    float dir[3], focal;
    float left[3], aperture;
    float up[3], yaw;
    float resolution[2], inversedResolution[2];
    float fov[2], tanHalfFov[2];
    float adjustedLeft[3], unused3;
    float adjustedUp[3], unused4;
    float adjustedFront[3], unused5;
    float apertureLeft[3], unused6;
    float apertureUp[3], unused7;
};
static_assert(sizeof(CameraRecord) == 176, "Camera record layout");
}  // namespace

extern "C" int rt_save_camera(const rt_context* cctx, const char* path) {
    rt_context* ctx = const_cast<rt_context*>(cctx);
    if (!ctx || !path || !*path) return RT_ERR_ARG;
    HostCamera hc;
    rt_camera_update(ctx->camera, ctx->renderW, ctx->renderH, hc);
    CameraRecord r{};
    memcpy(r.pos, hc.pos, 12);
    r.pitch = hc.pitch;
    memcpy(r.dir, hc.dir, 12);
    r.focal = hc.focal;
    memcpy(r.left, hc.left, 12);
    r.aperture = hc.aperture;
    memcpy(r.up, hc.up, 12);
    r.yaw = hc.yaw;
    memcpy(r.resolution, hc.res, 8);
    memcpy(r.inversedResolution, hc.invRes, 8);
    memcpy(r.fov, hc.fov, 8);
    memcpy(r.tanHalfFov, hc.tanHalfFov, 8);
    memcpy(r.adjustedLeft, hc.adjustedLeft, 12);
    memcpy(r.adjustedUp, hc.adjustedUp, 12);
    memcpy(r.adjustedFront, hc.adjustedFront, 12);
    memcpy(r.apertureLeft, hc.apertureLeft, 12);
    memcpy(r.apertureUp, hc.apertureUp, 12);
    std::ofstream f(path, std::ios::binary | std::ios::trunc);
    if (!f) { ctx->err = std::string("cannot write camera file ") + path; return RT_ERR_IO; }
    f.write(reinterpret_cast<const char*>(&r), sizeof(r));
    return f ? RT_OK : RT_ERR_IO;
}

extern "C" int rt_load_camera(rt_context* ctx, const char* path) {
    if (!ctx || !path || !*path) return RT_ERR_ARG;
    std::ifstream f(path, std::ios::binary);
    CameraRecord r{};
    if (!f || !f.read(reinterpret_cast<char*>(&r), sizeof(r))) {
        ctx->err = std::string("cannot read camera file ") + path;
        return RT_ERR_IO;
    }
    memcpy(ctx->camera.pos, r.pos, 12);
    ctx->camera.pitch = r.pitch;
    ctx->camera.yaw = r.yaw;
    ctx->camera.focal = r.focal;
    ctx->camera.aperture = r.aperture;
    ctx->camera.fovX = r.fov[0];
    return RT_OK;
}

extern "C" int rt_save_image(rt_context* ctx, const char* path, int kind) {
    if (!ctx || !path || !*path || (kind != RT_IMAGE_PPM_RGBA8 && kind != RT_IMAGE_PFM_HDR)) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_save_image before rt_init"; return RT_ERR_STATE; }
    if (int rc = sync_streams(ctx)) return rc;
    std::ofstream f(path, std::ios::binary | std::ios::trunc);
    if (!f) { ctx->err = std::string("cannot write image ") + path; return RT_ERR_IO; }
    if (kind == RT_IMAGE_PPM_RGBA8) {
        const size_t n = (size_t)ctx->screenW * ctx->screenH;
        std::vector<uint8_t> rgba(n * 4), rgb(n * 3);
        if (int rc = copy_rgba_out(ctx, rgba.data())) return rc;
        for (size_t i = 0; i < n; ++i) memcpy(&rgb[3 * i], &rgba[4 * i], 3);
        f << "P6\n" << ctx->screenW << " " << ctx->screenH << "\n255\n";
        f.write(reinterpret_cast<const char*>(rgb.data()), (std::streamsize)rgb.size());
    } else {
        const int W = ctx->renderW, H = ctx->renderH;
        std::vector<uint16_t> c((size_t)W * H * 4);
        HIP_TRY(ctx, hipMemcpy(c.data(), ctx->fr.renderColor, c.size() * 2, hipMemcpyDeviceToHost));
        std::vector<float> rgb((size_t)W * H * 3);
        for (int y = 0; y < H; ++y)  // PFM rows run bottom to top
            for (int x = 0; x < W; ++x)
                for (int k = 0; k < 3; ++k)
                    rgb[((size_t)(H - 1 - y) * W + x) * 3 + k] = rt_h2f(c[((size_t)y * W + x) * 4 + k]);
        f << "PF\n" << W << " " << H << "\n-1.0\n";  // negative scale: little endian
        f.write(reinterpret_cast<const char*>(rgb.data()), (std::streamsize)(rgb.size() * 4));
    }
    return f ? RT_OK : RT_ERR_IO;
}

// Batch ray query through the persistent queue tracer (the RaySceneIntersect traversal of
// traverse.cuh:107-253 for caller rays): rays = n x (org.xyz, pad, dir.xyz, pad) floats,
// hits = n x (t, triangle index as int bits (-1: miss), u, v), iters = per-ray TraverseBvh
// iterations (optional), kernel_ms = the tracer kernel's HIP-event time (optional).
int rt_trace_rays(rt_context* ctx, const float* rays, uint32_t n, float* hits, uint32_t* iters, float* kernel_ms) {
    if (!ctx || (n > 0 && (!rays || !hits))) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_trace_rays before rt_init"; return RT_ERR_STATE; }
    FrameResources& fr = ctx->fr;
    if (n > fr.ws.cap) { ctx->err = "more rays than the queue capacity (width x strip rows x spp)"; return RT_ERR_ARG; }
    if (kernel_ms) *kernel_ms = 0.0f;
    if (n == 0) return RT_OK;
    std::vector<float4> o(n), d(n);
    for (uint32_t i = 0; i < n; ++i) {
        float tag;
        memcpy(&tag, &i, 4);  // the queue's pixel slot carries the ray index
        o[i] = make_float4(rays[8 * i], rays[8 * i + 1], rays[8 * i + 2], tag);
        d[i] = make_float4(rays[8 * i + 4], rays[8 * i + 5], rays[8 * i + 6], 0.0f);
    }
    PathTraceParams p = {};
    p.triPos = ctx->dTriPos;
    p.triNrm = ctx->dTriNrm;
    p.nodes = ctx->dNodes;
    p.tlasNodes = ctx->dTlasNodes;
    p.ws = fr.ws;
    p.ws.itersOut = iters ? reinterpret_cast<uint32_t*>(fr.ws.pathL) : nullptr;  // pathL: per-frame scratch
    if (int rc = sync_streams(ctx)) return rc;  // the queue buffers are shared with in-flight frames
    HIP_TRY(ctx, hipMemcpyAsync(fr.ws.q3.rayO, o.data(), (size_t)n * 16, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(fr.ws.q3.rayD, d.data(), (size_t)n * 16, hipMemcpyHostToDevice, ctx->stream));
    fr.syncZeroed[0] = false;  // fr.ws.counters is syncCount[0]
    HIP_TRY(ctx, hipMemsetAsync(fr.ws.counters, 0, kWsCounterWords * sizeof(uint32_t), ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(fr.ws.counters + kCntQ3, &n, 4, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipEventRecord(ctx->ev0, ctx->stream));
    HIP_TRY(ctx, rtk_launch_trace_queue(&p, 3, ctx->stream));
    HIP_TRY(ctx, hipEventRecord(ctx->ev1, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(hits, fr.ws.hitRec, (size_t)n * 16, hipMemcpyDeviceToHost, ctx->stream));
    if (iters) HIP_TRY(ctx, hipMemcpyAsync(iters, p.ws.itersOut, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (kernel_ms) HIP_TRY(ctx, hipEventElapsedTime(kernel_ms, ctx->ev0, ctx->ev1));
    return RT_OK;
}
