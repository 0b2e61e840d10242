// context.cpp — RayTracer lifecycle, scene setup and hot-path stage dispatch behind the C-ABI.
//
//   rt_create  <- RayTracer::RayTracer + LoadConfig   (kernel.cuh:435-441, configLoader.cpp:5-27)
//   rt_init    <- RayTracer::init                    (init.cu:53-410)
//   rt_destroy <- RayTracer::cleanup                 (init.cu:601-663)
//   rt_build_bvh / rt_trace_primary <- BuildBvhLevel1/2 (bvh.cu:7-97) / PathTrace's first hit
#include "context.h"

#include <dlfcn.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <fstream>
#include <sstream>

#include "gaussian_tables.h"
#include "rtmath.h"
#include "toml_lite.h"

namespace {

thread_local std::string g_createError;

void default_params(rt_params& p) {
    // settingParams.h defaults
    p.sky.needRegenerate = 1;
    p.sky.timeOfDay = 0.25f;
    p.sky.sunAxisAngle = 45.0f;
    p.sky.skyScalar = 0.01f;
    p.sky.sunScalar = 0.01f;
    p.sky.sunAngle = 0.6f;
    p.sample.sampleSurfaceVsLightUseMisWeight = 1;
    p.sample.sampleSkyVsSunUseFluxWeight = 1;
    p.sample.sampleSurfaceVsLight = 0.5f;
    p.sample.sampleSkyVsSun = 0.5f;
    p.pass.enableTemporalDenoising = 1;
    p.pass.enableLocalSpatialFilter = 1;
    p.pass.enableNoiseLevelVisualize = 0;
    p.pass.enableWideSpatialFilter = 1;
    p.pass.enableTemporalDenoising2 = 1;
    p.pass.enablePostProcess = 1;
    p.pass.enableDownScalePasses = 1;
    p.pass.enableHistogram = 1;
    p.pass.enableAutoExposure = 1;
    p.pass.enableBloomEffect = 0;
    p.pass.enableLensFlare = 0;
    p.pass.enableToneMapping = 1;
    p.pass.enableSharpening = 1;
    p.post.toneMappingType = 3;
    p.post.exposure = 1.0f;
    p.post.gain = 40.0f;
    p.post.maxWhite = 7.0f;
    p.post.gamma = 2.2f;
    p.denoise.local_denoise_sigma_normal = 100.0f;
    p.denoise.local_denoise_sigma_depth = 0.1f;
    p.denoise.local_denoise_sigma_material = 100.0f;
    p.denoise.large_denoise_sigma_normal = 100.0f;
    p.denoise.large_denoise_sigma_depth = 0.01f;
    p.denoise.large_denoise_sigma_material = 100.0f;
    p.denoise.temporal_denoise_sigma_normal = 100.0f;
    p.denoise.temporal_denoise_sigma_depth = 0.1f;
    p.denoise.temporal_denoise_sigma_material = 100.0f;
    p.denoise.noise_threshold_local = 0.001f;
    p.denoise.noise_threshold_large = 0.001f;
}

bool read_file(const std::string& path, std::string& out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::stringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

// meshProcessor .bin (u32 count + Triangle[count], 128 B each: init.cu:28-50,
// tool/meshProcessor.cpp:204-209) -> unshared vertex/index buffers
bool load_triangle_bin(const std::string& path, rtscene::SceneMesh& m, std::string& err) {
    std::string blob;
    if (!read_file(path, blob) || blob.size() < 4) { err = "cannot read mesh file " + path; return false; }
    uint32_t n = 0;
    memcpy(&n, blob.data(), 4);
    // exactly u32 count + count Triangle records of 128 B: the reference reads count * 128 bytes
    // into an uninitialised buffer without checking the read (init.cu:33-43), so a short file
    // (e.g. resources/models/test.bin: 32,768 records of 64 B, the older 4-vertex Triangle) would
    // render uninitialised memory there; it is refused here
    if (n < 2 || blob.size() < 4 + (size_t)n * 128) {
        err = "malformed mesh file " + path + " (" + std::to_string(blob.size()) + " bytes for " + std::to_string(n) +
              " triangles of 128 B)";
        return false;
    }
    m.vertices.resize((size_t)n * 9);
    m.indices.resize((size_t)n * 3);
    for (uint32_t t = 0; t < n; ++t) {
        const char* rec = blob.data() + 4 + (size_t)t * 128;
        for (int k = 0; k < 3; ++k) {
            memcpy(&m.vertices[((size_t)t * 3 + k) * 3], rec + 16 * k, 12);  // v1 w1 v2 w2 v3 w3
            m.indices[(size_t)t * 3 + k] = t * 3 + k;
        }
    }
    m.triCount = n;
    m.triCountPadded = (n + 3u) & ~3u;
    m.indices.resize((size_t)m.triCountPadded * 3, 0u);
    m.cornerCount = n * 3;
    return true;
}

}  // namespace

namespace {
constexpr size_t kArenaChunk = 256ull << 20, kArenaMaxBuffer = 64ull << 20, kArenaAlign = 2ull << 20;
int raw_alloc(rt_context* ctx, void** p, size_t bytes) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, bytes);
    if (e != hipSuccess) {
        ctx->err = std::string("hipMalloc(") + std::to_string(bytes) + "): " + hipGetErrorString(e);
        return RT_ERR_HIP;
    }
    ctx->allocations.push_back(q);
    *p = q;
    return RT_OK;
}
}  // namespace

// A renderer stream.  The frame pipeline needs its streams to run concurrently, but HIP maps
// ordinary streams onto a few hardware queues (GPU_MAX_HW_QUEUES, 4) shared round-robin with every
// stream created before in the process — a framework's stream pool, say.  Measured: after torch
// had created its pools, rt_draw_device(RT_DRAW_ASYNC) ran 1.42 ms/frame instead of 1.10, two of
// its streams having landed on one queue.  A stream created with a CU mask gets a hardware queue
// of its own, so the renderer's streams use a full mask; they then carry no priority, which
// measured no difference.  [tuning] streams = "prio": plain streams with priorities.
// hipExtStreamCreateWithCUMask makes blocking streams (hipStreamDefault): work on the null stream
// (a framework's default-stream kernels, synchronous hipMemcpy / hipMemset) and the renderer's
// streams wait for each other.  The renderer itself issues synchronous copies only outside
// frames (rt_init, rt_bind_buffer, host reads, the ray-counter reset); a host that keeps default-
// stream work in flight beside pipelined frames should set [tuning] streams = "prio" (non-blocking
// streams).
int rt_create_stream(rt_context* ctx, hipStream_t* s, bool high) {
    if (!ctx->tune.prioStreams) {
        uint32_t mask[32];  // 1024 CUs' worth of bits; bits past the device's CU count are ignored
        for (uint32_t& m : mask) m = 0xFFFFFFFFu;
        HIP_TRY(ctx, hipExtStreamCreateWithCUMask(s, 32, mask));
        return RT_OK;
    }
    int least = 0, greatest = 0;
    HIP_TRY(ctx, hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIP_TRY(ctx, hipStreamCreateWithPriority(s, hipStreamNonBlocking, high ? greatest : least));
    return RT_OK;
}

// Device buffers of a context.  Buffers up to 64 MiB (the BVH, triangles, textures, sky tables,
// G-buffers, counters) are carved from 256-MiB chunks, each buffer starting on a 2-MiB boundary,
// so the data a frame reads lies in a few large, contiguous allocations rather than in dozens of
// separate ones wherever a fragmented device heap puts them; the large, sparsely
// used queue planes get allocations of their own.
int rt_dalloc_bytes(rt_context* ctx, void** p, size_t bytes) {
    if (bytes < 16) bytes = 16;
    if (!ctx->tune.arena || bytes > kArenaMaxBuffer) return raw_alloc(ctx, p, bytes);
    size_t at = (ctx->arenaUsed + kArenaAlign - 1) / kArenaAlign * kArenaAlign;
    if (!ctx->arenaPtr || at + bytes > ctx->arenaCap) {
        void* chunk = nullptr;
        const int rc = raw_alloc(ctx, &chunk, kArenaChunk);
        if (rc != RT_OK) return rc;
        ctx->arenaPtr = (char*)chunk;
        ctx->arenaCap = kArenaChunk;
        at = 0;
    }
    *p = ctx->arenaPtr + at;
    ctx->arenaUsed = at + bytes;
    return RT_OK;
}

std::string rt_data_dir() {
    Dl_info info;
    if (dladdr((void*)&rt_data_dir, &info) && info.dli_fname) {
        std::string so = info.dli_fname;
        size_t s = so.rfind('/');
        std::string dir = s == std::string::npos ? std::string(".") : so.substr(0, s);
        return dir + "/../data";
    }
    return "real-time-ray-tracing_amd/data";
}

// Camera::update (kernel.cuh:103-121), evaluated with the deterministic rtmath functions
void rt_camera_update(const rt_camera& in, int renderW, int renderH, HostCamera& c) {
    memcpy(c.pos, in.pos, sizeof(c.pos));
    c.yaw = in.yaw;
    c.pitch = in.pitch;
    c.focal = in.focal;
    c.aperture = in.aperture;
    c.res[0] = (float)renderW;
    c.res[1] = (float)renderH;
    c.fov[0] = in.fovX;
    const float sy = rt_sinf(c.yaw), cy = rt_cosf(c.yaw), sp = rt_sinf(c.pitch), cp = rt_cosf(c.pitch);
    float dir[3] = {sy * cp, sp, cy * cp};
    c.invRes[0] = 1.0f / c.res[0];
    c.invRes[1] = 1.0f / c.res[1];
    c.fov[1] = c.fov[0] / c.res[0] * c.res[1];
    c.tanHalfFov[0] = rt_tanf(c.fov[0] / 2);
    c.tanHalfFov[1] = rt_tanf(c.fov[1] / 2);
    auto dopf = [](float a, float b, float cc, float d) {
        float cd = cc * d;
        float e = fmaf(-cc, d, cd);
        float dp = fmaf(a, b, -cd);
        return dp + e;
    };
    auto crossf = [&](const float* a, const float* b, float* r) {
        r[0] = dopf(a[1], b[2], a[2], b[1]);
        r[1] = dopf(a[2], b[0], a[0], b[2]);
        r[2] = dopf(a[0], b[1], a[1], b[0]);
    };
    auto normf = [](float* v) {
        float n = sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        v[0] = v[0] / n; v[1] = v[1] / n; v[2] = v[2] / n;
    };
    float up0[3] = {0.0f, 1.0f, 0.0f}, left[3], up[3];
    crossf(up0, dir, left);
    normf(left);
    crossf(dir, left, up);
    normf(up);
    for (int k = 0; k < 3; ++k) {
        c.dir[k] = dir[k];
        c.left[k] = left[k];
        c.up[k] = up[k];
        c.adjustedFront[k] = dir[k] * c.focal;
        c.adjustedLeft[k] = left[k] * c.tanHalfFov[0] * c.focal;
        c.adjustedUp[k] = up[k] * c.tanHalfFov[1] * c.focal;
        c.apertureLeft[k] = left[k] * c.aperture;
        c.apertureUp[k] = up[k] * c.aperture;
    }
}

TraceCamera rt_trace_camera(const HostCamera& c) {
    TraceCamera t;
    memcpy(t.pos, c.pos, 12);
    memcpy(t.adjustedFront, c.adjustedFront, 12);
    memcpy(t.adjustedLeft, c.adjustedLeft, 12);
    memcpy(t.adjustedUp, c.adjustedUp, 12);
    memcpy(t.apertureLeft, c.apertureLeft, 12);
    memcpy(t.apertureUp, c.apertureUp, 12);
    memcpy(t.invRes, c.invRes, 8);
    return t;
}

extern "C" {

const char* rt_last_error(const rt_context* ctx) { return ctx ? ctx->err.c_str() : g_createError.c_str(); }

int rt_scene_noise3d(const float* xyz, size_t n, float* out) {
    if (n > 0 && (!xyz || !out)) return RT_ERR_ARG;
    for (size_t k = 0; k < n; ++k) out[k] = rtscene::noise3d(xyz[3 * k], xyz[3 * k + 1], xyz[3 * k + 2]);
    return RT_OK;
}

int rt_filter_kernel(int size, float* out, int count) {
    static const float g3[9] = RT_GAUSS3_INIT, g5[25] = RT_GAUSS5_INIT, g7[49] = RT_GAUSS7_INIT;
    const float* g = size == 3 ? g3 : size == 5 ? g5 : size == 7 ? g7 : nullptr;
    if (!g || !out || count < size * size) return RT_ERR_ARG;
    memcpy(out, g, sizeof(float) * size * size);
    return RT_OK;
}

int rt_scan_device(const float* in, float* out, float* tmp, int size, int block_size, int postfix, void* stream) {
    if (!in || !out || size <= 0) {
        g_createError = "rt_scan_device: null buffer or empty size";
        return RT_ERR_ARG;
    }
    const hipError_t e = rtk_launch_scan_ex(in, out, tmp, size, block_size, postfix ? 1 : 0, (hipStream_t)stream);
    if (e == hipErrorInvalidValue) {
        g_createError = "rt_scan_device: size / block_size must be powers of two with block_size and the block "
                        "count <= 8192, and tmp non-null when there is more than one block";
        return RT_ERR_ARG;
    }
    if (e != hipSuccess) {
        g_createError = std::string("rt_scan_device: ") + hipGetErrorString(e);
        return RT_ERR_HIP;
    }
    return RT_OK;
}

int rt_create(int screen_width, int screen_height, const char* config_toml, rt_context** out) {
    if (!out) return RT_ERR_ARG;
    *out = nullptr;
    rt_context* ctx = new rt_context();
    default_params(ctx->params);
    // CameraSetup defaults (init.cu:412-439)
    ctx->camera.pos[0] = -2.0f; ctx->camera.pos[1] = 2.0f; ctx->camera.pos[2] = -2.0f;
    ctx->camera.yaw = 0.0f; ctx->camera.pitch = 0.0f;
    ctx->camera.focal = 5.0f; ctx->camera.aperture = 0.001f;
    ctx->camera.fovX = 90.0f * 0.01745329251f;
    rttoml::Doc doc;
    if (config_toml && config_toml[0]) {
        std::string text, err;
        if (!read_file(config_toml, text)) { g_createError = std::string("cannot read config ") + config_toml; delete ctx; return RT_ERR_IO; }
        if (!rttoml::parse(text, doc, err)) { g_createError = "config parse error: " + err; delete ctx; return RT_ERR_IO; }
    }
    // LoadConfig (configLoader.cpp:15-26); the screen size passed in wins, as in main.cu:260
    int w = rttoml::find_or_int(doc, "resolution", "width", 1920);
    int h = rttoml::find_or_int(doc, "resolution", "height", 1080);
    ctx->screenW = screen_width > 0 ? screen_width : w;
    ctx->screenH = screen_height > 0 ? screen_height : h;
    ctx->inputMeshFileName = rttoml::find_or_string(doc, "file", "inputMeshFileName", "");
    ctx->inputTextureFileNames = rttoml::find_or_strings(doc, "file", "inputTextureFileNames");
    ctx->inputCameraFileName = rttoml::find_or_string(doc, "file", "inputCameraFileName", "");
    ctx->cameraSaveFileName = rttoml::find_or_string(doc, "file", "cameraSaveFileName", "");
    ctx->loadCameraAtInit = rttoml::find_or_bool(doc, "file", "loadCameraAtInit", false);
    ctx->useDynamicResolution = rttoml::find_or_bool(doc, "optimziation", "useDynamicResolution", true);
    ctx->targetFps = rttoml::find_or_float(doc, "optimziation", "targetFps", 60.0f);
    ctx->maxWidth = rttoml::find_or_int(doc, "optimziation", "maxWidth", 3840);
    ctx->maxHeight = rttoml::find_or_int(doc, "optimziation", "maxHeight", 2160);
    ctx->minWidth = rttoml::find_or_int(doc, "optimziation", "minWidth", 640);
    ctx->minHeight = rttoml::find_or_int(doc, "optimziation", "minHeight", 480);
    ctx->chunkDim = rttoml::find_or_int(doc, "scene", "chunkDim", 1);
    ctx->meshFile = rttoml::find_or_string(doc, "scene", "meshFile", "");
    ctx->spp = rttoml::find_or_int(doc, "render", "spp", 1);
    ctx->bvhThreads = rttoml::find_or_int(doc, "render", "bvhThreads", 0);  // LBVH workgroup shape (A/B, tests)
    ctx->device = rttoml::find_or_int(doc, "render", "device", -1);
    ctx->stripY0 = rttoml::find_or_int(doc, "render", "stripY0", 0);
    ctx->stripRows = rttoml::find_or_int(doc, "render", "stripRows", -1);
    ctx->stripCount = rttoml::find_or_int(doc, "render", "stripCount", 1);
    ctx->stripIndex = rttoml::find_or_int(doc, "render", "stripIndex", 0);
    ctx->materialOverride = rttoml::find_or_int(doc, "render", "materialOverride", -1);
    ctx->bvhSkipPublish = (uint32_t)rttoml::find_or_int(doc, "debug", "bvhSkipPublish", -1);
    ctx->bvhSkipBuilds = rttoml::find_or_int(doc, "debug", "bvhSkipPublishBuilds", -1);
    ctx->bvhWaitMs = rttoml::find_or_float(doc, "debug", "bvhWaitMs", 1000.0f);
    {
        rt_context::Tuning& t = ctx->tune;
        t.arena = rttoml::find_or_bool(doc, "tuning", "arena", true);
        t.prioStreams = rttoml::find_or_string(doc, "tuning", "streams", "cumask") == "prio";
        t.tracePerCu = rttoml::find_or_int(doc, "tuning", "tracePerCu", 0);
        t.trace4PerCu = rttoml::find_or_int(doc, "tuning", "trace4PerCu", 0);
        t.trace3ShortPerCu = rttoml::find_or_int(doc, "tuning", "trace3ShortPerCu", 2);
        const std::string chain = rttoml::find_or_string(doc, "tuning", "chain", "serial");
        t.chain = chain == "off" ? 0 : chain == "always" ? 2 : 1;
        t.shadeOnSide = rttoml::find_or_bool(doc, "tuning", "shadeOnSide", true);
        t.shadeBlocksPerCu = rttoml::find_or_int(doc, "tuning", "shadeBlocksPerCu", 0);
        t.overlapAfter = rttoml::find_or_int(doc, "tuning", "overlapAfter", -1);
        t.cameraAfter = rttoml::find_or_int(doc, "tuning", "cameraAfter", -1);
        t.syncSpec = rttoml::find_or_bool(doc, "tuning", "syncSpec", true);
        t.specChain = rttoml::find_or_int(doc, "tuning", "specChain", -1);
        t.specAfter = rttoml::find_or_int(doc, "tuning", "specAfter", 1);
        t.specShade = rttoml::find_or_int(doc, "tuning", "specShade", 2);
        t.specShadePerCu = rttoml::find_or_int(doc, "tuning", "specShadePerCu", 2);
        t.specTracePerCu = rttoml::find_or_int(doc, "tuning", "specTracePerCu", 2);
        t.dnSplit = rttoml::find_or_int(doc, "tuning", "dnSplit", 0);
        t.dnFold = rttoml::find_or_int(doc, "tuning", "dnFold", 0) != 0;
    }
    if (ctx->screenW <= 0 || ctx->screenH <= 0 || ctx->screenW > 16384 || ctx->screenH > 16384 || ctx->spp < 1 ||
        ctx->spp > 64 || ctx->chunkDim < 1 || ctx->chunkDim > 8 ||
        (ctx->bvhThreads != 0 && ctx->bvhThreads != 512 && ctx->bvhThreads != 1024)) {
        g_createError = "invalid resolution / spp / chunkDim / bvhThreads";
        delete ctx;
        return RT_ERR_ARG;
    }
    // init.cu:58-67: dynamic resolution renders at the max size
    if (ctx->useDynamicResolution) { ctx->renderW = ctx->maxWidth; ctx->renderH = ctx->maxHeight; }
    else { ctx->renderW = ctx->screenW; ctx->renderH = ctx->screenH; }
    if (ctx->stripCount > 1) {  // interleaved row blocks (row_of): stripY0 / stripRows do not apply
        if (ctx->stripIndex < 0 || ctx->stripIndex >= ctx->stripCount || ctx->stripY0 != 0 || ctx->stripRows >= 0) {
            g_createError = "stripCount > 1 needs 0 <= stripIndex < stripCount and no stripY0 / stripRows";
            delete ctx;
            return RT_ERR_ARG;
        }
        ctx->stripRows = (int)strip_row_count((uint32_t)ctx->renderH, (uint32_t)ctx->stripCount, (uint32_t)ctx->stripIndex);
    }
    if (ctx->stripRows < 0) ctx->stripRows = ctx->renderH - ctx->stripY0;
    ctx->fullFrame = ctx->stripCount == 1 && ctx->stripY0 == 0 && ctx->stripRows == ctx->renderH;
    ctx->histW = ctx->renderW;
    ctx->histH = ctx->renderH;
    ctx->allocW = ctx->renderW;  // the largest frame: dynamic resolution only shrinks from here
    ctx->allocH = ctx->renderH;
    ctx->allocStripRows = ctx->stripRows;
    if (ctx->stripCount < 1 || ctx->stripY0 < 0 || ctx->stripRows < 1 || ctx->stripY0 + ctx->stripRows > ctx->renderH) {
        g_createError = "invalid strip rows";
        delete ctx;
        return RT_ERR_ARG;
    }
    *out = ctx;
    return RT_OK;
}

int rt_init(rt_context* ctx) {
    if (!ctx) return RT_ERR_ARG;
    if (ctx->inited) { ctx->err = "rt_init called twice"; return RT_ERR_STATE; }
    // ---- scene (init.cu:78-130), built and checked on the host before any device call, so a bad
    // input is reported as such on any machine
    std::string err;
    const std::string dataDir = rt_data_dir();
    if (!ctx->meshFile.empty()) {
        if (!load_triangle_bin(ctx->meshFile, ctx->mesh, err)) { ctx->err = err; return RT_ERR_IO; }
    } else {
        std::vector<std::vector<float>> tiles;
        if (!rtscene::load_tiles(dataDir + "/roundcubes_l2.bin", tiles, err) ||
            !rtscene::generate(ctx->chunkDim, tiles, ctx->mesh, err)) {
            ctx->err = err;
            return RT_ERR_IO;
        }
    }
    const uint32_t N = ctx->mesh.triCount, NP = ctx->mesh.triCountPadded;
    // MIN_TRIANGLE_COUNT_ALLOWED 2 / MAX_TRIANGLE_COUNT_ALLOWED 1024 * 1024 (kernel.cuh:54-55), which
    // init.cu:89-90 asserts; the reference's LBVH needs two triangles for a BLAS (buildBVH.cuh:30)
    if (N < 2 || N > 1024u * 1024u) { ctx->err = "triangle count out of range [2, 1048576] (kernel.cuh:54-55)"; return RT_ERR_ARG; }
    ctx->B = (N + 1023) / 1024;
    if (ctx->B >= 1024) { ctx->err = "batch count must stay below 1024 (init.cu:126)"; return RT_ERR_ARG; }
    ctx->nv = (uint32_t)(ctx->mesh.vertices.size() / 3);

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) { ctx->err = "no HIP device visible"; return RT_ERR_NO_DEVICE; }
    if (ctx->device >= 0) HIP_TRY(ctx, hipSetDevice(ctx->device));
    int dev = 0;
    HIP_TRY(ctx, hipGetDevice(&dev));
    ctx->device = dev;
    hipDeviceProp_t prop;
    HIP_TRY(ctx, hipGetDeviceProperties(&prop, dev));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        ctx->err = std::string("librtx is built for gfx950, device is ") + prop.gcnArchName;
        return RT_ERR_NO_DEVICE;
    }
    ctx->cuCount = prop.multiProcessorCount;
    int wallKhz = 0;
    if (hipDeviceGetAttribute(&wallKhz, hipDeviceAttributeWallClockRate, dev) == hipSuccess && wallKhz > 0)
        ctx->wallTicksPerMs = (uint64_t)wallKhz;
    HIP_TRY(ctx, hipHostMalloc((void**)&ctx->status, 64, hipHostMallocDefault));
    memset(ctx->status, 0, 64);

    // the context stream (the trace chain, a frame's critical path); with [tuning] streams = "prio" it is
    // created at the highest priority and the side / internal post streams at the lowest, otherwise
    // all are CU-masked streams without priority (rt_create_stream)
    if (int rc = rt_create_stream(ctx, &ctx->ownStream, true)) return rc;
    ctx->stream = ctx->ownStream;
    HIP_TRY(ctx, hipEventCreate(&ctx->ev0));
    HIP_TRY(ctx, hipEventCreate(&ctx->ev1));

    int rc;
#define ALLOC(p, bytes) if ((rc = dalloc(ctx, &(p), (bytes))) != RT_OK) return rc
    ALLOC(ctx->dVerts, (size_t)ctx->nv * 12);
    ALLOC(ctx->dNormals, (size_t)ctx->nv * 12);
    ALLOC(ctx->dIdx, (size_t)NP * 12);
    // the record arena (traverse.h): BLAS nodes, TLAS nodes, triangle records, 64 B each
    ALLOC(ctx->dNodes, arena_bytes(ctx->B, NP));
    ctx->dTlasNodes = (char*)ctx->dNodes + (size_t)ctx->B * 1024 * 64;
    ctx->dTriPos = (float4*)((char*)ctx->dNodes + ((size_t)ctx->B * 1024 + ctx->B) * 64);
    ALLOC(ctx->dTriNrm, (size_t)NP * 48);
    ALLOC(ctx->dAabbs, (size_t)NP * 24);
    ALLOC(ctx->dBatchScene, (size_t)ctx->B * 24);
    ALLOC(ctx->dMorton, (size_t)ctx->B * 4096);
    ALLOC(ctx->dReorder, (size_t)ctx->B * 4096);
    ALLOC(ctx->dTlasAabbs, (size_t)ctx->B * 24);
    ALLOC(ctx->dTlasScene, 24);
    ALLOC(ctx->dTlasMorton, 4096);
    ALLOC(ctx->dTlasReorder, 4096);
    ALLOC(ctx->dCounter, 64);
    ctx->bvh[0] = BvhBufs{ctx->dTriPos, ctx->dTriNrm, ctx->dAabbs, ctx->dBatchScene, ctx->dMorton, ctx->dReorder,
                          ctx->dNodes, ctx->dTlasAabbs, ctx->dTlasScene, ctx->dTlasMorton, ctx->dTlasReorder,
                          ctx->dTlasNodes, ctx->dCounter};
    ALLOC(ctx->dBlueNoise, 327680);
    const size_t P = (size_t)ctx->renderW * ctx->renderH;
    ALLOC(ctx->dHits, P * 16);
    ALLOC(ctx->dHitNrm, P * 16);
    ALLOC(ctx->dHitFake, P * 16);
    ALLOC(ctx->dHitStats, P * 16);

    HIP_TRY(ctx, hipMemcpy(ctx->dVerts, ctx->mesh.vertices.data(), (size_t)ctx->nv * 12, hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemcpy(ctx->dIdx, ctx->mesh.indices.data(), (size_t)NP * 12, hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemset(ctx->dCounter, 0, 64));
    HIP_TRY(ctx, hipMemset(ctx->dNodes, 0, arena_bytes(ctx->B, NP)));

    std::string bn;
    if (!read_file(dataDir + "/bluenoise_4spp.bin", bn) || bn.size() != 327680) {
        ctx->err = "cannot read " + dataDir + "/bluenoise_4spp.bin";
        return RT_ERR_IO;
    }
    HIP_TRY(ctx, hipMemcpy(ctx->dBlueNoise, bn.data(), bn.size(), hipMemcpyHostToDevice));

    // ---- frame-1 smooth normals (kernel.cu:313-327): vertex -> corner CSR in triangle order
    {
        std::vector<uint32_t> off(ctx->nv + 1, 0), corners((size_t)NP * 3);
        for (size_t c = 0; c < (size_t)NP * 3; ++c) off[ctx->mesh.indices[c] + 1]++;
        for (uint32_t v = 0; v < ctx->nv; ++v) off[v + 1] += off[v];
        std::vector<uint32_t> fill(off.begin(), off.end() - 1);
        for (size_t c = 0; c < (size_t)NP * 3; ++c) corners[fill[ctx->mesh.indices[c]]++] = (uint32_t)c;
        ALLOC(ctx->dAdjOff, off.size() * 4);
        ALLOC(ctx->dAdjCorner, corners.size() * 4);
        HIP_TRY(ctx, hipMemcpy(ctx->dAdjOff, off.data(), off.size() * 4, hipMemcpyHostToDevice));
        HIP_TRY(ctx, hipMemcpy(ctx->dAdjCorner, corners.data(), corners.size() * 4, hipMemcpyHostToDevice));
        HIP_TRY(ctx, rtk_launch_smooth_normals(ctx->dVerts, ctx->dAdjOff, ctx->dAdjCorner, ctx->dIdx, ctx->nv,
                                               ctx->dNormals, ctx->stream));
    }
#undef ALLOC
    if ((rc = rt_frame_init(ctx)) != RT_OK) return rc;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    ctx->inited = true;
    // CameraSetup (init.cu:433-435): a missing or short file leaves the default camera, and the
    // reference only prints its error, so this is not an rt_init failure either
    if (ctx->loadCameraAtInit && rt_load_camera(ctx, ctx->inputCameraFileName.c_str()) != RT_OK)
        fprintf(stderr, "librtx: %s (default camera kept)\n", ctx->err.c_str());
    return RT_OK;
}

void rt_destroy(rt_context* ctx) {
    if (!ctx) return;
    if (ctx->inited) (void)sync_streams(ctx, false);  // also when the context stream is the null stream
    for (hipEvent_t e : {ctx->overlapEv, ctx->cameraGate, ctx->specGate, ctx->specDone, ctx->buildDone[0], ctx->buildDone[1],
                         ctx->bvhFree[0], ctx->bvhFree[1]})
        if (e) (void)hipEventDestroy(e);
    for (int k = 0; k < kGbSets; ++k)
        for (hipEvent_t e : {ctx->ptDone[k], ctx->postDone[k], ctx->camDone[k], ctx->restDone[k], ctx->gatherDone[k]})
            if (e) (void)hipEventDestroy(e);
    if (ctx->sideStream) (void)hipStreamDestroy(ctx->sideStream);
    if (ctx->ownPostStream) (void)hipStreamDestroy(ctx->ownPostStream);
    for (void* p : ctx->allocations) (void)hipFree(p);
    if (ctx->fr.q3Host) (void)hipHostFree(ctx->fr.q3Host);
    if (ctx->status) (void)hipHostFree(ctx->status);
    for (hipEvent_t e : ctx->markPool)
        if (e) (void)hipEventDestroy(e);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->ownStream) {
        (void)hipStreamSynchronize(ctx->ownStream);
        (void)hipStreamDestroy(ctx->ownStream);
    }
    delete ctx;
}

int rt_get_params(const rt_context* ctx, rt_params* out) {
    if (!ctx || !out) return RT_ERR_ARG;
    *out = ctx->params;
    return RT_OK;
}

int rt_set_params(rt_context* ctx, const rt_params* in) {
    if (!ctx || !in) return RT_ERR_ARG;
    ctx->params = *in;
    return RT_OK;
}

int rt_get_camera(const rt_context* ctx, rt_camera* out) {
    if (!ctx || !out) return RT_ERR_ARG;
    *out = ctx->camera;
    return RT_OK;
}

int rt_set_camera(rt_context* ctx, const rt_camera* in) {
    if (!ctx || !in) return RT_ERR_ARG;
    ctx->camera = *in;
    return RT_OK;
}

int rt_set_frame_index(rt_context* ctx, int frame_num) {
    if (!ctx || frame_num < 1) return RT_ERR_ARG;
    ctx->nextFrame = frame_num;
    return RT_OK;
}

int rt_set_delta_time(rt_context* ctx, float ms) {
    if (!ctx) return RT_ERR_ARG;
    ctx->deltaMs = ms;
    return RT_OK;
}

int rt_get_info(const rt_context* ctx, rt_info* out) {
    if (!ctx || !out) return RT_ERR_ARG;
    out->triCount = ctx->mesh.triCount;
    out->triCountPadded = ctx->mesh.triCountPadded;
    out->batchCount = ctx->B;
    out->vertexCount = ctx->nv;
    out->renderWidth = ctx->renderW;
    out->renderHeight = ctx->renderH;
    out->screenWidth = ctx->screenW;
    out->screenHeight = ctx->screenH;
    out->frameNum = ctx->lastFrame;
    out->deviceId = ctx->device;
    out->spp = (uint32_t)ctx->spp;
    out->gbufferSet = ctx->fr.gbSet;
    uint32_t a = 0, b = (uint32_t)ctx->renderH;
    if (ctx->stripCount > 1) denoise_rows((uint32_t)ctx->renderH, (uint32_t)ctx->stripCount, (uint32_t)ctx->stripIndex, a, b);
    out->denoiseRowBegin = (int32_t)a;
    out->denoiseRowEnd = (int32_t)b;
    uint32_t sa = 0, sb = 0, lo = 0, hi = (uint32_t)ctx->renderH;
    out->stripLocalDenoise = 0;
    out->shadeOnSide = ctx->postStream && ctx->shadeOnSide ? 1 : 0;
    out->lastChain = ctx->fr.lastChain ? 1 : 0;
    if (ctx->inited && strip_local_denoise(ctx, sa, sb)) {
        gbuffer_rows((uint32_t)ctx->renderH, sa, sb, lo, hi);
        out->stripLocalDenoise = 1;
    }
    out->gbufferRowBegin = (int32_t)lo;
    out->gbufferRowEnd = (int32_t)hi;
    return RT_OK;
}

void bvh_select(rt_context* ctx, int k) {
    const BvhBufs& b = ctx->bvh[k];
    ctx->bvhSet = k;
    ctx->dTriPos = b.triPos;
    ctx->dTriNrm = b.triNrm;
    ctx->dAabbs = b.aabbs;
    ctx->dBatchScene = b.batchScene;
    ctx->dMorton = b.morton;
    ctx->dReorder = b.reorder;
    ctx->dNodes = b.nodes;
    ctx->dTlasAabbs = b.tlasAabbs;
    ctx->dTlasScene = b.tlasScene;
    ctx->dTlasMorton = b.tlasMorton;
    ctx->dTlasReorder = b.tlasReorder;
    ctx->dTlasNodes = b.tlasNodes;
    ctx->dCounter = b.counter;
}

int rt_build_bvh(rt_context* ctx) {
    if (!ctx) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_build_bvh before rt_init"; return RT_ERR_STATE; }
    if (int rc = check_device_status(ctx)) return rc;  // a previous build's failure, once it is known
    hipStream_t stream = ctx->stream;
    // camera rays a synchronous draw traced ahead read this set (frame.cpp launch_spec_camera): the
    // rebuild writes the same values, but after them
    if (ctx->fr.spec.valid) HIP_TRY(ctx, hipStreamWaitEvent(stream, ctx->specDone, 0));
    ctx->bvhPrebuilt = false;  // an explicit build supersedes a synchronous draw's prebuild
    if (!ctx->postStream) ctx->buildOnSide[ctx->bvhSet] = false;
    if (ctx->postStream) {  // frame pipelining: build into the other set, on the side stream
        const int k = ctx->bvhSet ^ 1;
        if (ctx->bvhInFlight[k]) HIP_TRY(ctx, hipStreamWaitEvent(ctx->sideStream, ctx->bvhFree[k], 0));
        bvh_select(ctx, k);
        stream = ctx->sideStream;
    }
    BvhBuildParams p;
    p.vertices = ctx->dVerts;
    p.normals = ctx->dNormals;
    p.indices = ctx->dIdx;
    p.triCount = ctx->mesh.triCount;
    p.triCountPadded = ctx->mesh.triCountPadded;
    p.batchCount = ctx->B;
    p.triPos = ctx->dTriPos;
    p.triNrm = ctx->dTriNrm;
    p.aabbs = ctx->dAabbs;
    p.batchSceneAabbs = ctx->dBatchScene;
    p.morton = ctx->dMorton;
    p.reorder = ctx->dReorder;
    p.nodes = ctx->dNodes;
    p.tlasAabbs = ctx->dTlasAabbs;
    p.tlasSceneAabb = ctx->dTlasScene;
    p.tlasMorton = ctx->dTlasMorton;
    p.tlasReorder = ctx->dTlasReorder;
    p.tlasNodes = ctx->dTlasNodes;
    p.counter = ctx->dCounter;
    p.threads = (uint32_t)ctx->bvhThreads;
    p.cus = (uint32_t)ctx->cuCount;
    p.status = ctx->status;
    p.waitTicks = (uint64_t)((double)ctx->bvhWaitMs * (double)ctx->wallTicksPerMs);
    p.skipPublish = ctx->bvhSkipBuilds != 0 ? ctx->bvhSkipPublish : 0xFFFFFFFFu;
    if (ctx->bvhSkipBuilds > 0) --ctx->bvhSkipBuilds;
    p.buildSeq = ++ctx->buildSeq;
    HIP_TRY(ctx, rtk_launch_build_bvh(&p, stream));
    if (ctx->postStream) {
        HIP_TRY(ctx, hipEventRecord(ctx->buildDone[ctx->bvhSet], stream));
        ctx->buildOnSide[ctx->bvhSet] = true;
    }
    return RT_OK;
}

// a context-stream user of the current LBVH waits for its build on the side stream
int wait_bvh(rt_context* ctx) {
    if (ctx->buildOnSide[ctx->bvhSet])
        HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->buildDone[ctx->bvhSet], 0));
    return RT_OK;
}

int rt_trace_primary(rt_context* ctx, int frame_num, int with_detail) {
    if (!ctx) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_trace_primary before rt_init"; return RT_ERR_STATE; }
    HostCamera hc;
    rt_camera_update(ctx->camera, ctx->renderW, ctx->renderH, hc);
    TracePrimaryParams p;
    p.cam = rt_trace_camera(hc);
    p.width = (uint32_t)ctx->renderW;
    p.height = (uint32_t)ctx->renderH;
    p.y0 = (uint32_t)ctx->stripY0;
    p.rows = (uint32_t)ctx->stripRows;
    p.nStrips = (uint32_t)ctx->stripCount;
    p.strip = (uint32_t)ctx->stripIndex;
    p.frameNum = frame_num;
    p.bluenoise = ctx->dBlueNoise;
    p.triPos = ctx->dTriPos;
    p.triNrm = ctx->dTriNrm;
    p.nodes = ctx->dNodes;
    p.tlasNodes = ctx->dTlasNodes;
    p.hitOut = ctx->dHits;
    p.normalOut = with_detail ? ctx->dHitNrm : nullptr;
    p.fakeNormalOut = with_detail ? ctx->dHitFake : nullptr;
    p.statsOut = with_detail ? ctx->dHitStats : nullptr;
    if (int rc = wait_bvh(ctx)) return rc;
    HIP_TRY(ctx, rtk_launch_trace_primary(&p, ctx->stream));
    return RT_OK;
}

int rt_sync(rt_context* ctx) {
    if (!ctx) return RT_ERR_ARG;
    if (!ctx->inited) return RT_OK;  // NULL is a valid stream (the null stream): test the init state
    return sync_streams(ctx);
}

int rt_draw_frame_internal(rt_context* ctx);  // frame.cpp

int rt_time_stage(rt_context* ctx, int stage, int iters, float* total_ms) {
    if (!ctx || !total_ms || iters < 1) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_time_stage before rt_init"; return RT_ERR_STATE; }
    if (ctx->postStream) {  // stages are timed serially on the context stream
        void* post = ctx->postStream;
        int rc = rt_set_post_stream(ctx, nullptr);
        if (rc == RT_OK) rc = rt_time_stage(ctx, stage, iters, total_ms);
        const int rc2 = rt_set_post_stream(ctx, post);
        return rc != RT_OK ? rc : rc2;
    }
    HIP_TRY(ctx, hipEventRecord(ctx->ev0, ctx->stream));
    for (int i = 0; i < iters; ++i) {
        int rc = RT_OK;
        if (stage == 0) rc = rt_build_bvh(ctx);
        else if (stage == 1) rc = rt_trace_primary(ctx, 1 + i, 0);
        else if (stage == 2) rc = rt_path_trace(ctx, 1 + i, 0);
        else if (stage == 3) {
            const int f = ctx->nextFrame++;
            if ((rc = rt_build_bvh(ctx)) == RT_OK && (rc = rt_path_trace(ctx, f, 0)) == RT_OK)
                rc = rt_denoise_post(ctx, f, 0);
        } else if (stage == 4) rc = rt_denoise_post(ctx, 2 + i, 0);
        else { ctx->err = "unknown stage"; return RT_ERR_ARG; }
        if (rc != RT_OK) return rc;
    }
    HIP_TRY(ctx, hipEventRecord(ctx->ev1, ctx->stream));
    HIP_TRY(ctx, hipEventSynchronize(ctx->ev1));
    HIP_TRY(ctx, hipEventElapsedTime(total_ms, ctx->ev0, ctx->ev1));
    return RT_OK;
}

// per-kernel HIP-event split of `iters` path traces: serial ones (stage 2 of rt_time_stage) or,
// with `frames` set, whole frames (BVH + path trace + denoise/post) as the caller runs them, so
// on a pipelined context each kernel is timed beside the other streams' work (bench.py).  Kernels
// 0..6 are the path trace's, 7..14 (frames only, n >= 15) the denoise / post chain's; a denoise
// kernel's average is over the frames that launched it (its events read 0 ms otherwise).
static int time_kernels(rt_context* ctx, int first_frame, int iters, float* kernel_ms, int n, bool frames) {
    if (!ctx || !kernel_ms || iters < 1 || n < kPtKernels || first_frame < 1) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_time_*_kernels before rt_init"; return RT_ERR_STATE; }
    const int nk = frames ? (n < kFrameKernels ? n : kFrameKernels) : kPtKernels;
    std::vector<hipEvent_t> marks((size_t)iters * 2 * kFrameKernels, nullptr);
    int rc = RT_OK;
    for (size_t i = 0; i < marks.size(); ++i) {
        if ((int)(i % (2 * kFrameKernels)) / 2 >= nk) continue;  // kernels the caller does not ask for
        if (hipEventCreate(&marks[i]) != hipSuccess) { rc = RT_ERR_HIP; ctx->err = "hipEventCreate failed"; break; }
    }
    for (int k = 0; k < n; ++k) kernel_ms[k] = k < nk ? 0.0f : -1.0f;
    for (int i = 0; i < iters && rc == RT_OK; ++i) {
        const int f = first_frame + i;
        if (frames) rc = rt_build_bvh(ctx);
        ctx->ptMarks = marks.data() + (size_t)i * 2 * kFrameKernels;
        if (rc == RT_OK) rc = rt_path_trace(ctx, f, 0);
        ctx->ptMarks = nullptr;
        if (rc == RT_OK && frames) rc = rt_denoise_post(ctx, f, 0);
        ctx->dnMarks = nullptr;
        if (rc == RT_OK && !frames && hipEventSynchronize(marks[(size_t)i * 2 * kFrameKernels + 2 * kPtKernels - 1]) != hipSuccess)
            rc = RT_ERR_HIP;
    }
    if (rc == RT_OK) rc = sync_streams(ctx);
    std::vector<int> cnt(nk, 0);
    for (int i = 0; i < iters && rc == RT_OK; ++i)
        for (int k = 0; k < nk && rc == RT_OK; ++k) {
            float ms = 0.0f;
            hipEvent_t* m = marks.data() + (size_t)i * 2 * kFrameKernels;
            if (hipEventElapsedTime(&ms, m[2 * k], m[2 * k + 1]) != hipSuccess) { rc = RT_ERR_HIP; ctx->err = "HIP event timing failed"; }
            if (k < kPtKernels || ms > 0.0f) {
                kernel_ms[k] += ms;
                ++cnt[k];
            }
        }
    for (int k = 0; k < nk; ++k) kernel_ms[k] = cnt[k] ? kernel_ms[k] / (float)cnt[k] : 0.0f;
    for (auto& m : marks)
        if (m) (void)hipEventDestroy(m);
    return rc;
}

int rt_time_path_trace_kernels(rt_context* ctx, int iters, float* kernel_ms, int n) {
    if (ctx && ctx->inited && ctx->postStream) {  // kernels are timed serially on the context stream
        void* post = ctx->postStream;
        int rc = rt_set_post_stream(ctx, nullptr);
        if (rc == RT_OK) rc = rt_time_path_trace_kernels(ctx, iters, kernel_ms, n);
        const int rc2 = rt_set_post_stream(ctx, post);
        return rc != RT_OK ? rc : rc2;
    }
    return time_kernels(ctx, 1, iters, kernel_ms, n, false);
}

int rt_time_frame_kernels(rt_context* ctx, int first_frame, int iters, float* kernel_ms, int n) {
    return time_kernels(ctx, first_frame, iters, kernel_ms, n, true);
}

int rt_frame_marks_begin(rt_context* ctx, int frames, uint32_t kernel_mask) {
    if (!ctx || frames < 0 || frames > 100000 || (kernel_mask & ~((1u << kFrameKernels) - 1u)) != 0) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_frame_marks_begin before rt_init"; return RT_ERR_STATE; }
    if (int rc = sync_streams(ctx, false)) return rc;  // the events of earlier frames are complete
    ctx->dnMarks = nullptr;
    const size_t need = (size_t)frames * 2 * kFrameKernels;
    while (ctx->markPool.size() < need) {
        hipEvent_t e = nullptr;
        HIP_TRY(ctx, hipEventCreate(&e));
        ctx->markPool.push_back(e);
    }
    ctx->markRing.assign(need, nullptr);  // unmarked kernels keep null entries (no event recorded)
    for (size_t i = 0; i < need; ++i)
        if (kernel_mask & (1u << ((i % (2 * kFrameKernels)) / 2))) ctx->markRing[i] = ctx->markPool[i];
    ctx->markMask = kernel_mask;
    ctx->markFrames = frames;
    ctx->markNext = 0;
    return RT_OK;
}

int rt_frame_marks_read(rt_context* ctx, float* kernel_ms, int n, int* frames_recorded) {
    if (!ctx || !kernel_ms || n < kPtKernels) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_frame_marks_read before rt_init"; return RT_ERR_STATE; }
    if (int rc = sync_streams(ctx)) return rc;
    const int frames = ctx->markNext, nk = n < kFrameKernels ? n : kFrameKernels;
    for (int k = 0; k < nk; ++k) {
        kernel_ms[k] = -1.0f;
        if (!(ctx->markMask & (1u << k))) continue;
        float sum = 0.0f;
        int cnt = 0;
        for (int i = 0; i < frames; ++i) {
            const hipEvent_t* m = ctx->markRing.data() + (size_t)i * 2 * kFrameKernels;
            float ms = 0.0f;
            HIP_TRY(ctx, hipEventElapsedTime(&ms, m[2 * k], m[2 * k + 1]));
            if (k < kPtKernels || ms > 0.0f) {  // a denoise kernel the frame did not launch reads 0
                sum += ms;
                ++cnt;
            }
        }
        kernel_ms[k] = cnt ? sum / (float)cnt : 0.0f;
    }
    if (frames_recorded) *frames_recorded = frames;
    ctx->markFrames = 0;
    ctx->markNext = 0;
    ctx->dnMarks = nullptr;
    return RT_OK;
}

size_t rt_array_bytes(const rt_context* ctx, int what) {
    if (!ctx) return 0;
    const size_t NP = ctx->mesh.triCountPadded, B = ctx->B, P = (size_t)ctx->renderW * ctx->renderH;
    switch (what) {
        case RT_ARR_VERTICES: return (size_t)ctx->nv * 12;
        case RT_ARR_INDICES: return NP * 12;
        case RT_ARR_NORMALS: return (size_t)ctx->nv * 12;
        case RT_ARR_TRI_POS: return NP * 48;
        case RT_ARR_TRI_NRM: return NP * 48;
        case RT_ARR_AABBS: return NP * 24;
        case RT_ARR_MORTON: return B * 4096;
        case RT_ARR_REORDER: return B * 4096;
        case RT_ARR_NODES: return B * 1024 * 64;
        case RT_ARR_TLAS_AABBS: return B * 24;
        case RT_ARR_TLAS_MORTON: return 4096;
        case RT_ARR_TLAS_REORDER: return 4096;
        case RT_ARR_TLAS_NODES: return B * 64;
        case RT_ARR_BVH_ARENA: return arena_bytes(B, NP);
        case RT_ARR_TLAS_SCENE_AABB: return 24;
        case RT_ARR_BATCH_SCENE_AABBS: return B * 24;
        case RT_ARR_HITS: return P * 16;
        case RT_ARR_HIT_NORMALS: return P * 16;
        case RT_ARR_HIT_FAKE_NORMALS: return P * 16;
        case RT_ARR_HIT_STATS: return P * 16;
        case RT_ARR_RAYS: return P * 4;
        case RT_ARR_SKY_PDF: case RT_ARR_SKY_CDF: return (size_t)kSkySize * 4;
        case RT_ARR_SUN_PDF: case RT_ARR_SUN_CDF: return (size_t)kSunSize * 4;
        case RT_ARR_SUN_DIR: return 16;
        case RT_ARR_HISTOGRAM: return 256;
        case RT_ARR_EXPOSURE: return 16;
        case RT_ARR_COLOR4: return (size_t)((ctx->renderW + 3) / 4) * ((ctx->renderH + 3) / 4) * 8;
        case RT_ARR_COLOR16: return (size_t)((((ctx->renderW + 3) / 4) + 3) / 4) * ((((ctx->renderH + 3) / 4) + 3) / 4) * 8;
        case RT_ARR_COLOR64: {
            const size_t w16 = (((size_t)ctx->renderW + 3) / 4 + 3) / 4, h16 = (((size_t)ctx->renderH + 3) / 4 + 3) / 4;
            return ((w16 + 3) / 4) * ((h16 + 3) / 4) * 8;
        }
        case RT_ARR_RGBA8: return (size_t)ctx->screenW * ctx->screenH * 4;
        case RT_ARR_HDR: return P * 16;
        case RT_ARR_PT_STATS: return P * 16;
        case RT_ARR_TEX_ALBEDO_AO: case RT_ARR_TEX_NORMAL_ROUGHNESS: return (size_t)kTexTexels * 8;
        case RT_ARR_TEX_HEIGHT: return (size_t)kTexTexels * 2;
        case RT_ARR_PT_QUEUE: return 64 * 4;
        case RT_ARR_PT_Q3_ORIGINS:
        case RT_ARR_PT_Q3_DIRS:
        case RT_ARR_PT_Q4_ORIGINS:
        case RT_ARR_PT_Q4_DIRS: return (size_t)ctx->fr.ws.cap * 16;
        default: return 0;
    }
}

int rt_download(const rt_context* cctx, int what, void* dst, size_t bytes) {
    rt_context* ctx = const_cast<rt_context*>(cctx);
    if (!ctx || !dst) return RT_ERR_ARG;
    if (!ctx->inited) { ctx->err = "rt_download before rt_init"; return RT_ERR_STATE; }
    const void* src = nullptr;
    switch (what) {
        case RT_ARR_VERTICES: src = ctx->dVerts; break;
        case RT_ARR_INDICES: src = ctx->dIdx; break;
        case RT_ARR_NORMALS: src = ctx->dNormals; break;
        case RT_ARR_TRI_POS: src = ctx->dTriPos; break;
        case RT_ARR_TRI_NRM: src = ctx->dTriNrm; break;
        case RT_ARR_AABBS: src = ctx->dAabbs; break;
        case RT_ARR_MORTON: src = ctx->dMorton; break;
        case RT_ARR_REORDER: src = ctx->dReorder; break;
        case RT_ARR_NODES: src = ctx->dNodes; break;
        case RT_ARR_BVH_ARENA: src = ctx->dNodes; break;
        case RT_ARR_TLAS_AABBS: src = ctx->dTlasAabbs; break;
        case RT_ARR_TLAS_MORTON: src = ctx->dTlasMorton; break;
        case RT_ARR_TLAS_REORDER: src = ctx->dTlasReorder; break;
        case RT_ARR_TLAS_NODES: src = ctx->dTlasNodes; break;
        case RT_ARR_TLAS_SCENE_AABB: src = ctx->dTlasScene; break;
        case RT_ARR_BATCH_SCENE_AABBS: src = ctx->dBatchScene; break;
        case RT_ARR_HITS: src = ctx->dHits; break;
        case RT_ARR_HIT_NORMALS: src = ctx->dHitNrm; break;
        case RT_ARR_HIT_FAKE_NORMALS: src = ctx->dHitFake; break;
        case RT_ARR_HIT_STATS: src = ctx->dHitStats; break;
        case RT_ARR_RAYS: src = ctx->fr.rays; break;
        case RT_ARR_SKY_PDF: src = ctx->fr.skyPdf; break;
        case RT_ARR_SKY_CDF: src = ctx->fr.skyCdf; break;
        case RT_ARR_SUN_PDF: src = ctx->fr.sunPdf; break;
        case RT_ARR_SUN_CDF: src = ctx->fr.sunCdf; break;
        case RT_ARR_HISTOGRAM: src = ctx->fr.histogram; break;
        case RT_ARR_EXPOSURE: src = ctx->fr.exposure; break;
        case RT_ARR_COLOR4: src = ctx->fr.c4; break;
        case RT_ARR_COLOR16: src = ctx->fr.c16; break;
        case RT_ARR_COLOR64: src = ctx->fr.c64; break;
        case RT_ARR_RGBA8:  // the last frame's output, wherever it was drawn (rt_draw_device)
            if (bytes < rt_array_bytes(ctx, what)) { ctx->err = "destination too small"; return RT_ERR_ARG; }
            return copy_rgba_out(ctx, dst);
        case RT_ARR_HDR: src = ctx->fr.hdr; break;
        case RT_ARR_PT_STATS: src = ctx->fr.ptStats; break;
        case RT_ARR_TEX_ALBEDO_AO: src = ctx->fr.texAlbedo; break;
        case RT_ARR_TEX_NORMAL_ROUGHNESS: src = ctx->fr.texNormal; break;
        case RT_ARR_TEX_HEIGHT: src = ctx->fr.texHeight; break;
        case RT_ARR_PT_QUEUE: src = ctx->fr.lastCounters ? ctx->fr.lastCounters : ctx->fr.ws.counters; break;
        case RT_ARR_PT_Q3_ORIGINS: src = ctx->fr.camQ3[ctx->fr.lastSlot].rayO; break;
        case RT_ARR_PT_Q3_DIRS: src = ctx->fr.camQ3[ctx->fr.lastSlot].rayD; break;
        case RT_ARR_PT_Q4_ORIGINS: src = ctx->fr.camQ4[ctx->fr.lastSlot].rayO; break;
        case RT_ARR_PT_Q4_DIRS: src = ctx->fr.camQ4[ctx->fr.lastSlot].rayD; break;
        case RT_ARR_SUN_DIR: {
            if (bytes < 16) { ctx->err = "destination too small"; return RT_ERR_ARG; }
            float* o = (float*)dst;
            memcpy(o, ctx->fr.sunDir, 12);
            o[3] = ctx->fr.cosThetaMax;
            return RT_OK;
        }
        default: ctx->err = "unknown array"; return RT_ERR_ARG;
    }
    const size_t need = rt_array_bytes(ctx, what);
    if (bytes < need) { ctx->err = "destination too small"; return RT_ERR_ARG; }
    if (int rc = sync_streams(ctx)) return rc;
    if (what == RT_ARR_TRI_POS) {  // the arena's 64-B triangle records -> the reference's [N][3] float4
        HIP_TRY(ctx, hipMemcpy2D(dst, 48, src, 64, 48, ctx->mesh.triCountPadded, hipMemcpyDeviceToHost));
        return RT_OK;
    }
    HIP_TRY(ctx, hipMemcpy(dst, src, need, hipMemcpyDeviceToHost));
    if (what == RT_ARR_NODES || what == RT_ARR_TLAS_NODES) {
        // the reference's q3 (idxLeft, idxRight, isLeftLeaf, isRightLeaf) from the child references
        // the build keeps in q3.z (traverse.h, the record arena); a slot never written stays zero
        uint32_t* q = (uint32_t*)dst;
        for (size_t k = 0; k < need / 64; ++k) {
            uint32_t* q3 = q + 16 * k + 12;
            const uint32_t cl = q3[2] & 0xFFFFu, cr = q3[2] >> 16;
            q3[0] = cl & 0x7FFFu;
            q3[1] = cr & 0x7FFFu;
            q3[2] = (cl >> 15) & 1u;
            q3[3] = (cr >> 15) & 1u;
        }
    }
    return RT_OK;
}

}  // extern "C"
