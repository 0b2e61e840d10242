// context.h — host-side renderer state behind the C-ABI (the RayTracer of kernel.cuh:431-621).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/rtx_amd.h"
#include "bvh_kernels.h"
#include "frame_kernels.h"
#include "scene_gen.h"
#include "soil_textures.h"

struct HostCamera {  // Camera::update outputs (kernel.cuh:103-121)
    float pos[3], dir[3], left[3], up[3];
    float yaw, pitch, focal, aperture;
    float res[2], invRes[2], fov[2], tanHalfFov[2];
    float adjustedLeft[3], adjustedUp[3], adjustedFront[3], apertureLeft[3], apertureUp[3];
};

// Device buffers of RayTracer::draw after the BVH (kernel.cu:259-398)
// Build outputs and scratch of one LBVH (bvh_build.hip).  With frame pipelining there are two,
// so frame f+1's build and camera rays run beside frame f's trace kernels.
// Bytes of an LBVH set's record arena (traverse.h): B*1024 BLAS nodes, B TLAS nodes and NP
// triangle records of 64 B.  BvhBufs::nodes is the arena; tlasNodes and triPos point into it.
inline size_t arena_bytes(size_t B, size_t NP) { return (B * 1024 + B + NP) * 64; }

struct BvhBufs {
    float4* triPos = nullptr;
    float4* triNrm = nullptr;
    float* aabbs = nullptr;
    float* batchScene = nullptr;
    uint32_t* morton = nullptr;
    uint32_t* reorder = nullptr;
    void* nodes = nullptr;
    float* tlasAabbs = nullptr;
    float* tlasScene = nullptr;
    uint32_t* tlasMorton = nullptr;
    uint32_t* tlasReorder = nullptr;
    void* tlasNodes = nullptr;
    uint32_t* counter = nullptr;
};

// G-buffer sets in flight with frame pipelining: with four, frame f+4's camera rays wait for the
// denoise of f instead of f+3's for f's; 3 -> 4 measured 0.787 -> 0.771 ms per pipelined 1080p
// frame (tools/ab.sh, three repeats, profiles/r05_ab/gbuffer_sets/)
#ifndef RTX_GB_SETS  // A/B builds only (tools/abl_build.sh): 2..4 with RT_GBUFFER_SETS set alike
#define RTX_GB_SETS RT_GBUFFER_SETS
#endif
constexpr int kGbSets = RTX_GB_SETS;  // G-buffer / camera-output sets in flight with frame pipelining

struct FrameResources {
    bool ready = false;
    // sky / sun (kernel.cu:280-307)
    float* solar = nullptr;
    float* limb = nullptr;
    float* cie = nullptr;
    float4* sky = nullptr;
    float* skyPdf = nullptr;
    float* skyCdf = nullptr;
    float4* sun = nullptr;
    float* sunPdf = nullptr;
    float* sunCdf = nullptr;
    float* scanSums = nullptr;
    float* skyTree = nullptr;   // light-CDF probe heaps (kSkyTreeNodes / kSunTreeNodes)
    float* sunTree = nullptr;
    float* lightSel = nullptr;   // [4] SampleLight's per-frame terms (k_light_select)
    bool skyValid = false;
    rt_sky_params lastSky{};
    float sunDir[3] = {0, 1, 0};
    float cosThetaMax = 1.0f, sunArea = 0.0f;
    // soil textures (init.cu:524-577)
    uint2* texAlbedo = nullptr;
    uint2* texNormal = nullptr;
    uint16_t* texHeight = nullptr;  // SoilHeight (ushort chain; feeds only the reference's disabled displacement)
    // path-trace G-buffer (pathtrace.cuh:11-128): the set the last path trace wrote.  With a
    // post stream (rt_set_post_stream) the path tracer cycles through kGbSets sets, so the
    // camera rays of frame f+1 and the rest of frame f are traced while frame f-1 is denoised;
    // without one it always uses set 0.
    uint2* gColor[kGbSets] = {};
    uint2* gNormal[kGbSets] = {};
    uint2* gAlbedo[kGbSets] = {};
    uint16_t* gDepth[kGbSets] = {};
    uint32_t* gMotion[kGbSets] = {};
    int gbSet = 0;
    bool setInFlight[kGbSets] = {};  // a denoise on the post stream reads this set
    uint2* color = nullptr;
    uint2* normal = nullptr;
    uint2* albedo = nullptr;
    uint16_t* depth = nullptr;
    uint32_t* motion = nullptr;
    uint32_t* rays = nullptr;
    uint4* ptStats = nullptr;
    unsigned long long* rayCounter = nullptr;
    PtWorkspace ws{};              // wavefront queues of the path tracer (pathtrace.hip)
    // camera-kernel outputs, one slot per G-buffer set (the camera rays of frame f+1 are traced
    // while the shade/trace kernels of frame f still read slot f's hit records)
    float4* camHit0Rec[kGbSets] = {};
    float* camHit0Err[kGbSets] = {};
    uint32_t* camSurface[kGbSets] = {};
    uint32_t* camCount[kGbSets] = {};  // counter block per slot (PtWorkspace::counters)
    uint32_t* lastCounters = nullptr;  // the block of the last path trace (RT_ARR_PT_QUEUE)
    // serial frames: three counter blocks in turn, syncCount[0] = camCount[0]; the resolve of a
    // frame using block b zeroes block b + 2 (syncZeroed), so the camera kernel of the frame after
    // next needs no memset — and the next frame's, traced ahead (spec), has a zeroed block of its own
    uint32_t* syncCount[3] = {};
    int syncIdx = 0;
    bool syncZeroed[3] = {};
    // synchronous draws: the next frame's camera rays traced ahead, beside this frame's bounces and
    // denoise, into the other G-buffer set (frame.cpp launch_spec_camera); the next rt_path_trace
    // uses them when its launch parameters equal `p`, and traces them again otherwise
    struct Spec {
        bool valid = false;
        bool shade = false;  // the shade kernel went ahead too
        int block = 0;
        PathTraceParams p{};
    } spec;
    bool specReady = false;          // set 1's buffers and the events exist (ensure_sync_spec)
    bool gbBound = false;            // a G-buffer is the caller's (rt_bind_buffer): no set rotation
    unsigned long long* specRayCounter = nullptr;  // the rays of the launches ahead (folded in when used)
    int specCounts = 0;  // specRayCounter holds: 0 nothing, 1 the counts of used launches (to fold), 2 dropped ones
    bool camInFlight[kGbSets] = {};
    // ... and the bounce queues with their hit records, one slot per set when the shade kernel
    // runs on the side stream (shadeOnSide: frame f+1's shade appends to its queues while frame
    // f's tracers and resume kernels still read theirs); slot 0 is `ws`'s own buffers
    PtQueue camQ3[kGbSets] = {}, camQ4[kGbSets] = {};
    float4* camHitRec[kGbSets] = {};
    float* camHitErr[kGbSets] = {};
    float4* camPathL[kGbSets] = {};
    uint32_t* camPending[kGbSets] = {};
    int lastSlot = 0;                  // slot of the last path trace (RT_ARR_PT_Q*)
    // queue 3's length after the last serial path trace, copied to pinned host memory behind it
    // (the fused chain's on/off choice for serial frames)
    unsigned long long* q3Host = nullptr;  // {length, tag} stored by k_pt_resolve (poll_q3)
    uint32_t q3Tag = 0;                    // tag of the serial frame whose length is pending
    bool q3Pending = false;
    uint32_t lastQ3 = 0;
    bool lastChain = false;  // the last path trace ran the fused k_pt_chain (rt_info.lastChain)
    HistCamera hist{};
    bool histValid = false;
    // denoise + post (denoising.cu, postprocessing.cu)
    uint2* colorB = nullptr;       // ping-pong partner of color
    uint2* accum = nullptr;        // AccumulationColorBuffer (the latest)
    uint2* accumAlt = nullptr;     // the list chain writes this one and swaps (null: in place only)
    bool accumBound = false;       // accum is the caller's (rt_bind_buffer): the list chain copies back
    uint2* histBuf[2] = {};        // HistoryColorBuffer pair: histBuf[histIdx] is the latest, TemporalFilter2
    int histIdx = 0;               // writes the other one, then they swap roles
    uint16_t* histDepth = nullptr; // HistoryDepthBuffer
    uint16_t* noise8 = nullptr;
    uint16_t* noise16 = nullptr;
    uint32_t* chainCounter = nullptr;  // k_downscale_chain's finished-workgroup count (re-armed by its last one)
    uint32_t* tileList = nullptr;  // the noise-gated passes' active-tile lists (denoise.hip)
    uint32_t tileCap = 0;
    int tileParity = 0;            // counter set of the next list frame
    uint2* c4 = nullptr;
    uint2* c16 = nullptr;
    uint2* c64 = nullptr;
    uint2* bloom4 = nullptr;       // BloomBuffer4 / BloomBuffer16 (postprocessing.cu:73-88)
    uint2* bloom16 = nullptr;
    uint32_t* histogram = nullptr;
    float* exposure = nullptr;
    uint2* scaledA = nullptr;
    uint2* scaledB = nullptr;
    uint32_t* rgba = nullptr;
    uint32_t* outRgba = nullptr;   // where the last rt_denoise_post wrote RGBA8 (rgba or a draw target)
    uint32_t outPitch = 0;         // its row pitch in pixels
    uint32_t* drawTarget = nullptr;  // set by rt_draw_device for the frame it enqueues
    uint32_t drawPitch = 0;
    float4* hdr = nullptr;
    uint2* renderColor = nullptr;  // buffer that currently holds RenderColorBuffer
    uint2* scaledColor = nullptr;  // buffer that currently holds ScaledColorBuffer
    double lastDrawTime = -1.0;    // wall clock of the previous rt_draw (s)
    float drawDt = -1.0f;          // this rt_draw's frame time (ms), taken once by UpdateFrame
};

struct InputState {  // InputControl (inputControl.cu:8-25) + RayTracer::cursorReset (kernel.cuh:465)
    float moveSpeed = 0.01f;
    float cursorMoveSpeed = 0.001f;
    double xpos = 0, ypos = 0;
    bool moveW = false, moveS = false, moveA = false, moveD = false, moveC = false, moveX = false;
    float deltax = 0, deltay = 0;
    bool cursorReset = true;
};

struct rt_context {
    // ---- settings (GlobalSettings, globalSettings.h:5-22) + extensions
    int screenW = 1920, screenH = 1080;
    int renderW = 1920, renderH = 1080;
    int histW = 1920, histH = 1080;   // historyRenderWidth / Height (kernel.cu:83-84): previous frame's size
    int allocW = 1920, allocH = 1080; // render size every render-size buffer is allocated for (the max)
    int allocStripRows = 1080;        // strip rows the path-trace workspace is allocated for
    bool fullFrame = true;            // no strip split: dynamic resolution may resize the frame
    bool useDynamicResolution = true;
    float targetFps = 60.0f;
    int maxWidth = 3840, maxHeight = 2160, minWidth = 640, minHeight = 480;
    std::string inputMeshFileName, inputCameraFileName, cameraSaveFileName;
    std::vector<std::string> inputTextureFileNames;
    bool loadCameraAtInit = false;
    int chunkDim = 1;
    std::string meshFile;  // [scene] meshFile: meshProcessor .bin instead of the procedural scene
    int spp = 1;
    int bvhThreads = 0;  // LBVH workgroup shape: 0 = by batch count, 512 or 1024 ([render] bvhThreads)
    int stripY0 = 0, stripRows = -1;  // [render] stripY0/stripRows: screen-strip split
    int stripCount = 1, stripIndex = 0;  // [render] stripCount/stripIndex: interleaved row blocks (row_of)
    int device = -1;
    int materialOverride = -1;  // [render] materialOverride: one material for every triangle (tests)
    // [debug] fault injection (tests): a batch whose TLAS leaf box is never published, and the TLAS
    // workgroup's wait bound (rt_device.h report_status)
    uint32_t bvhSkipPublish = 0xFFFFFFFFu;
    int bvhSkipBuilds = -1;  // [debug] bvhSkipPublishBuilds: the fault applies to this many builds (-1: all)
    float bvhWaitMs = 1000.0f;
    uint32_t buildSeq = 0;   // LBVH builds issued so far (a timeout report names the build)
    // [tuning] scheduling knobs (A/B aids, config only; the defaults are the measured best,
    // DESIGN.md §7): the device-buffer arena, plain prioritised streams instead of CU-masked ones,
    // the queue tracers' workgroups per CU (0: automatic), the bounce-chain choice (0 off, 1 serial
    // frames with a short queue 3, 2 always), the shade kernel on the side stream, and the
    // pipelined frame's issue points (-1: automatic)
    struct Tuning {
        bool arena = true;
        bool prioStreams = false;
        int tracePerCu = 0, trace4PerCu = 0, trace3ShortPerCu = 2;
        int chain = 1;
        bool shadeOnSide = true;
        int shadeBlocksPerCu = 0;  // k_pt_shade0's grid per CU (0: its residency)
        int overlapAfter = -1, cameraAfter = -1;
        bool syncSpec = true;   // synchronous draws trace the next frame's camera rays ahead
        int specChain = -1;     // ... and their bounces with the fused chain (1), the four kernels (0) or by queue 3's length (-1)
        int specAfter = 1;      // ... the next camera rays after kernel k of this frame (1 shade, 2 trace<3>, ..)
        int specShade = 2;      // ... and the next frame's shade kernel after them: 0 never, 1 beside the lean kernels, 2 always
        int specShadePerCu = 2; // ... that shade kernel's grid per CU (0: its residency)
        int specTracePerCu = 2; // ... this frame's bounce chain / queue-3 tracer at so many workgroups per CU (0: as usual)
        int dnSplit = 0;        // the denoise list passes at two threads per pixel: 0 never, 1 synchronous frames, 2 always
        bool dnFold = false;    // the last a-trous pass over list 1 only, its other tiles written by the first
    } tune;

    std::string err;
    bool inited = false;
    rt_params params{};
    rt_camera camera{};
    int nextFrame = 1;     // frameNum of the next draw (kernel.cu:64 starts at 1)
    int lastFrame = 0;
    float deltaMs = 16.667f;
    InputState input;

    // ---- scene
    rtscene::SceneMesh mesh;
    uint32_t B = 0, nv = 0;

    // ---- device
    int cuCount = 0;                   // the device's CUs (LBVH workgroup shape)
    uint64_t wallTicksPerMs = 100000;  // s_memrealtime rate (hipDeviceAttributeWallClockRate)
    uint32_t* status = nullptr;        // pinned host words the kernels report failures into (kStatus*)
    hipStream_t stream = nullptr;      // stream every stage is enqueued on
    hipStream_t ownStream = nullptr;   // the one rt_init created (destroyed by rt_destroy)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipStream_t postStream = nullptr;  // optional: denoise + post run here (rt_set_post_stream)
    hipStream_t ownPostStream = nullptr;  // created by an asynchronous rt_draw_device (destroyed by rt_destroy)
    hipStream_t sideStream = nullptr;  // pipelining: LBVH build + camera rays of the next frame
    hipEvent_t ptDone[kGbSets] = {}, postDone[kGbSets] = {}, overlapEv = nullptr;
    rt_collective_fn hook = nullptr;     // multi-GPU strip-local denoise exchanges (rt_set_collective_hook)
    void* hookArg = nullptr;
    uint32_t hookStages = (1u << RT_HOOK_HISTOGRAM) | (1u << RT_HOOK_ROWS);  // rt_set_hook_stages
    hipStream_t gatherStream = nullptr;  // optional: the caller's G-buffer gathers (rt_set_gather_stream)
    bool gatherOn = false;               // gatherStream is set (it may be the null stream)
    hipEvent_t gatherDone[kGbSets] = {};
    bool postGather = false;             // the pending denoise also waits for gatherDone[its set]
    hipEvent_t buildDone[2] = {}, bvhFree[2] = {}, camDone[kGbSets] = {}, restDone[kGbSets] = {};
    bool bvhInFlight[2] = {false, false}, buildOnSide[2] = {false, false};
    BvhBufs bvh[2];
    int bvhSet = 0;
    bool bvhPrebuilt = false;  // synchronous draws: the next frame's LBVH is being built into set bvhSet ^ 1
    // frame pipelining: rt_denoise_post(f) is enqueued on the post stream only once the next
    // path trace has enqueued kernel `overlapAfter` (so it fills the trace stages' idle tails), or
    // at the next host read / denoise call, whichever comes first
    bool postPending = false;
    int postPendingSet = 0;
    int overlapAfter = 1;  // after k_pt_shade0: measured best at 1-8 ranks
    int cameraAfter = 3;   // the next frame's camera rays start after this frame's kernel cameraAfter
                           // ends (0: no gate; 1 GPU), kernel 2 = trace<3> on 2 GPUs, kernel 3 =
                           // resume<3> on more (set by rt_set_post_stream)
    hipEvent_t cameraGate = nullptr;
    hipEvent_t specGate = nullptr, specDone = nullptr;  // synchronous draws' camera rays traced ahead
    bool cameraGated = false;
    // pipelined frames: the shade kernel follows the camera kernel on the side stream (set by
    // rt_set_post_stream), so the next frame's shading runs beside this frame's tracers;
    // the context stream keeps trace<3> .. resolve
    bool shadeOnSide = false;
    DenoisePostParams postParams{};
    hipEvent_t* ptMarks = nullptr;  // set only inside rt_time_path_trace_kernels
    hipEvent_t* dnMarks = nullptr;  // the denoise marks of the frame the last marked path trace traced
    // rt_frame_marks_begin: events around the marked kernels of the next markFrames frames (path trace
    // and denoise / post: 2 * kFrameKernels ring entries per frame)
    std::vector<hipEvent_t> markPool, markRing;  // ring: pool entries of the marked kernels, else null
    uint32_t markMask = 0;
    int markFrames = 0, markNext = 0;
    float* dVerts = nullptr;
    float* dNormals = nullptr;
    uint32_t* dIdx = nullptr;
    uint32_t* dAdjOff = nullptr;
    uint32_t* dAdjCorner = nullptr;
    float4* dTriPos = nullptr;
    float4* dTriNrm = nullptr;
    float* dAabbs = nullptr;
    float* dBatchScene = nullptr;
    uint32_t* dMorton = nullptr;
    uint32_t* dReorder = nullptr;
    void* dNodes = nullptr;
    float* dTlasAabbs = nullptr;
    float* dTlasScene = nullptr;
    uint32_t* dTlasMorton = nullptr;
    uint32_t* dTlasReorder = nullptr;
    void* dTlasNodes = nullptr;
    uint32_t* dCounter = nullptr;
    uint8_t* dBlueNoise = nullptr;
    float4* dHits = nullptr;
    float4* dHitNrm = nullptr;
    float4* dHitFake = nullptr;
    uint32_t* dHitStats = nullptr;
    FrameResources fr{};  // path-trace / denoise / post buffers (frame_kernels.h)

    std::vector<void*> allocations;
    // device arena (rt_dalloc_bytes): buffers up to kArenaMaxBuffer are carved from 256-MiB chunks
    char* arenaPtr = nullptr;
    size_t arenaUsed = 0, arenaCap = 0;
};

// helpers shared by the C-ABI translation units
#define HIP_TRY(ctx, expr)                                                            \
    do {                                                                              \
        hipError_t e__ = (expr);                                                      \
        if (e__ != hipSuccess) {                                                      \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e__);          \
            return RT_ERR_HIP;                                                        \
        }                                                                             \
    } while (0)

int rt_dalloc_bytes(rt_context* ctx, void** p, size_t bytes);  // hipMalloc, freed by rt_destroy
template <typename T>
int dalloc(rt_context* ctx, T** p, size_t bytes) {
    void* q = nullptr;
    const int rc = rt_dalloc_bytes(ctx, &q, bytes);
    *p = (T*)q;
    return rc;
}
int rt_create_stream(rt_context* ctx, hipStream_t* s, bool high);  // context.cpp: renderer streams
extern "C" int ensure_bvh_pair(rt_context* ctx);  // frame.cpp: second LBVH set, side stream, build events
int rt_frame_init(rt_context* ctx);  // frame.cpp: sky tables, textures, G-buffers
int sync_streams(rt_context* ctx, bool report = true);  // frame.cpp: context, post and side streams (report: RT_ERR_DEVICE)
void poll_q3(rt_context* ctx);       // frame.cpp: the last serial frame's queue-3 length, if stored
int check_device_status(rt_context* ctx);  // frame.cpp: kernel failure reports (RT_ERR_DEVICE)
bool strip_local_denoise(const rt_context* ctx, uint32_t& a, uint32_t& b);  // frame.cpp: next denoise's rows
extern "C" int copy_rgba_out(rt_context* ctx, void* dst);  // frame.cpp: the last frame's RGBA8 to host memory
extern "C" size_t rt_alloc_bytes(const rt_context* ctx, int name);  // frame.cpp: allocated size of a render buffer
extern "C" void bvh_select(rt_context* ctx, int k);  // context.cpp: point the dTriPos.. views at bvh[k]
extern "C" int wait_bvh(rt_context* ctx);  // context.cpp: context stream waits for the LBVH build
std::string rt_data_dir();
void rt_camera_update(const rt_camera& in, int renderW, int renderH, HostCamera& c);
void rt_input_control_update(rt_context* ctx, float deltaTime);  // input.cpp
TraceCamera rt_trace_camera(const HostCamera& c);
