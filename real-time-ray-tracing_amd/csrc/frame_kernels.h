// frame_kernels.h — launch parameters of the per-frame kernels after the BVH build:
// sky/sun generation + CDF scan, the path tracer, the SVGF denoiser and post-processing.
// Plain-old-data structs passed by value as kernel arguments; device pointers only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bvh_kernels.h"
#include "rtx_amd.h"

constexpr int kSkyW = 512, kSkyH = 256, kSkySize = kSkyW * kSkyH;  // kernel.cuh SKY_WIDTH/HEIGHT
constexpr int kSunW = 32, kSunH = 32, kSunSize = kSunW * kSunH;    // SUN_WIDTH/HEIGHT
constexpr int kSkyScanBlock = 256, kSunScanBlock = 32;               // SKY/SUN_SCAN_BLOCK_SIZE
constexpr int kTexLevels = 11, kTexSize = 1024;                      // soil textures, 11 mips

// ushort4-texel offset of mip level l in the concatenated chain: sum over k < l of (S >> k)^2
// = 4 (S^2 - (S >> l)^2) / 3 for a power-of-two S (closed form: no loop on the texture path)
static_assert((kTexSize & (kTexSize - 1)) == 0 && kTexSize <= 16384, "power-of-two texture size");
__host__ __device__ constexpr uint32_t tex_level_offset(int l) {
    return 4u * ((uint32_t)(kTexSize * kTexSize) - (uint32_t)(kTexSize >> l) * (uint32_t)(kTexSize >> l)) / 3u;
}
constexpr uint32_t kTexTexels = tex_level_offset(kTexLevels);

// Hosek-Wilkie sky state (UpdateSkyState, sky.cuh:90-146), evaluated on the host
struct SkyState {
    float configs[90];   // 10 spectral channels x 9 coefficients
    float radiances[10];
};

struct SkyGenParams {
    float sunDir[3];
    float skyScalar, sunScalar, sunAngle;  // already clamped (kernel.cu:291-293)
    float cosThetaMax;                     // cos(sunAngle * pi / 360) in float
    SkyState st;
    const float* solar;   // [10][180] h_solarDatasets
    const float* limb;    // [10][6]  h_limbDarkeningDatasets
    const float* cie;     // [3][10]  spectrumCieX | Y | Z
    float4* skyBuffer;    // [256][512]
    float* skyPdf;        // [131072]
    float* skyCdf;        // [131072]
    float4* sunBuffer;    // [32][32]
    float* sunPdf;        // [1024]
    float* sunCdf;        // [1024]
    float* scanSums;      // [>= 512] block totals
    float* skyTree;       // [kSkyTreeNodes] bisection probe tree of skyCdf (cdf_tree)
    float* sunTree;       // [kSunTreeNodes] of sunCdf
    float* lightSel;      // [4] SampleLight's per-frame terms: pSky, maxSky, maxSun, 2 pi (1 - cosThetaMax)
};

// The first levels of SampleLight's CDF bisection (light.cuh:9-31) as a heap: node 1 holds the
// CDF value the search probes first, node j's children 2j / 2j + 1 the values it probes after
// a[mid] >= target / a[mid] < target.  Kernels stage the heap in LDS and walk it for the first
// log2(nodes) probes, then continue in global memory: the same probes, the same result.
constexpr int kSkyTreeNodes = 4096, kSunTreeNodes = 1024;

struct HistCamera { float pos[3], left[3], up[3], dir[3]; };  // HistoryCamera (kernel.cuh:135-155)

// One queue of deferred rays (wavefront path tracing).  Entry i is five float4
// planes: the ray (orig + pixel index, dir + flags) that k_trace_queue reads, and the path
// state the resume kernel needs after the hit.
//   rayO  = orig.xyz, pixel index (bits)            rayD = dir.xyz, flags (bits, kQFlag*)
//   st0   = albedo.xyz, rayConeWidth                 st1  = beta1.xyz, rayConeSpread
//   st2   = beta0.xyz, 0
// rayD.w bit 0: the entry is a shadow ray (isShadowRay).  Only whether a shadow ray, or any
// step-4 ray, hits something decides its sample's colour (the path ends there, and a hit never
// has matType MAT_SKY), so the queue tracer ends those traversals at their first hit.
constexpr uint32_t kQShadowFlag = 1u;

struct PtQueue {
    float4* rayO;
    float4* rayD;
    float4* st0;
    float4* st1;
    float4* st2;
};

// counters[] slots (zeroed before every path-trace launch sequence)
// [12..21]: per-kernel traversal / shading work of detail launches (statsOut set), for the
// per-kernel roofline (bench.py): node visits and triangle tests of the camera kernel, the
// shade kernel's inline (glossy) traces and the two queue tracers; diffuse events of the shade
// and resume<3> kernels; [22] camera rays the scene cull settled without a traversal
enum PtCounter : int { kCntQ3 = 0, kCntQ4 = 1, kCntFetch3 = 2, kCntFetch4 = 3, kCntPending = 4, kCntResume3 = 5,
                       kCntResume4 = 6, kCntResolve = 7, kCntMaxIter3 = 8, kCntMaxIter4 = 9, kCntError = 10,
                       kCntSurface = 11, kCntVisCam = 12, kCntTstCam = 13, kCntVisShade = 14, kCntTstShade = 15,
                       kCntVisQ3 = 16, kCntTstQ3 = 17, kCntVisQ4 = 18, kCntTstQ4 = 19, kCntDiffShade = 20,
                       kCntDiffRes3 = 21, kCntCulledCam = 22, kCntSlots = 23 };
// counters | fetch: [2][8 parts x 16] queue-tracer fetch counters, then [8 parts x 16] the shade
// kernel's batch claims (k_pt_shade0), all zeroed together
constexpr int kWsCounterWords = 64 + 3 * 8 * 16;
constexpr uint32_t kChainMaxQ3 = 1u << 20;  // serial frames fuse the bounce chain below this queue-3 length

struct PtWorkspace {
    float4* hit0Rec;            // [spp][rows*W] camera-ray hits (t, triangle index bits, u, v)
    float* hit0Err;             // [spp][rows*W] their errorT
    PtQueue q3, q4;             // rays deferred at step 3 / step 4 of PathTrace's sequence
    float4* hitRec;             // [cap] (t, triangle index bits, u, v) of the closest hit
    float* hitErr;              // [cap] its errorT
    float4* pathL;              // [rows*W*spp] per-sample radiance of pixels resolved late
    uint32_t* pending;          // [rows*W] pixel (strip-local) | first deferred sample << 26
    uint32_t* surface;          // [rows*W] strip-local pixels with a sample that hit geometry
    // counters + fetch: one block per camera-output slot, zeroed on the camera's stream right
    // before k_pt_camera appends to counters[kCntSurface], so the shade..resolve kernels start
    // with no memset or copy of their own
    uint32_t* counters;         // [kWsCounterWords]: kCntSlots counters, then `fetch`
    uint32_t* fetch;            // [2][8 parts x 16]: k_trace_queue fetch counters, 64 B apart
    uint32_t cap;               // entries per queue (= rows * W * spp)
    uint32_t persistBlocks;     // grid of the persistent queue kernels
    int shadeClaim = 0;         // k_pt_shade0 claims its batches dynamically (synchronous frames)
    uint32_t shadeBlocksPerCu = 0;  // ... on this grid per CU (0: its residency); cus: the device's CUs
    uint32_t cus = 256;
    uint32_t traceBlocks;       // grid of the queue tracer of queue 3 (k_trace_queue)
    uint32_t trace3ShortBlocks = 0;  // its workgroups that run when queue 3 is short (0: all)
    uint32_t trace4Blocks;      // ... of queue 4 (a short queue: a few percent of queue 3)
    int glossy;                 // materials can be glossy: steps 1-2 may trace (materialOverride)
    int microfacet;             // materials can be the microfacet one (materialOverride 4): GGX compiled in
    int chain = 1;              // default materials: trace<3> .. resume<4> as one launch (k_pt_chain)
    uint32_t* itersOut = nullptr;  // optional [cap]: traversal iterations per queue entry (rt_trace_rays)
    unsigned long long* q3HostOut = nullptr;  // optional, pinned host memory: {queue 3's length, q3Tag},
    uint32_t q3Tag = 0;                       // stored by k_pt_resolve in one 64-bit store
    // serial frames alternate two counter blocks: k_pt_resolve zeroes the other one (zeroNext) for
    // the next frame, whose camera kernel then starts without a memset (countersZeroed)
    uint32_t* zeroNext = nullptr;
    int countersZeroed = 0;
};

// The frame's traced-ray count is kept as partial sums in kRayCounterSlots slots 128 B apart
// (one atomic per workgroup into slot blockId % slots; the host adds them): a device-scope
// atomic on one address serialises at the memory side, and one per workgroup on a single
// counter cost ~190 us of a 1080p camera-ray launch.
constexpr int kRayCounterSlots = 256, kRayCounterStride = 16;  // stride in u64

struct PathTraceParams {
    TraceCamera cam;
    float tanHalfFov[2];
    float res[2];
    float halfRes[2];           // res / 2 (exact), from the host: a kernel argument, not a VGPR pair
    HistCamera hist;
    uint32_t width, height;     // full render size (strides)
    uint32_t y0, rows;          // strip rows (row_of): contiguous [y0, y0 + rows) when nStrips = 1
    uint32_t nStrips, strip;
    int frameNum;
    uint32_t spp;               // samples per pixel (>= 1), frame index spp*(frameNum-1)+1+s
    float invSpp;               // 1 / spp when spp is a power of two (exact), else 0 (div_spp)
    int materialOverride;       // < 0: reference material table (material 3 everywhere)
    uint32_t triCount;
    const uint8_t* bluenoise;
    const float4* triPos;       // the record arena's triangle records (traverse.h)
    const float4* triNrm;
    const void* nodes;          // the record arena
    const void* tlasNodes;      // its TLAS nodes
    const uint2* texAlbedo;     // ushort4 texels, kTexLevels levels concatenated
    const uint2* texNormal;
    const float4* skyBuffer;
    const float4* sunBuffer;
    const float* skyCdf;
    const float* sunCdf;
    const float* skyTree;       // [kSkyTreeNodes] (SkyGenParams::skyTree)
    const float* sunTree;       // [kSunTreeNodes]
    const float* lightSel;      // [4] (SkyGenParams::lightSel): uniform loads instead of per-sample math
    float sunDir[3];
    float sunT[3], sunB[3];     // LocalizeSample(sunDir) frame (sky.cuh:64-87), evaluated once on the host
    float cosThetaMax;
    float oneMinusCosThetaMax;  // 1 - cosThetaMax (exact on the host): a kernel argument
    uint2* colorOut;            // [W*H] half3 demodulated colour + ushort material mask
    uint2* normalOut;           // [W*H] half4
    uint2* albedoOut;           // [W*H] half4
    uint16_t* depthOut;         // [W*H] half
    uint32_t* motionOut;        // [W*H] half2
    uint32_t* raysOut;          // optional [W*H] RaySceneIntersect calls that traced
    uint4* statsOut;            // optional [W*H] rays, node visits, triangle tests, diffuse events
    unsigned long long* rayCounter;  // optional: total traced rays, kRayCounterSlots partial sums
    PtWorkspace ws;
};

// TemporalSpatialDenoising + PostProcessing + CopyToOutput (denoise.hip)
struct DenoisePostParams {
    uint32_t W, H;              // render size
    uint32_t Ws, Hs;            // screen size
    uint32_t histW, histH;      // render size of the previous frame (historyDim, kernel.cu:266):
                                // the accumulation / history colour buffers are read at that size
    int frameNum;
    float deltaTime;            // ms
    int temporal, localSpatial, visualize, wideSpatial, temporal2;   // RenderPassSettings
    int postProcess, downScale, histogramOn, autoExposure, sharpen, tonemap;
    int bloom, lensFlare;       // enableBloomEffect; lens-flare pass launched (host predicate)
    int toneMappingType;        // ToneMappingType: 0 Uncharted, 1 ACES1, 2 ACES2, 3 Reinhard (extended)
    float sunPos[2];            // LensFlare's sun position (centred, aspect-scaled)
    int sunUv[2];               // render texel whose depth gates the lens flare (LensFlarePred)
    uint2* bloom4;              // BloomBuffer4 / BloomBuffer16 (half4)
    uint2* bloom16;
    float gain, fixedExposure, maxWhite, gamma;                      // PostProcessParams
    rt_denoising_params dn;
    uint2* colorA;              // path-trace colour in; ping-pong pair
    uint2* colorB;
    uint2* normal;              // written only by the noise-visualize debug pass
    const uint2* albedo;
    uint16_t* depth;            // written only by the noise-visualize debug pass
    const uint32_t* motion;
    uint2* accum;               // AccumulationColorBuffer (the previous frame's, which TemporalFilter reads)
    uint2* accumAlt;            // the list chain's output accumulation buffer (null: none, filters write accum)
    uint2* histColor;           // HistoryColorBuffer of the previous frame (read by TemporalFilter2)
    uint2* histColorOut;        // HistoryColorBuffer written this frame (the other of the pair)
    uint16_t* histDepth;        // HistoryDepthBuffer
    uint16_t* noise8;
    uint16_t* noise16;
    uint2* c4;
    uint2* c16;
    uint2* c64;
    uint32_t* histogram;        // [64]
    float* exposure;            // [4], persistent
    uint2* scaledA;             // screen-size pair
    uint2* scaledB;
    uint32_t* rgba;             // screen-size RGBA8 (the context's own buffer or a caller's device target)
    uint32_t rgbaPitch;         // row pitch of rgba in pixels (>= Ws)
    const uint8_t* bluenoise;
    float4* hdrOut;             // optional render-size float4 copy of the denoised HDR colour
    uint2* finalColor;          // out: buffer holding RenderColorBuffer after denoising
    uint2* finalScaled;         // out: buffer holding ScaledColorBuffer after tone mapping
    int stripLocal;             // multi-GPU: compute only what rows [rowA, rowB) need (rtk_denoise_phase)
    uint32_t rowA, rowB;        // this context's output rows (64-row aligned; [0, H) when not strip-local)
    int histOutSet;             // which buffer of the history pair histColorOut is (the hook reports it)
    int gbSet;                  // G-buffer set the frame was traced into (the hook reports it)
    uint32_t* rgbaTarget;       // strip-local: the caller's draw target, filled from `rgba` after the rows
    uint32_t rgbaTargetPitch;   // exchange (rgba is then the exchanged buffer); pitch in pixels
    int ty0, ty1;               // per launch (set by the launcher): tile rows of the 16x16-tile kernels
    int cty0, cty1;             // the list chain's first a-trous launch: tile rows of the last pass it
                                // finishes for tiles off list 1 (set by the launcher)
    uint32_t* chainCounter;     // k_downscale_chain's workgroup counter (zero between launches)
    int exposureDone;           // set by phase 0 when k_downscale_chain ran AutoExposure
    int histDepthInTemporal;    // k_temporal also copies depth into the history depth (per launch)
    uint2* svgfOut;             // phase 2 -> 3: the colour buffer TemporalSpatialDenoising ended in
    int histDepthDone;          // phase 2 -> 3: k_temporal already wrote the history depth
    uint32_t* tileList;         // active-tile lists of the noise-gated passes (denoise.hip), or null
    uint32_t tileCap;           // tiles the lists can hold (16x16 tiles of the allocated render size)
    int tileParity;             // this frame's counter set (the other one is zeroed by TemporalFilter)
    int listUsed;               // out (phase 0 / 2): the chain ran over the lists; the host flips tileParity
    int listSplit;              // the list passes at two threads per pixel (512-thread workgroups, denoise.hip)
    int listFold;               // the last a-trous pass over list 1 only (the first finishes the other tiles)
    float rcpDepth[3];          // RN(1 / sigma_depth) of TemporalFilter, SpatialFilter7x7, the a-trous passes
    int rcpDepthOk;             // bit k: that sigma is in rt_div_rcp's range (else the taps divide)
    hipEvent_t* marks;          // optional, host side only: 2 * kDnKernels events, marks[2k] / [2k + 1]
                                // recorded right before / after denoise kernel k (null entries: not marked)
};
// the denoise / post kernels of a whole-frame chain, in launch order (the marks' kernel index)
constexpr int kDnKernels = 8;  // k_temporal, k_spatial7, k_spatial5<3>, <6>, <12>, k_temporal2,
                               // k_downscale_chain, k_scale_post

extern "C" hipError_t rtk_denoise_post(DenoisePostParams* p, hipStream_t stream);
// phase 0: denoise .. DownScale4 + Histogram2; phase 1: AutoExposure .. RGBA8 (finalColor of phase 0 in).
// Phase 0 = phase 2 (TemporalSpatialDenoising: TemporalFilter .. the a-trous passes) then phase 3
// (TemporalFilter2 .. Histogram2).
extern "C" hipError_t rtk_denoise_phase(DenoisePostParams* p, hipStream_t stream, int phase);
// the render-size float4 HDR copy (rt_draw's hdr_out) of a denoised colour buffer
extern "C" hipError_t rtk_hdr_out(const uint2* color, float4* hdr, size_t n, hipStream_t stream);

extern "C" hipError_t rtk_launch_sky(const SkyGenParams* p, hipStream_t stream);
// MipmapGen (texture.hip): levels 1.. of a square 16-bit chain whose level 0 is in place
extern "C" hipError_t rtk_launch_mipgen(uint16_t* chain, int size, int levels, int channels, hipStream_t stream);
extern "C" hipError_t rtk_launch_scan(const float* in, float* out, float* sums, int size, int blockSize,
                                      hipStream_t stream);
// Scan (scan.cuh:258-298) with the reference's postfix flag and size range (rt_scan_device)
extern "C" hipError_t rtk_launch_scan_ex(const float* in, float* out, float* sums, int size, int blockSize,
                                         int postfix, hipStream_t stream);
// kernels of one path-trace launch: camera, shade, trace<3>, resume<3>, trace<4>, resume<4>, resolve
constexpr int kPtKernels = 7;
constexpr int kFrameKernels = kPtKernels + kDnKernels;  // a frame's marks: path trace, then denoise / post
struct PtLaunchHook {
    hipError_t (*fn)(void* arg, int kernel);  // after each kernel is enqueued (1 = shade, 2 = trace<3>, ...)
    void* arg;
};
// The camera kernel (writes the hit records, the surface list and the sky pixels' G-buffer) and
// the rest (shade .. resolve) can go to different streams: the frame pipeline runs the camera
// rays of frame f+1 beside the trace tails of frame f (frame.cpp).  marks: 2 * kPtKernels events,
// marks[2k] / marks[2k + 1] recorded right before / after kernel k on the stream it runs on
// (k = 0 by the camera launcher, 1..6 by the rest; rt_time_path_trace_kernels, rt_time_frame_kernels).
extern "C" hipError_t rtk_launch_pt_camera(const PathTraceParams* p, hipStream_t stream, hipEvent_t* marks);
extern "C" hipError_t rtk_launch_pt_rest(const PathTraceParams* p, hipStream_t stream, hipEvent_t* marks,
                                         const PtLaunchHook* hook);
// The shade kernel alone (kernel 1, marks[2] / marks[3]), for a caller that runs it behind the
// camera kernel on another stream; rtk_launch_pt_rest_after_shade then enqueues trace<3> ..
// resolve and calls the hook for kernel 1 first, with nothing enqueued for it.
extern "C" hipError_t rtk_launch_pt_shade(const PathTraceParams* p, hipStream_t stream, hipEvent_t* marks);
// dst[k * kRayCounterStride] += src[k * kRayCounterStride] over the kRayCounterSlots slots (the
// ray counts of kernels launched ahead, folded into the frame's when it uses them), then src = 0;
// dst null: only the zeroing
extern "C" hipError_t rtk_fold_ray_counts(unsigned long long* dst, unsigned long long* src, hipStream_t stream);
extern "C" hipError_t rtk_launch_pt_rest_after_shade(const PathTraceParams* p, hipStream_t stream, hipEvent_t* marks,
                                                     const PtLaunchHook* hook);
extern "C" int rtk_trace_queue_blocks_per_cu();
extern "C" hipError_t rtk_launch_trace_queue(const PathTraceParams* p, int step, hipStream_t stream);
