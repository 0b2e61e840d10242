// ORACLE C API — test infrastructure only (see ocommon.h header comment).
// Loaded by tests/ and bench.py's cpu_baseline through ctypes (oracle/_build/liboracle.so).
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct OrcBvhIO {
    // inputs
    const float* vertices;   // [nverts][3]
    const float* normals;    // [nverts][3] or NULL
    const uint32_t* indices; // [triCountPadded][3]
    uint32_t triCount;
    uint32_t triCountPadded;
    // outputs (caller allocated; B = ceil(triCount / 1024))
    float* triangles;        // [triCountPadded][18]  v1 v2 v3 n1 n2 n3
    float* aabbs;            // [triCountPadded][6]   min xyz, max xyz
    uint32_t* mortonUnsorted;  // [B*1024]
    uint32_t* mortonSorted;    // [B*1024]
    uint32_t* reorderIdx;      // [B*1024]
    void* nodes;               // [triCountPadded] canonical 64-B nodes
    float* batchSceneAabbs;    // [B][6]
    float* tlasAabbs;          // [B][6]
    float* tlasSceneAabb;      // [6] the (quirky) reduction box used for TLAS Morton codes
    uint32_t* tlasMortonUnsorted;  // [1024]
    uint32_t* tlasMortonSorted;    // [1024]
    uint32_t* tlasReorderIdx;      // [1024]
    void* tlasNodes;               // [B]
} OrcBvhIO;

// returns B (>0) or a negative error
int orc_build_bvh(const OrcBvhIO* io);
uint32_t orc_morton3(uint32_t x, uint32_t y, uint32_t z);

// GenerateSmoothNormals x2 (kernel.cu:228-257, 313-327) accumulated in triangle order into
// a zeroed buffer. normals: [nverts][3] output.
void orc_smooth_normals(const float* vertices, uint32_t nverts, const uint32_t* indices, uint32_t triCountPadded,
                        float* normals);

typedef struct OrcScene {
    const float* triangles;  // [triCountPadded][18] as written by orc_build_bvh
    const void* nodes;       // BLAS canonical nodes [triCountPadded]
    const void* tlasNodes;   // [B]
    uint32_t triCountPadded;
    uint32_t batchCount;
} OrcScene;

typedef struct OrcHit {
    float t;
    int32_t objectIdx;
    float u, v;
    float normal[3];      // geometric normal, flipped to face the ray (traverse.cuh:193-199)
    float fakeNormal[3];  // interpolated shading normal, flipped likewise
    float pos[3];         // re-projected hit point (geometry.cuh:252-262)
    float offset;         // errT + errP
    uint32_t hit;
    uint32_t nodeVisits;  // internal-node box-pair tests
    uint32_t triTests;    // ray/triangle tests
    uint32_t droppedPushes;  // pushes lost to the 16-entry stack (traverse.h:34-36)
    uint32_t iterations;     // loop iterations used (cap 1024, traverse.h:132)
    uint32_t intoSurface;    // isRayIntoSurface (traverse.cuh:193)
    float ndr;               // normalDotRayDir after the flip (traverse.cuh:192-198)
    uint32_t maxDepth;       // most entries the stack held at once (test diagnostics: deep-stack coverage)
} OrcHit;

// RaySceneIntersect core (traverse.cuh:64-225 without the material bookkeeping) for n rays.
// rays: [n][6] orig xyz, dir xyz.  threads: host threads to use (0 = all).
void orc_intersect(const OrcScene* scene, const float* rays, uint32_t n, OrcHit* hits, int threads);

typedef struct OrcCamera {
    float pos[3];
    float yaw, pitch;
    float focal, aperture;
    float fovX;          // radians
    float resolution[2]; // render width, height
} OrcCamera;

// Camera::update + GenerateRay with blue-noise sample frameNum*4+0 (pathtrace.cuh:40-59,
// raygen.cuh:7-38).  rays: [W*H][6]; also writes the per-pixel ray-cone spread if non-NULL.
void orc_primary_rays(const OrcCamera* cam, uint32_t W, uint32_t H, int frameNum, const uint8_t* bluenoise,
                      float* rays, float* coneSpread);

// Blue-noise sampler (blueNoiseRandGen.h:113-146): value for pixel, sample index, dimension.
float orc_bluenoise(const uint8_t* tables, int px, int py, int sampleIdx, int dim);

// deterministic math probes (rtmath.h), for tests
float orc_rtmath(int fn, float x, float y);

// ---------------------------------------------------------------- sky (sky.cpp)
typedef struct OrcSkyTables {
    const float* skyDataSets;            // 540
    const float* skyDataSetsRad;         // 60
    const float* solarDatasets;          // 1800
    const float* limbDarkeningDatasets;  // 60
    const float* cieX; const float* cieY; const float* cieZ;  // 10 each
} OrcSkyTables;

typedef struct OrcSkyParams {
    float timeOfDay, sunAxisAngle, skyScalar, sunScalar, sunAngle;
} OrcSkyParams;

typedef struct OrcSkyOut {
    float sunDir[3];
    float* skyBuffer;   // [256][512][4]
    float* skyPdf;      // [131072]
    float* skyCdf;      // [131072]
    float* sunBuffer;   // [32][32][4]
    float* sunPdf;      // [1024]
    float* sunCdf;      // [1024]
    float sunArea, sunAngleCosThetaMax;
} OrcSkyOut;

void orc_sky(const OrcSkyTables* tables, const OrcSkyParams* params, OrcSkyOut* out);
void orc_sun_dir(float timeOfDay, float sunAxisAngle, float* out);
void orc_scan(const float* in, float* out, int size, int blockSize);

// ---------------------------------------------------------------- path trace (pathtrace.cpp)
typedef struct OrcFrame {
    OrcScene scene;
    uint32_t triCount;
    int32_t materialOverride;    // < 0: reference materialsIdx (3 for every triangle)
    OrcCamera cam;               // current camera
    OrcCamera histCam;           // camera of the previous frame (HistoryCamera::Setup)
    int frameNum;
    uint32_t spp;                // samples per pixel (build definition)
    const uint8_t* bluenoise;
    const uint16_t* texAlbedoAo;       // ushort4, 11 mip levels concatenated (1024 >> l)
    const uint16_t* texNormalRough;
    const float* skyBuffer; const float* sunBuffer;
    const float* skyCdf; const float* sunCdf;
    float sunDir[3];
    float sunAngleCosThetaMax;
} OrcFrame;

typedef struct OrcGBuffer {
    uint16_t* color;    // [P][4] half rgb + ushort mask
    uint16_t* normal;   // [P][4] half
    uint16_t* albedo;   // [P][4] half
    uint16_t* depth;    // [P] half
    uint16_t* motion;   // [P][2] half
    uint32_t* rays;     // [P] RaySceneIntersect calls that traced (may be NULL)
} OrcGBuffer;

void orc_pathtrace(const OrcFrame* f, uint32_t W, uint32_t H, uint32_t y0, uint32_t rows, OrcGBuffer* out,
                   int threads);
void orc_textures(uint16_t* albedoAo, uint16_t* normalRough);  // 1398101 ushort4 texels each

// ---------------------------------------------------------------- denoise + post (denoise.cpp)
struct rt_params;  // include/rtx_amd.h

typedef struct OrcPostState {  // persists across frames
    uint16_t* accum;       // [P][4] AccumulationColorBuffer
    uint16_t* histColor;   // [P][4] HistoryColorBuffer
    uint16_t* histDepth;   // [P]    HistoryDepthBuffer
    float exposure[4];     // d_exposure (init.cu:331-333: 1,1,1,1)
} OrcPostState;

typedef struct OrcDrawIO {
    uint32_t W, H;          // render size
    uint32_t Ws, Hs;        // screen (output) size
    int frameNum;
    float deltaTime;        // ms, AutoExposure's adaptation step
    const struct rt_params* params;
    const uint8_t* bluenoise;
    uint16_t* color;        // in: PathTrace colour (half3 + mask); out: RenderColorBuffer after denoise
    const uint16_t* normal; const uint16_t* albedo; const uint16_t* depth; const uint16_t* motion;
    uint16_t* noise8;       // out [ceil(W/8) * ceil(H/8)] half (last computed)
    uint16_t* noise16;      // out [ceil(W/16) * ceil(H/16)] half
    uint16_t* c4; uint16_t* c16; uint16_t* c64;   // out DownScale4 chain, half4
    uint32_t* histogram;    // out [64]
    uint16_t* scaled;       // out [Ws*Hs][4] half (ScaledColorBuffer, tone mapped)
    uint8_t* rgba;          // out [Ws*Hs][4] (may be NULL)
    OrcPostState* state;
    uint16_t* bloom4;       // out [ceil(W/4) * ceil(H/4)][4] half (BloomBuffer4; NULL: scratch)
    uint16_t* bloom16;      // out [ceil(W/16) * ceil(H/16)][4] half (BloomBuffer16; NULL: scratch)
    int lensFlare;          // the host-side lens-flare predicate held (orc_lens_flare_setup)
    float sunPos[2];        // LensFlare's sun position (already centred and aspect-scaled)
    int sunUv[2];           // render texel of the sun (LensFlarePred's depth test)
    uint32_t histW, histH;  // historyDim (kernel.cu:266): the previous frame's render size; 0: (W, H)
} OrcDrawIO;

// UpdateFrame's dynamic resolution (kernel.cu:77-100): the next render size from the current
// width and the frame time (ms).  Height clamped to maxH as the renderer does.
void orc_dynamic_resolution(int w, float dt, float targetFps, int minW, int maxW, int maxH, int* outW, int* outH);

// UpdateFrame's sunPos / sunUv (kernel.cu:126-127) and PostProcessing's lens-flare predicate
// (postprocessing.cu:88-94).  Returns 1 when the lens flare pass is launched.
int orc_lens_flare_setup(const OrcCamera* cam, const float* sunDir, uint32_t W, uint32_t H, float* sunPos,
                         int* sunUv);

// TemporalSpatialDenoising + PostProcessing + CopyToOutput; returns < 0 for unsupported settings
int orc_denoise_post(const OrcDrawIO* io);

#ifdef __cplusplus
}
#endif
