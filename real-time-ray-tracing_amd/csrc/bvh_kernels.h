// bvh_kernels.h — launch interface of the LBVH build and traversal kernels (host side).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// words of rt_context::status, the pinned host block kernels report failures into (rt_device.h
// report_status; checked by sync_streams and rt_build_bvh)
constexpr int kStatusTlasTimeout = 0;       // the TLAS workgroup gave up waiting: the number of missing batches
constexpr int kStatusTlasTimeoutBuild = 1;  // ... and the sequence number of the (last) build that did

struct BvhBuildParams {
    const float* vertices;     // [nv][3]
    const float* normals;      // [nv][3]
    const uint32_t* indices;   // [triCountPadded][3]
    uint32_t triCount;
    uint32_t triCountPadded;
    uint32_t batchCount;
    float4* triPos;            // the arena's triangle records [triCountPadded][4]: v1, v2, v3 (w 0), one quad unused
    float4* triNrm;            // [triCountPadded][3] (xyz, 0)
    float* aabbs;              // [triCountPadded][6]
    float* batchSceneAabbs;    // [B][6]
    uint32_t* morton;          // [B*1024] sorted keys
    uint32_t* reorder;         // [B*1024]
    void* nodes;               // the record arena (traverse.h): [B*1024] BLAS nodes, then the TLAS nodes, then
                               // the triangle records (triPos = nodes + 64 * (B*1024 + B) bytes)
    float* tlasAabbs;          // [B][6]
    float* tlasSceneAabb;      // [6]
    uint32_t* tlasMorton;      // [1024]
    uint32_t* tlasReorder;     // [1024]
    void* tlasNodes;           // [B] = nodes + 64 * B*1024 bytes
    uint32_t* counter;         // arrival counter, zero between launches (re-armed by the TLAS workgroup)
    uint32_t threads;          // workgroup shape: 0 = by batch count, 512 or 1024 ([render] bvhThreads)
    uint32_t cus;              // the device's CU count (rt_init), for the shape choice
    uint32_t* status;          // pinned host words of device failure reports (rt_device.h report_status)
    uint64_t waitTicks;        // the TLAS workgroup's wait bound in s_memrealtime ticks
    uint32_t skipPublish;      // fault injection: this batch does not publish (0xFFFFFFFF: none)
    uint32_t buildSeq;         // this build's sequence number in the context (reported with a timeout)
};

struct TraceCamera {
    float pos[3];
    float adjustedFront[3], adjustedLeft[3], adjustedUp[3];
    float apertureLeft[3], apertureUp[3];
    float invRes[2];
};

// The frame rows one context traces (multi-GPU split).  Strip-local row yl maps to
// frame row y0 + yl for a contiguous strip (nStrips = 1); with nStrips > 1 the frame's blocks of
// kRowBlock rows are dealt round-robin and this context owns every block b with b mod nStrips ==
// strip (starting at y0 = 0), so every rank gets an equal share of the expensive (geometry)
// rows wherever the camera puts them.
constexpr uint32_t kRowBlock = 16;
__host__ __device__ inline uint32_t row_of(uint32_t y0, uint32_t nStrips, uint32_t strip, uint32_t yl) {
    return y0 + ((yl / kRowBlock) * nStrips + strip) * kRowBlock + yl % kRowBlock;
}
__host__ __device__ inline uint32_t local_row(uint32_t y0, uint32_t nStrips, uint32_t y) {
    const uint32_t r = y - y0;
    return (r / kRowBlock / nStrips) * kRowBlock + r % kRowBlock;
}
// rows of strip `strip` in a frame of `height` rows
inline uint32_t strip_row_count(uint32_t height, uint32_t nStrips, uint32_t strip) {
    uint32_t n = 0;
    for (uint32_t b = strip; b * kRowBlock < height; b += nStrips) {
        const uint32_t lo = b * kRowBlock, hi = lo + kRowBlock < height ? lo + kRowBlock : height;
        n += hi - lo;
    }
    return n;
}

// The rows one rank denoises in a strip-local (multi-GPU) denoise: the frame's 64-row blocks
// (kDenoiseBlock: one texel row of the 1/64 DownScale4 level) split into nStrips contiguous runs
// as evenly as whole blocks allow; false when there are fewer blocks than strips.
constexpr uint32_t kDenoiseBlock = 64;
inline bool denoise_rows(uint32_t height, uint32_t nStrips, uint32_t strip, uint32_t& a, uint32_t& b) {
    const uint32_t nb = (height + kDenoiseBlock - 1) / kDenoiseBlock;
    if (nStrips < 1 || strip >= nStrips || nb < nStrips) return false;
    const uint32_t b0 = (uint32_t)((uint64_t)strip * nb / nStrips), b1 = (uint32_t)((uint64_t)(strip + 1) * nb / nStrips);
    a = b0 * kDenoiseBlock;
    b = b1 * kDenoiseBlock < height ? b1 * kDenoiseBlock : height;
    return true;
}

// G-buffer rows a strip-local denoise of [a, b) reads: its passes run on the strip's 16-row tiles
// widened by at most 4 tiles (TemporalFilter, denoise.hip tile_range) and read the G-buffers at
// most one row beyond those (3x3 taps; the wider stencils run on narrower tile ranges), so one
// more tile on each side covers every read.  Multi-GPU hosts move only these rows between ranks.
constexpr uint32_t kGbufHaloTiles = 5;
inline void gbuffer_rows(uint32_t height, uint32_t a, uint32_t b, uint32_t& lo, uint32_t& hi) {
    const uint32_t t0 = a / 16, t1 = (b + 15) / 16;
    lo = t0 > kGbufHaloTiles ? (t0 - kGbufHaloTiles) * 16 : 0;
    hi = (t1 + kGbufHaloTiles) * 16 < height ? (t1 + kGbufHaloTiles) * 16 : height;
}

struct TracePrimaryParams {
    TraceCamera cam;
    uint32_t width, height;
    uint32_t y0, rows;          // strip rows (row_of): contiguous [y0, y0 + rows) when nStrips = 1
    uint32_t nStrips, strip;
    int frameNum;
    const uint8_t* bluenoise;   // sobol | scrambling | ranking
    const float4* triPos;       // the arena's triangle records
    const float4* triNrm;
    const void* nodes;          // the record arena
    const void* tlasNodes;      // its TLAS nodes
    float4* hitOut;             // [W*H] (t, objectIdx bits, u, v)
    float4* normalOut;          // [W*H] optional (geometric normal, hit)
    float4* fakeNormalOut;      // [W*H] optional
    uint32_t* statsOut;         // [W*H][4] optional: visits, tests, dropped, iterations
};

extern "C" hipError_t rtk_launch_build_bvh(const BvhBuildParams* p, hipStream_t stream);
extern "C" hipError_t rtk_launch_trace_primary(const TracePrimaryParams* p, hipStream_t stream);
extern "C" hipError_t rtk_launch_smooth_normals(const float* vertices, const uint32_t* adjOffsets,
                                                const uint32_t* adjCorners, const uint32_t* indices,
                                                uint32_t nverts, float* normals, hipStream_t stream);
