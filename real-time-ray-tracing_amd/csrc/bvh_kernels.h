// bvh_kernels.h — launch interface of the LBVH build and traversal kernels (host side).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct BvhBuildParams {
    const float* vertices;     // [nv][3]
    const float* normals;      // [nv][3]
    const uint32_t* indices;   // [triCountPadded][3]
    uint32_t triCount;
    uint32_t triCountPadded;
    uint32_t batchCount;
    float4* triPos;            // [triCountPadded][3] (xyz, 0)
    float4* triNrm;            // [triCountPadded][3] (xyz, 0)
    float* aabbs;              // [triCountPadded][6]
    float* batchSceneAabbs;    // [B][6]
    uint32_t* morton;          // [B*1024] sorted keys
    uint32_t* reorder;         // [B*1024]
    void* nodes;               // [triCountPadded] 64-B nodes
    float* tlasAabbs;          // [B][6]
    float* tlasSceneAabb;      // [6]
    uint32_t* tlasMorton;      // [1024]
    uint32_t* tlasReorder;     // [1024]
    void* tlasNodes;           // [B]
    uint32_t* counter;         // arrival counter, zero between launches
};

struct TraceCamera {
    float pos[3];
    float adjustedFront[3], adjustedLeft[3], adjustedUp[3];
    float apertureLeft[3], apertureUp[3];
    float invRes[2];
};

struct TracePrimaryParams {
    TraceCamera cam;
    uint32_t width, height;
    uint32_t y0, rows;          // rows [y0, y0 + rows) of the frame are traced
    int frameNum;
    const uint8_t* bluenoise;   // sobol | scrambling | ranking
    const float4* triPos;
    const float4* triNrm;
    const void* nodes;
    const void* tlasNodes;
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
