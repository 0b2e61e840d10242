// trace_primary.hip — primary-ray traversal (BASELINE config 2) and the frame-1 smooth
// normals, for gfx950.
//
// k_trace_primary: GenerateRay (raygen.cuh:7-38, blue-noise sample frameNum*4,
// pathtrace.cuh:116-129) + RaySceneIntersect geometry (traverse.cuh:64-222) per pixel.
// 256-thread workgroups cover 16x16 pixels; each wave64 owns an 8x8 tile so its rays are
// coherent.  Of the 16-entry traversal stack, 10 entries live in LDS (20 KB per workgroup) and
// the deepest 6 in registers (traverse.h trav_step<10>); each node's record is loaded by the
// iteration that chooses it.
//
// k_smooth_normals: GenerateSmoothNormals run twice into an un-cleared buffer
// (kernel.cu:228-257, 313-327), made deterministic: one thread per vertex gathers its
// corners in triangle order (CSR built once at init) instead of float atomics.
#include "bvh_kernels.h"
#include "pt_common.h"
#include "traverse.h"

using namespace rtd;

// kStats: the launch writes per-ray statistics (P.statsOut), so the traversal counts visits, tests
// and dropped pushes
template <bool kStats>
#ifndef RTX_PRIMARY_WPE  // ablation builds only (tools/abl_build.sh): force waves per SIMD
__global__ __launch_bounds__(256) void k_trace_primary(TracePrimaryParams P) {
#else
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RTX_PRIMARY_WPE, RTX_PRIMARY_WPE)))
void k_trace_primary(TracePrimaryParams P) {
#endif
    constexpr int kLds = 10;
    __shared__ uint2 stk[kLds * 256];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int x = blockIdx.x * 16 + (w & 1) * 8 + (lane & 7);
    const int yl = blockIdx.y * 16 + (w >> 1) * 8 + (lane >> 3);
    if (x >= (int)P.width || yl >= (int)P.rows) return;
    const int y = (int)row_of(P.y0, P.nStrips, P.strip, (uint32_t)yl);

    const int s = P.frameNum * 4 + 0;
    const F2 pix = {bluenoise(P.bluenoise, x, y, s, 0), bluenoise(P.bluenoise, x, y, s, 1)};
    const F2 ap = {bluenoise(P.bluenoise, x, y, s, 2), bluenoise(P.bluenoise, x, y, s, 3)};
    F3 org, dir, centerDir;
    F2 sampleUv;
    generate_ray(P.cam, x, y, pix, ap, org, dir, centerDir, sampleUv);

    const SceneView sc = scene_view(P.nodes, P.tlasNodes, P.triPos, P.triNrm);
    HitInfo hi;
    intersect<kLds, kStats>(sc, org, dir, stk + tid, 256, hi);

    const size_t p = (size_t)y * P.width + x;
    P.hitOut[p] = make_float4(hi.t, __int_as_float(hi.objectIdx), hi.u, hi.v);
    if (P.normalOut) P.normalOut[p] = make_float4(hi.normal.x, hi.normal.y, hi.normal.z, hi.hit ? 1.0f : 0.0f);
    if (P.fakeNormalOut) P.fakeNormalOut[p] = make_float4(hi.fakeNormal.x, hi.fakeNormal.y, hi.fakeNormal.z, hi.offset);
    if (kStats) {
        P.statsOut[4 * p + 0] = hi.visits;
        P.statsOut[4 * p + 1] = hi.tests;
        P.statsOut[4 * p + 2] = hi.dropped;
        P.statsOut[4 * p + 3] = hi.iters;
    }
}

extern "C" hipError_t rtk_launch_trace_primary(const TracePrimaryParams* p, hipStream_t stream) {
    dim3 grid((p->width + 15) / 16, (p->rows + 15) / 16);
    if (p->statsOut) hipLaunchKernelGGL(k_trace_primary<true>, grid, dim3(256), 0, stream, *p);
    else hipLaunchKernelGGL(k_trace_primary<false>, grid, dim3(256), 0, stream, *p);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_smooth_normals(const float* V, const uint32_t* adjOffsets,
                                                        const uint32_t* adjCorners, const uint32_t* indices,
                                                        uint32_t nverts, float* N) {
    const uint32_t vtx = blockIdx.x * 256 + threadIdx.x;
    if (vtx >= nverts) return;
    F3 acc = f3(0.0f);
    const uint32_t a0 = adjOffsets[vtx], a1 = adjOffsets[vtx + 1];
    for (int pass = 0; pass < 2; ++pass) {
        for (uint32_t a = a0; a < a1; ++a) {
            const uint32_t c = adjCorners[a];
            const uint32_t t = c / 3, k = c - 3 * t;
            const uint32_t i0 = indices[3 * t], i1 = indices[3 * t + 1], i2 = indices[3 * t + 2];
            const F3 v0 = f3(V[3 * i0], V[3 * i0 + 1], V[3 * i0 + 2]);
            const F3 v1 = f3(V[3 * i1], V[3 * i1 + 1], V[3 * i1 + 2]);
            const F3 v2 = f3(V[3 * i2], V[3 * i2 + 1], V[3 * i2 + 2]);
            const F3 pnma = cross(v2 - v0, v2 - v1) / 2.0f;
            F3 ea, eb;
            if (k == 0) { ea = v2 - v0; eb = v1 - v0; }
            else if (k == 1) { ea = v2 - v1; eb = v0 - v1; }
            else { ea = v0 - v2; eb = v1 - v2; }
            const float wgt = rt_acosf(dot(ea, eb) / __builtin_sqrtf(length2(ea) * length2(eb)));
            acc = acc + pnma * wgt;
        }
    }
    N[3 * vtx] = acc.x;
    N[3 * vtx + 1] = acc.y;
    N[3 * vtx + 2] = acc.z;
}

extern "C" hipError_t rtk_launch_smooth_normals(const float* vertices, const uint32_t* adjOffsets,
                                                const uint32_t* adjCorners, const uint32_t* indices,
                                                uint32_t nverts, float* normals, hipStream_t stream) {
    hipLaunchKernelGGL(k_smooth_normals, dim3((nverts + 255) / 256), dim3(256), 0, stream, vertices, adjOffsets,
                       adjCorners, indices, nverts, normals);
    return hipGetLastError();
}
