// lat_probe.hip — measurement probe (not product code): the lanes of one wave traverse one ray
// with the product's trav_step<16> on the product's record arena (RT_ARR_BVH_ARENA) and stamp two
// s_memtime counts per iteration through the RTX_TRAV_HOOK points: at the iteration's start
// (k = 0) and once its record has arrived (k = 1, after a forced wait on the record).
// arrive - start is the load latency the previous iteration did not cover; next start - arrive
// is the iteration's own work.
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr uint32_t kMaxIt = 1100;
__shared__ uint32_t s_t[2 * kMaxIt];   // s_memtime (low 32 bits) at the two hook points
__shared__ uint32_t s_kind[kMaxIt];    // 0 internal node, 1 BLAS leaf (triangle), 2 TLAS leaf

// s_memtime into LDS: no global store, no pointer reload between iterations (SHADER_CYCLES is not
// readable on gfx950)
#define RTX_TRAV_HOOK(k, s, rec)                                                              \
    do {                                                                                      \
        if ((s).iters < kMaxIt) {                                                             \
            if ((k) == 1) {                                                                   \
                float _x;                                                                     \
                asm volatile("v_mov_b32 %0, %1" : "=v"(_x) : "v"((rec).a.x));                 \
                asm volatile("v_mov_b32 %0, %1" : "=v"(_x) : "v"((rec).d.x));                 \
            }                                                                                 \
            const uint32_t _c = (uint32_t)__builtin_readcyclecounter();                       \
            s_t[2 * (s).iters + (k)] = _c;                                                    \
            if ((k) == 0) s_kind[(s).iters] = !((s).cur & kLeafBit) ? 0u : (((s).cur & kBlasBit) ? 1u : 2u); \
        }                                                                                     \
    } while (0)

#include "traverse.h"

using namespace rtd;

// laneStride is 0 at run time: every lane traces the same ray, read through a lane-dependent
// address so that the compiler treats the traversal as divergent, as in the product's kernels
__global__ void k_probe(const float4* arena, uint32_t root, uint32_t triBase, const float* ray0, float4* hitOut,
                        uint32_t* itersOut, uint32_t* tOut, uint32_t* kindOut, int laneStride) {
    __shared__ uint2 stk[17 * 64];  // [entry][lane] as in the product
    const float* ray = ray0 + threadIdx.x * laneStride;
    const uint32_t c0 = (uint32_t)__builtin_readcyclecounter();
    const uint32_t c1 = (uint32_t)__builtin_readcyclecounter();
    SceneView sc;
    sc.arena = arena;
    sc.tris = arena + 4u * triBase;
    sc.triNrm = nullptr;
    sc.root = root;
    sc.triBase = triBase;
    TravRay r;
    TravState s;
    trav_setup(sc, f3(ray[0], ray[1], ray[2]), f3(ray[3], ray[4], ray[5]), r);
    trav_init(s, sc.root);
    TravRec rec = trav_first_rec(sc);
    const bool occlusion = ray[6] != 0.0f;
    while (true) {
        const bool done = trav_step<16>(sc, r, s, rec, stk + threadIdx.x, 64, nullptr) || s.iters >= 1024u ||
                          (occlusion && s.hitIdx >= 0);
        if (done) break;
    }
    if (threadIdx.x != 0) return;
    *hitOut = make_float4(s.t, __uint_as_float((uint32_t)s.hitIdx), s.hitU, s.hitV);
    itersOut[0] = s.iters;
    itersOut[1] = c1 - c0;  // one reading's own cost
    const uint32_t n = s.iters < kMaxIt ? s.iters : kMaxIt;
    for (uint32_t i = 0; i < n; ++i) {
        tOut[2 * i] = s_t[2 * i];
        tOut[2 * i + 1] = s_t[2 * i + 1];
        kindOut[i] = s_kind[i];
    }
}

extern "C" int lp_run(const void* arena, uint32_t root, uint32_t triBase, const float* dRay, void* dHit, void* dIters,
                      void* dT, void* dKind) {
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, (const float4*)arena, root, triBase, dRay, (float4*)dHit,
                       (uint32_t*)dIters, (uint32_t*)dT, (uint32_t*)dKind, 0);
    if (hipGetLastError() != hipSuccess) return -2;
    return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}
