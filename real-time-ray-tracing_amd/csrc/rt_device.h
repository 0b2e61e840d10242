// rt_device.h — device-side value types and the reference's numeric conventions.
//
// Conventions kept bit-for-bit (every .hip file is built with -ffp-contract=off):
//   * min/max are the ternaries of linearMath.h:27-31 (operand order fixes NaN/±0 results)
//   * dot() is the compensated InnerProduct, cross() uses dop() (linearMath.h:41-98, 466, 484)
//   * float -> uint conversions saturate like CUDA's cvt.rzi.u32.f32
//   * transcendentals come from rtmath.h (bit-identical to the host oracle)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rtmath.h"

#define RT_DEV __device__ __forceinline__

namespace rtd {

constexpr float kFltMax = 3.402823466e+38f;
constexpr float kRayMax = 10e10f;                          // kernel.cuh:69
constexpr float kMachineEps = 1.1920928955078125e-07f;     // precision.cuh:18-23

struct F2 { float x, y; };
struct F3 { float x, y, z; };

RT_DEV F3 f3(float x, float y, float z) { F3 r; r.x = x; r.y = y; r.z = z; return r; }
RT_DEV F3 f3(float a) { return f3(a, a, a); }
RT_DEV F3 operator+(F3 a, F3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }
RT_DEV F3 operator-(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
RT_DEV F3 operator*(F3 a, F3 b) { return f3(a.x * b.x, a.y * b.y, a.z * b.z); }
RT_DEV F3 operator/(F3 a, F3 b) { return f3(a.x / b.x, a.y / b.y, a.z / b.z); }
RT_DEV F3 operator+(F3 a, float b) { return f3(a.x + b, a.y + b, a.z + b); }
RT_DEV F3 operator-(F3 a, float b) { return f3(a.x - b, a.y - b, a.z - b); }
RT_DEV F3 operator*(F3 a, float b) { return f3(a.x * b, a.y * b, a.z * b); }
RT_DEV F3 operator/(F3 a, float b) { return f3(a.x / b, a.y / b, a.z / b); }
RT_DEV F3 operator*(float b, F3 a) { return f3(a.x * b, a.y * b, a.z * b); }
RT_DEV F3 operator-(F3 a) { return f3(-a.x, -a.y, -a.z); }
RT_DEV float comp(F3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

RT_DEV float fmx(float a, float b) { return a > b ? a : b; }
RT_DEV float fmn(float a, float b) { return a < b ? a : b; }
RT_DEV float max1f(float a, float b) { return (a < b) ? b : a; }
RT_DEV float min1f(float a, float b) { return (a > b) ? b : a; }
RT_DEV F3 max3(F3 a, F3 b) { return f3(fmx(a.x, b.x), fmx(a.y, b.y), fmx(a.z, b.z)); }
RT_DEV F3 min3(F3 a, F3 b) { return f3(fmn(a.x, b.x), fmn(a.y, b.y), fmn(a.z, b.z)); }
RT_DEV F3 abs3(F3 a) { return f3(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }

RT_DEV float dop(float a, float b, float c, float d) {
    float cd = c * d;
    float err = __builtin_fmaf(-c, d, cd);
    float dp = __builtin_fmaf(a, b, -cd);
    return dp + err;
}
RT_DEV float inner3(float a, float b, float c, float d, float e, float f) {
    float ef = e * f, efe = __builtin_fmaf(e, f, -ef);
    float cd = c * d, cde = __builtin_fmaf(c, d, -cd);
    float s2 = cd + ef, dl2 = s2 - cd, s2e = (cd - (s2 - dl2)) + (ef - dl2);
    float tpv = s2, tpe = cde + (efe + s2e);
    float ab = a * b, abe = __builtin_fmaf(a, b, -ab);
    float s1 = ab + tpv, dl1 = s1 - ab, s1e = (ab - (s1 - dl1)) + (tpv - dl1);
    float rv = s1, re = abe + (tpe + s1e);
    return rv + re;
}
RT_DEV float dot(F3 a, F3 b) { return inner3(a.x, b.x, a.y, b.y, a.z, b.z); }
RT_DEV F3 cross(F3 a, F3 b) {
    return f3(dop(a.y, b.z, a.z, b.y), dop(a.z, b.x, a.x, b.z), dop(a.x, b.y, a.y, b.x));
}
RT_DEV float length2(F3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
RT_DEV F3 normalize(F3 v) {
    float n = __builtin_sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    return f3(v.x / n, v.y / n, v.z / n);
}
RT_DEV float safe_divide(float a, float b) {
    const float eps = 1e-20f;
    return a / ((fabsf(b) > eps) ? b : copysignf(eps, b));
}
RT_DEV uint32_t sat_u32(float x) {
    if (!(x > 0.0f)) return 0u;
    if (x >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)x;
}
RT_DEV float err_gamma(int n) { return (n * kMachineEps) / (1.0f - n * kMachineEps); }

// 64-byte BVH node: 4 x 16 B
//   q0 = lmin.x lmin.y lmin.z lmax.x
//   q1 = lmax.y lmax.z rmin.x rmin.y
//   q2 = rmin.z rmax.x rmax.y rmax.z
//   q3 = left word, right word, left | right << 16 (the reference's child references), 0
// (the reference's q3 is idxLeft idxRight isLeftLeaf isRightLeaf; rt_download restores it).  A
// word is a record-arena index with the child's kind on top (traverse.h, the record arena).
constexpr uint32_t kLeafBit = 0x80000000u, kBlasBit = 0x40000000u, kIdxMask = 0x3FFFFFFFu;
struct alignas(16) Node {
    float4 q0, q1, q2;
    uint4 q3;
};
struct Box { F3 mn, mx; };

RT_DEV Box box_empty() { Box b; b.mn = f3(kFltMax); b.mx = f3(-kFltMax); return b; }
RT_DEV Box box_merge(const Box& a, const Box& b) {  // AABBCompact::GetMerged order: max(a, b)
    Box r; r.mx = max3(a.mx, b.mx); r.mn = min3(a.mn, b.mn); return r;
}

// ---- Cross-workgroup hand-offs inside one launch: producers publish values, then count
// themselves on a launch counter; one consumer workgroup (the LBVH's TLAS workgroup, the downscale
// chain's last workgroup) reads them once the count is complete.
//
// The producer side carries no release fence on purpose: on gfx950 an agent-scope release is
// `buffer_wbl2 sc1`, a write-back of the producer XCD's whole L2, which doubled the LBVH gather
// phase and cost the downscale chain a write-back per workgroup.  Instead the
// values go out as agent-scope atomic stores — `global_store ... sc1`, written through to the
// memory side, coherent across the XCDs' L2s by themselves — and `s_waitcnt vmcnt(0)` holds the
// count back until they are complete: on gfx9 vmcnt counts stores too.  The consumer observes the
// count, then takes an agent-scope acquire (`buffer_inv sc1`: once, in one workgroup) and reads
// the values with agent-scope loads.  That ordering argument is specific to gfx950 (gfx10+ count
// stores in vscnt, not vmcnt), so these helpers refuse to compile for anything else.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "rt_device.h xwg_* hand-offs rely on gfx950's sc1 write-through stores and vmcnt store counting"
#endif
RT_DEV void xwg_store(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
RT_DEV void xwg_store(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
RT_DEV uint32_t xwg_load(const uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
RT_DEV unsigned long long xwg_load(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the producer's count, after its xwg_store values are complete; returns the count before it
RT_DEV uint32_t xwg_arrive(uint32_t* counter) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the consumer, once it has seen the complete count
RT_DEV void xwg_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); }

// Device-side failure report to the host: a word of pinned host memory (rt_context::status, one
// word per failure kind, bvh_kernels.h kStatus*, so a plain store suffices: no PCIe atomics), which
// sync_streams checks after its stream synchronisations.
RT_DEV void report_status(uint32_t* status, int word, uint32_t value) {
    if (status) __hip_atomic_store(status + word, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace rtd
