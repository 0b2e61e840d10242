// lat_probe.hip — measurement probe (not product code): one lane traverses one ray with the
// product's trav_step_pf<16> and stamps two s_memtime counts per iteration through the
// RTX_TRAV_HOOK points: at the iteration's start (k = 0) and once its record has arrived (k = 1,
// after a forced wait on the record).  arrive - start is the load latency the previous
// iteration's bookkeeping did not cover; next start - arrive is the iteration's own work.
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
            if ((k) == 0) s_kind[(s).iters] = !(s).cLeaf ? 0u : ((s).cBlas ? 1u : 2u);        \
        }                                                                                     \
    } while (0)

#include "traverse.h"

using namespace rtd;

// laneStride is 0 at run time: the ray is read through a lane-dependent address so that the
// compiler treats it (and the whole traversal) as divergent, as in the product's kernels
__global__ void k_probe(const float4* triPos, const Node* nodes, const Node* tlas, const float* ray0, float4* hitOut,
                        uint32_t* itersOut, uint32_t* tOut, uint32_t* kindOut, int laneStride) {
    __shared__ uint2 stk[16 * 64];  // [entry][lane] as in the product
    // every lane traces the same ray (no single-lane region the compiler could specialise)
    const float* ray = ray0 + threadIdx.x * laneStride;
    const uint32_t c0 = (uint32_t)__builtin_readcyclecounter();
    const uint32_t c1 = (uint32_t)__builtin_readcyclecounter();
    SceneView sc;
    sc.triPos = triPos;
    sc.triNrm = nullptr;
    sc.nodes = nodes;
    sc.tlas = tlas;
    TravRay r;
    TravState s;
    trav_setup(sc, f3(ray[0], ray[1], ray[2]), f3(ray[3], ray[4], ray[5]), r);
    trav_init(s);
    TravRec rec = trav_first_rec(sc);
    const bool occlusion = ray[6] != 0.0f;
    while (true) {
        const bool done = trav_step_pf<16>(sc, r, s, rec, stk + threadIdx.x, 64, nullptr) || s.iters >= 1024u ||
                          (occlusion && s.hitIdx >= 0);
        if (done) break;
    }
    if (threadIdx.x != 0) return;
    *hitOut = make_float4(s.t, __uint_as_float((uint32_t)s.hitIdx), s.hitU, s.hitV);
    *itersOut = s.iters;
    itersOut[1] = c1 - c0;  // one reading's own cost
    const uint32_t n = s.iters < kMaxIt ? s.iters : kMaxIt;
    for (uint32_t i = 0; i < n; ++i) {
        tOut[2 * i] = s_t[2 * i];
        tOut[2 * i + 1] = s_t[2 * i + 1];
        kindOut[i] = s_kind[i];
    }
}

// ---- candidate traversal record format (probe only): one joint node array [BLAS nodes of every
// batch | TLAS nodes], whose fourth quad holds ready child words: bit 31 leaf, bit 30 BLAS,
// bits 0..29 the absolute record index (node in the joint array, triangle in triPos, or for a
// TLAS leaf its BLAS root's node).  Iterations, pushes, pops, drops and counters are TraverseBvh's.
constexpr uint32_t kLeafBit = 0x80000000u, kBlasBit = 0x40000000u, kIdxMask = 0x3FFFFFFFu;

struct TS2 {
    float t;
    int hitIdx;
    float hitU, hitV, hitErrT, u, v, errT;
    int top;
    uint32_t cur;
    uint32_t visits, tests, dropped, iters;
};

RT_DEV TravRec load2(const float4* nodes, const float4* tris, uint32_t w) {
    const bool tri = w >= (kLeafBit | kBlasBit);
    const uint32_t i = w & kIdxMask;
    const float4* base = tri ? tris + 3u * i : nodes + 4u * i;
    TravRec rec;
    rec.a = base[0];
    rec.b = base[1];
    rec.c = base[2];
    rec.d = *(const uint4*)(base + (tri ? 0 : 3));
    return rec;
}

RT_DEV bool step2(const float4* nodes, const float4* tris, const TravRay& r, TS2& s, TravRec& rec, uint2* stk,
                  int stride) {
    if (s.iters < kMaxIt) {
        s_t[2 * s.iters] = (uint32_t)__builtin_readcyclecounter();
        s_kind[s.iters] = !(s.cur & kLeafBit) ? 0u : ((s.cur & kBlasBit) ? 1u : 2u);
        float _x;
        asm volatile("v_mov_b32 %0, %1" : "=v"(_x) : "v"(rec.a.x));
        asm volatile("v_mov_b32 %0, %1" : "=v"(_x) : "v"(rec.d.x));
        s_t[2 * s.iters + 1] = (uint32_t)__builtin_readcyclecounter();
    }
    ++s.iters;
    const uint32_t cur = s.cur;
    uint32_t next = cur, pw = 0u, pt = 0u;
    bool pop = false, push = false, tl = false;
    if (!(cur & kLeafBit)) {
        Node nd;
        nd.q0 = rec.a; nd.q1 = rec.b; nd.q2 = rec.c; nd.q3 = rec.d;
        ++s.visits;
        float t1, t2;
        bool i1, i2;
        box_test2(r.h, nd, i1, i2, t1, t2);
        const bool both = i1 && i2;
        const bool goLeft = both ? (t1 < t2) : i1;
        push = both && s.top < 15;
        s.dropped += (both && !push) ? 1u : 0u;
        next = goLeft ? rec.d.x : rec.d.y;
        pw = goLeft ? rec.d.y : rec.d.x;
        pt = __float_as_uint(goLeft ? t2 : t1);
        pop = !i1 && !i2;
    } else if (cur & kBlasBit) {
        ++s.tests;
        float tt;
        if (watertight(r.tr, r.org, f3_of(rec.a), f3_of(rec.b), f3_of(rec.c), s.t, tt, s.u, s.v, s.errT) && tt < s.t) {
            s.t = tt;
            s.hitIdx = (int)(cur & kIdxMask);
            s.hitU = s.u; s.hitV = s.v; s.hitErrT = s.errT;
        }
        pop = true;
    } else {
        tl = true;
        next = (cur & kIdxMask) | kBlasBit;
    }
    if (pop) {
        int top = s.top;
        float et;
        do {
            if (top < 0) {
                s.top = top;
                return true;
            }
            const unsigned long long e = *(volatile LdsU64*)(&stk[top * stride]);
            next = (uint32_t)e;
            et = __uint_as_float((uint32_t)(e >> 32));
            --top;
        } while (et > s.t);
        s.top = top;
    }
    if (!tl) rec = load2(nodes, tris, next);
    if (push) {
        stk[(s.top + 1) * stride] = make_uint2(pw, pt);
        ++s.top;
    }
    s.cur = next;
    return false;
}

// step3: the same iteration as mostly straight-line code.  Every iteration runs the box test on
// whatever record it holds (a triangle's is ignored), reads the stack top speculatively, stores the
// would-be pushed entry unconditionally one slot above the top (17 slots per lane), loads the next
// record unconditionally (a TLAS leaf re-reads its BLAS root); branches remain for the triangle
// test and for pops past entries farther than the closest hit.
RT_DEV bool step3(const float4* nodes, const float4* tris, const TravRay& r, TS2& s, TravRec& rec, uint2* stk,
                  int stride) {
    if (s.iters < kMaxIt) {
        s_t[2 * s.iters] = (uint32_t)__builtin_readcyclecounter();
        s_kind[s.iters] = !(s.cur & kLeafBit) ? 0u : ((s.cur & kBlasBit) ? 1u : 2u);
        float _x;
        asm volatile("v_mov_b32 %0, %1" : "=v"(_x) : "v"(rec.a.x));
        asm volatile("v_mov_b32 %0, %1" : "=v"(_x) : "v"(rec.d.x));
        s_t[2 * s.iters + 1] = (uint32_t)__builtin_readcyclecounter();
    }
    ++s.iters;
    const uint32_t cur = s.cur;
    const bool isNode = !(cur & kLeafBit);
    const bool isTri = cur >= (kLeafBit | kBlasBit);
    const int tp = s.top;
    const unsigned long long e = *(volatile LdsU64*)(&stk[(tp < 0 ? 0 : tp) * stride]);
    Node nd;
    nd.q0 = rec.a; nd.q1 = rec.b; nd.q2 = rec.c; nd.q3 = rec.d;
    float t1, t2;
    bool i1, i2;
    box_test2(r.h, nd, i1, i2, t1, t2);
    const bool both = isNode && i1 && i2;
    const bool goLeft = both ? (t1 < t2) : i1;
    const bool push = both && tp < 15;
    s.dropped += (both && !push) ? 1u : 0u;
    s.visits += isNode ? 1u : 0u;
    stk[(tp + 1) * stride] = make_uint2(goLeft ? rec.d.y : rec.d.x, __float_as_uint(goLeft ? t2 : t1));
    uint32_t next = isNode ? (goLeft ? rec.d.x : rec.d.y) : ((cur & kIdxMask) | kBlasBit);
    if (isTri) {
        ++s.tests;
        float tt;
        if (watertight(r.tr, r.org, f3_of(rec.a), f3_of(rec.b), f3_of(rec.c), s.t, tt, s.u, s.v, s.errT) && tt < s.t) {
            s.t = tt;
            s.hitIdx = (int)(cur & kIdxMask);
            s.hitU = s.u; s.hitV = s.v; s.hitErrT = s.errT;
        }
    }
    const bool pop = isNode ? (!i1 && !i2) : isTri;
    bool done = pop && tp < 0;
    int top = pop ? tp - 1 : (push ? tp + 1 : tp);
    next = pop ? (uint32_t)e : next;
    float et = pop ? __uint_as_float((uint32_t)(e >> 32)) : -kFltMax;
    while (!done && et > s.t) {  // entries farther than the closest hit (rare)
        if (top < 0) {
            done = true;
            break;
        }
        const unsigned long long f = *(volatile LdsU64*)(&stk[top * stride]);
        next = (uint32_t)f;
        et = __uint_as_float((uint32_t)(f >> 32));
        --top;
    }
    next = done ? cur : next;  // a finished ray loads a valid record
    rec = load2(nodes, tris, next);
    s.top = top;
    s.cur = next;
    return done;
}

// step4: step3 on one joint array of 64-B records [BLAS nodes | TLAS nodes | triangles (v0 v1 v2 +
// a pad quad)], so a record's address is joint + 64 * index whatever its kind, and the choice of
// the near child as mask arithmetic (goLeft = i1 && (!i2 || t1 < t2)).
RT_DEV bool step4(const float4* joint, const TravRay& r, TS2& s, TravRec& rec, uint2* stk, int stride) {
    if (s.iters < kMaxIt) {
        s_t[2 * s.iters] = (uint32_t)__builtin_readcyclecounter();
        s_kind[s.iters] = !(s.cur & kLeafBit) ? 0u : ((s.cur & kBlasBit) ? 1u : 2u);
        float _x;
        asm volatile("v_mov_b32 %0, %1" : "=v"(_x) : "v"(rec.a.x));
        asm volatile("v_mov_b32 %0, %1" : "=v"(_x) : "v"(rec.d.x));
        s_t[2 * s.iters + 1] = (uint32_t)__builtin_readcyclecounter();
    }
    ++s.iters;
    const uint32_t cur = s.cur;
    const bool isNode = !(cur & kLeafBit);
    const bool isTri = cur >= (kLeafBit | kBlasBit);
    const int tp = s.top;
    const unsigned long long e = *(volatile LdsU64*)(&stk[(tp < 0 ? 0 : tp) * stride]);
    Node nd;
    nd.q0 = rec.a; nd.q1 = rec.b; nd.q2 = rec.c; nd.q3 = rec.d;
    float t1, t2;
    bool i1, i2;
    box_test2(r.h, nd, i1, i2, t1, t2);
    i1 = i1 && isNode;
    i2 = i2 && isNode;
    const bool both = i1 && i2;
    const bool goLeft = i1 && (!i2 || t1 < t2);
    const bool push = both && tp < 15;
    s.dropped += (both && !push) ? 1u : 0u;
    s.visits += isNode ? 1u : 0u;
    stk[(tp + 1) * stride] = make_uint2(goLeft ? rec.d.y : rec.d.x, __float_as_uint(goLeft ? t2 : t1));
    uint32_t next = isNode ? (goLeft ? rec.d.x : rec.d.y) : ((cur & kIdxMask) | kBlasBit);
    if (isTri) {
        ++s.tests;
        float tt;
        if (watertight(r.tr, r.org, f3_of(rec.a), f3_of(rec.b), f3_of(rec.c), s.t, tt, s.u, s.v, s.errT) && tt < s.t) {
            s.t = tt;
            s.hitIdx = (int)rec.d.x;  // the pad quad's x: the triangle's index in triPos
            s.hitU = s.u; s.hitV = s.v; s.hitErrT = s.errT;
        }
    }
    const bool pop = isTri || (isNode && !i1 && !i2);
    bool done = pop && tp < 0;
    int top = pop ? tp - 1 : (push ? tp + 1 : tp);
    next = pop ? (uint32_t)e : next;
    float et = pop ? __uint_as_float((uint32_t)(e >> 32)) : -kFltMax;
    while (!done && et > s.t) {
        if (top < 0) {
            done = true;
            break;
        }
        const unsigned long long f = *(volatile LdsU64*)(&stk[top * stride]);
        next = (uint32_t)f;
        et = __uint_as_float((uint32_t)(f >> 32));
        --top;
    }
    next = done ? cur : next;
    const float4* base = joint + 4u * (next & kIdxMask);
    rec.a = base[0];
    rec.b = base[1];
    rec.c = base[2];
    rec.d = *(const uint4*)(base + 3);
    s.top = top;
    s.cur = next;
    return done;
}

template <int kVer>
__global__ void k_probe2(const float4* triPos, const float4* joint, uint32_t rootWord, const float* ray0,
                         float4* hitOut, uint32_t* itersOut, uint32_t* tOut, uint32_t* kindOut, int laneStride) {
    __shared__ uint2 stk[17 * 64];
    const float* ray = ray0 + threadIdx.x * laneStride;
    const uint32_t c0 = (uint32_t)__builtin_readcyclecounter();
    const uint32_t c1 = (uint32_t)__builtin_readcyclecounter();
    SceneView sc;  // trav_setup reads the root record (tlas[0]) for the scene box
    sc.triPos = triPos;
    sc.triNrm = nullptr;
    sc.nodes = (const Node*)joint;
    sc.tlas = (const Node*)joint + (rootWord & kIdxMask);
    TravRay r;
    trav_setup(sc, f3(ray[0], ray[1], ray[2]), f3(ray[3], ray[4], ray[5]), r);
    TS2 s;
    s.t = kRayMax; s.hitIdx = -1;
    s.hitU = 0.0f; s.hitV = 0.0f; s.hitErrT = 1e-7f;
    s.u = 0.0f; s.v = 0.0f; s.errT = 1e-7f;
    s.top = -1; s.cur = rootWord;
    s.visits = 0; s.tests = 0; s.dropped = 0; s.iters = 0;
    TravRec rec = load2(joint, triPos, rootWord);  // the root is a node: the same record in either format
    const bool occlusion = ray[6] != 0.0f;
    while (true) {
        const bool done = (kVer == 4   ? step4(joint, r, s, rec, stk + threadIdx.x, 64)
                           : kVer == 3 ? step3(joint, triPos, r, s, rec, stk + threadIdx.x, 64)
                                       : step2(joint, triPos, r, s, rec, stk + threadIdx.x, 64)) || s.iters >= 1024u ||
                          (occlusion && s.hitIdx >= 0);
        if (done) break;
    }
    if (threadIdx.x != 0) return;
    *hitOut = make_float4(s.t, __uint_as_float((uint32_t)s.hitIdx), s.hitU, s.hitV);
    *itersOut = s.iters;
    itersOut[1] = c1 - c0;
    const uint32_t n = s.iters < kMaxIt ? s.iters : kMaxIt;
    for (uint32_t i = 0; i < n; ++i) {
        tOut[2 * i] = s_t[2 * i];
        tOut[2 * i + 1] = s_t[2 * i + 1];
        kindOut[i] = s_kind[i];
    }
}

extern "C" int lp_run2(const void* triPos, const void* joint, uint32_t rootWord, const float* dRay, void* dHit,
                       void* dIters, void* dT, void* dKind, int ver) {
    hipLaunchKernelGGL(ver == 4 ? k_probe2<4> : ver == 3 ? k_probe2<3> : k_probe2<2>, dim3(1), dim3(64), 0, 0, (const float4*)triPos, (const float4*)joint, rootWord, dRay,
                       (float4*)dHit, (uint32_t*)dIters, (uint32_t*)dT, (uint32_t*)dKind, 0);
    if (hipGetLastError() != hipSuccess) return -2;
    return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}

extern "C" int lp_run(const void* triPos, const void* nodes, const void* tlas, const float* dRay, void* dHit,
                      void* dIters, void* dT, void* dKind) {
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, (const float4*)triPos, (const Node*)nodes, (const Node*)tlas,
                       dRay, (float4*)dHit, (uint32_t*)dIters, (uint32_t*)dT, (uint32_t*)dKind, 0);
    if (hipGetLastError() != hipSuccess) return -2;
    return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}
