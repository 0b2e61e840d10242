// traverse.h — device-side two-level BVH traversal with the reference's semantics.
//
//   CreateRayBoxIntersectionHelper  geometry.cuh:519-583 (conservative Up/Dn rounding)
//   RayAABBIntersect (pair)         geometry.cuh:585-629
//   RayTriangleWatertight           geometry.cuh:375-472 (fp64 fallback on U/V/W == 0)
//   TraverseBvh                     traverse.h:107-253: 16-entry stack whose overflowing
//                                   pushes are dropped, 1024-iteration cap, nearer child
//                                   first (tie -> right), pop while entry.t > tHit
//   RaySceneIntersect tail          traverse.cuh:192-217 (normal flips, miss normal)
//
// GPU mapping: the per-ray box helper is re-expressed per world axis (near/far plane
// selection by direction sign) so the inner loop indexes nothing dynamically; the stack
// lives in LDS as [entry][thread] columns (conflict-free ds_read/write_b64); every record the
// traversal reads — BLAS node, TLAS node, triangle — is a 64-B slot of one record arena (below).
#pragma once
#include "rt_device.h"

namespace rtd {

// explicit LDS (address space 3) view: reads through it are ds_read_*, whatever the compiler can
// infer about the generic pointer it is made from (which must point into LDS)
typedef __attribute__((address_space(3))) const unsigned long long LdsU64;

typedef float F2v __attribute__((ext_vector_type(2)));

// The conservative ray-box helper per world axis a = x, y, z as (near, far) pairs: o_a = (origin
// of the near plane test, of the far plane test), s_a = (near reciprocal rounded down twice, far
// one rounded up twice), n_a = direction component < 0.  Scalar members, no arrays: the box test
// runs on packed pairs, and arrays of these ended up in scratch.
struct RayBox {
    F2v o0, o1, o2;
    F2v s0, s1, s2;
    int n0, n1, n2;
};

RT_DEV int max_dim(F3 d) {
    if (d.x > d.y) return d.z > d.x ? 2 : 0;
    return d.z > d.y ? 2 : 1;
}

RT_DEV float Up(float a) { return a * (1.0f + 1.1920928955078125e-07f); }
RT_DEV float Dn(float a) { return a * (1.0f - 1.1920928955078125e-07f); }
RT_DEV float up_(float a) { return a > 0.0f ? Up(a) : Dn(a); }
RT_DEV float dn_(float a) { return a > 0.0f ? Dn(a) : Up(a); }

// CreateRayBoxIntersectionHelper (geometry.cuh:519-582) names the axes kx, ky, kz (kz the
// dominant one, kx / ky swapped when dir[kz] < 0) and gives each of kx and ky the same formulas
// of its own coordinates and the shared max_z, kz its origin coordinate, and swaps an axis's
// near / far origins when dir is negative along it.  So per world axis a: the kz value when a is
// kz, else the kx / ky formula on a's coordinates — which of kx and ky it is changes nothing.
// Evaluated that way, the axis permutation costs one select per axis instead of select chains.
RT_DEV void raybox_axis(float o, float d, float lower, float upper, float max_z, bool isZ, float& on, float& of) {
    const float eps = 5.0f * 5.9604644775390625e-08f;
    const float n = up_(o + Up(eps * Up(lower + max_z)));
    const float f = dn_(o - Up(eps * Up(upper + max_z)));
    const bool neg = d < 0.0f;
    on = isZ ? o : (neg ? f : n);
    of = isZ ? o : (neg ? n : f);
}

RT_DEV RayBox make_raybox(F3 org, F3 dir, const Box& scene, F3 inv) {
    const int kz = max_dim(abs3(dir));
    const F3 lo = abs3(org - scene.mn), hi = abs3(org - scene.mx);
    const F3 lower = f3(Dn(lo.x), Dn(lo.y), Dn(lo.z));
    const F3 upper = f3(Up(hi.x), Up(hi.y), Up(hi.z));
    const float max_z = fmx(comp(lower, kz), comp(upper, kz));
    float on[3], of[3];
    raybox_axis(org.x, dir.x, lower.x, upper.x, max_z, kz == 0, on[0], of[0]);
    raybox_axis(org.y, dir.y, lower.y, upper.y, max_z, kz == 1, on[1], of[1]);
    raybox_axis(org.z, dir.z, lower.z, upper.z, max_z, kz == 2, on[2], of[2]);
    RayBox h;
    h.o0 = F2v{on[0], of[0]};
    h.o1 = F2v{on[1], of[1]};
    h.o2 = F2v{on[2], of[2]};
    h.s0 = F2v{Dn(Dn(inv.x)), Up(Up(inv.x))};
    h.s1 = F2v{Dn(Dn(inv.y)), Up(Up(inv.y))};
    h.s2 = F2v{Dn(Dn(inv.z)), Up(Up(inv.z))};
    h.n0 = dir.x < 0.0f;
    h.n1 = dir.y < 0.0f;
    h.n2 = dir.z < 0.0f;
    return h;
}

// Box test of both children of a node (CreateRayBoxIntersectionHelper / RayAABBIntersect,
// geometry.cuh:519-629).  Per child and axis the near and far plane distances form one packed
// pair: ((near coord, far coord) - o_a) * s_a is one v_pk_add_f32 + one v_pk_mul_f32 (gfx950
// packed FP32), each component rounded exactly as the scalar expression.  min/max order is
// irrelevant here (no NaN can arise, and the sign of a zero tNear is erased by max(tNear, 0)),
// so the hardware 3-operand min/max are used.
RT_DEV void box_pair(const RayBox& h, float mnx, float mny, float mnz, float mxx, float mxy, float mxz, bool& hit,
                     float& tNear) {
    const F2v tx = (F2v{h.n0 ? mxx : mnx, h.n0 ? mnx : mxx} - h.o0) * h.s0;
    const F2v ty = (F2v{h.n1 ? mxy : mny, h.n1 ? mny : mxy} - h.o1) * h.s1;
    const F2v tz = (F2v{h.n2 ? mxz : mnz, h.n2 ? mnz : mxz} - h.o2) * h.s2;
    const float tn = __builtin_fmaxf(__builtin_fmaxf(tx.x, ty.x), tz.x);
    const float tf = __builtin_fminf(__builtin_fminf(tx.y, ty.y), tz.y);
    hit = tn <= tf && tf > 0.0f;
    tNear = fmx(tn, 0.0f);
}

RT_DEV void box_test2(const RayBox& h, const Node& nd, bool& i1, bool& i2, float& t1, float& t2) {
    box_pair(h, nd.q0.x, nd.q0.y, nd.q0.z, nd.q0.w, nd.q1.x, nd.q1.y, i1, t1);
    box_pair(h, nd.q1.z, nd.q1.w, nd.q2.x, nd.q2.y, nd.q2.z, nd.q2.w, i2, t2);
}

struct TriRay {
    int kx, ky, kz;
    float Sx, Sy, Sz;
};

RT_DEV TriRay make_triray(F3 dir) {
    TriRay r;
    r.kz = max_dim(abs3(dir));
    r.kx = r.kz + 1; if (r.kx == 3) r.kx = 0;
    r.ky = r.kx + 1; if (r.ky == 3) r.ky = 0;
    if (comp(dir, r.kz) < 0.0f) { const int t = r.kx; r.kx = r.ky; r.ky = t; }
    r.Sx = comp(dir, r.kx) / comp(dir, r.kz);
    r.Sy = comp(dir, r.ky) / comp(dir, r.kz);
    r.Sz = 1.0f / comp(dir, r.kz);
    return r;
}

RT_DEV float xorf(float a, uint32_t b) { return __uint_as_float(__float_as_uint(a) ^ b); }

// RayTriangleWatertight (geometry.cuh:406-472); u, v, e are written whenever it returns true
RT_DEV bool watertight(const TriRay& r, F3 org, F3 v1, F3 v2, F3 v3, float tCur, float& t, float& u, float& v, float& e) {
    const F3 A = v1 - org, B = v2 - org, C = v3 - org;
    const float Akz = comp(A, r.kz), Bkz = comp(B, r.kz), Ckz = comp(C, r.kz);
    const float Ax = comp(A, r.kx) - r.Sx * Akz;
    const float Ay = comp(A, r.ky) - r.Sy * Akz;
    const float Bx = comp(B, r.kx) - r.Sx * Bkz;
    const float By = comp(B, r.ky) - r.Sy * Bkz;
    const float Cx = comp(C, r.kx) - r.Sx * Ckz;
    const float Cy = comp(C, r.ky) - r.Sy * Ckz;
    float U = Cx * By - Cy * Bx;
    float V = Ax * Cy - Ay * Cx;
    float W = Bx * Ay - By * Ax;
    if (U == 0.0f || V == 0.0f || W == 0.0f) {
        const double CxBy = (double)Cx * (double)By, CyBx = (double)Cy * (double)Bx;
        U = (float)(CxBy - CyBx);
        const double AxCy = (double)Ax * (double)Cy, AyCx = (double)Ay * (double)Cx;
        V = (float)(AxCy - AyCx);
        const double BxAy = (double)Bx * (double)Ay, ByAx = (double)By * (double)Ax;
        W = (float)(BxAy - ByAx);
    }
    if ((U < 0.0f || V < 0.0f || W < 0.0f) && (U > 0.0f || V > 0.0f || W > 0.0f)) return false;
    const float det = U + V + W;
    if (det == 0.0f) return false;
    const float Az = r.Sz * Akz, Bz = r.Sz * Bkz, Cz = r.Sz * Ckz;
    const float T = U * Az + V * Bz + W * Cz;
    const uint32_t ds = __float_as_uint(det) & 0x80000000u;
    if ((xorf(T, ds) < 0.0f) || (xorf(T, ds) > tCur * xorf(det, ds))) return false;
    const float rcp = 1.0f / det;
    u = U * rcp;
    v = V * rcp;
    t = T * rcp;
    e = err_gamma(16) * fabsf(t);
    return true;
}

// ---- the record arena
//
// One allocation of 64-B records per LBVH set, written by k_build_bvh:
//
//   [0, B*1024)              BLAS nodes, batch b's at b*1024 (the reference's per-batch arrays)
//   [B*1024, B*1024 + B)     TLAS nodes
//   [B*1024 + B, .. + NP)    triangle records: the three vertices (w = 0), a fourth quad unused
//
// A node's boxes sit where the reference's BVHNode keeps them (q0..q2); its fourth quad holds the
// two children as ready traversal words (q3.x, q3.y) and the reference's child references (q3.z:
// left | right << 16, leaf = bit 15 of each), from which rt_download rebuilds the reference layout.
// A traversal word is the arena index of the record the next iteration reads, with the
// reference's (isLeaf, isBlas) pair on top:
//
//   bit 31 leaf, bit 30 BLAS   00 TLAS node   01 BLAS node   10 TLAS leaf   11 BLAS leaf (triangle)
//
// A TLAS leaf's word indexes its batch's BLAS root (the iteration at a TLAS leaf only switches
// to that BLAS, traverse.h:140-145), a BLAS leaf's the triangle record.  So forming the next
// node, the pushed entry and the record address takes no index arithmetic: a stack entry is
// (word, t) and a record is arena + 64 * (word & kIdxMask), whatever its kind.
// (kLeafBit, kBlasBit, kIdxMask: rt_device.h)

struct SceneView {
    const float4* arena;    // 64-B records (4 float4 each)
    const float4* tris;     // the arena's triangle records (triangle i at tris + 4 * i)
    const float4* triNrm;   // [N][3]
    uint32_t root;          // arena index of the TLAS root (B*1024)
    uint32_t triBase;       // arena index of triangle 0 (B*1024 + B)
};

// nodes = the arena (its BLAS nodes), tlas = its TLAS nodes, tris = its triangle records
RT_DEV SceneView scene_view(const void* nodes, const void* tlas, const float4* tris, const float4* triNrm) {
    SceneView sc;
    sc.arena = (const float4*)nodes;
    sc.tris = tris;
    sc.triNrm = triNrm;
    sc.root = (uint32_t)(((const float4*)tlas - sc.arena) / 4);
    sc.triBase = (uint32_t)((tris - sc.arena) / 4);
    return sc;
}

struct HitInfo {
    float t;
    int objectIdx;
    float u, v;
    F3 normal, fakeNormal, pos;
    float offset;
    float ndr;   // normalDotRayDir after the flip (<= 0)
    bool into;   // isRayIntoSurface
    bool hit;
    uint32_t visits, tests, dropped, iters;
};

RT_DEV Node node_at(const SceneView& sc, uint32_t idx) {
    const float4* p = sc.arena + 4u * idx;
    Node n;
    n.q0 = p[0];
    n.q1 = p[1];
    n.q2 = p[2];
    n.q3 = *(const uint4*)(p + 3);
    return n;
}

RT_DEV Box node_merged(const Node& n) {
    Box b;
    b.mx = f3(fmx(n.q0.w, n.q2.y), fmx(n.q1.x, n.q2.z), fmx(n.q1.y, n.q2.w));
    b.mn = f3(fmn(n.q0.x, n.q1.z), fmn(n.q0.y, n.q1.w), fmn(n.q0.z, n.q2.x));
    return b;
}

RT_DEV F3 f3_of(float4 a) { return f3(a.x, a.y, a.z); }

// The traversal is split into setup / one loop iteration / hit finalisation so that the inline
// callers (camera and primary rays, intersect()) and the persistent queue tracer (trace_queue.hip)
// run the same per-iteration code: one call of trav_step == one iteration of TraverseBvh's loop
// (traverse.h:120-160), which keeps the 1024-iteration cap exact per ray.
struct TravRay {
    F3 org;
    RayBox h;
    TriRay tr;
};

// stack entry: uint2 {traversal word, bits of float t}; stk points at this thread's column: entry
// k lives at [k * stride], so a push is one ds_write_b64 and a pop one ds_read_b64.
struct TravState {
    float t;
    int hitIdx;
    float hitU, hitV, hitErrT;   // of the closest hit
    float u, v, errT;            // of the last successful triangle test (HitInfo.u/.v)
    int top;
    uint32_t cur;                // traversal word of the record this iteration processes
    uint32_t visits, tests, dropped, iters;
};

RT_DEV void trav_setup(const SceneView& sc, F3 org, F3 dir, TravRay& r) {
    const F3 inv = f3(safe_divide(1.0f, dir.x), safe_divide(1.0f, dir.y), safe_divide(1.0f, dir.z));
    const Box sceneBox = node_merged(node_at(sc, sc.root));
    r.org = org;
    r.h = make_raybox(org, dir, sceneBox, inv);
    r.tr = make_triray(dir);
}

// Scene cull.  TraverseBvh's first iteration visits the TLAS root and ends the ray when neither
// child box is hit (85 % of the default view's camera rays).  A plain float slab test against the
// root's merged box grown by a margin — 1 % of its largest extent plus 0.01 — settles that case
// without the conservative ray-box helper: the helper's rounding terms move a box face by
// ulp-level amounts (origin offsets of ~5 * 2^-24 times the distance to the scene box, reciprocals
// scaled by (1 +- 2^-23)^2), and the plain test's own rounding is of the same order, both many
// orders below the margin.  So when even the grown box is missed, both children (inside the
// merged box) are missed by the exact test, and the ray's result is that first iteration's:
// a miss after one iteration and one node visit.  Any NaN leaves the ray to the full traversal.
RT_DEV bool root_surely_missed(const SceneView& sc, F3 org, F3 dir) {
    const Box b = node_merged(node_at(sc, sc.root));
    const float m = 0.01f * fmx(fmx(b.mx.x - b.mn.x, b.mx.y - b.mn.y), b.mx.z - b.mn.z) + 0.01f;
    // the hardware reciprocal (1 ulp): its error is as far below the margin as the helper's
    // rounding; a zero component gives an infinity, and a 0 * inf NaN goes to the full traversal
    const F3 inv = f3(__builtin_amdgcn_rcpf(dir.x), __builtin_amdgcn_rcpf(dir.y), __builtin_amdgcn_rcpf(dir.z));
    const float ax = (b.mn.x - m - org.x) * inv.x, bx = (b.mx.x + m - org.x) * inv.x;
    const float ay = (b.mn.y - m - org.y) * inv.y, by = (b.mx.y + m - org.y) * inv.y;
    const float az = (b.mn.z - m - org.z) * inv.z, bz = (b.mx.z + m - org.z) * inv.z;
    const float tn = fmx(fmx(fmn(ax, bx), fmn(ay, by)), fmn(az, bz));
    const float tf = fmn(fmn(fmx(ax, bx), fmx(ay, by)), fmx(az, bz));
    const bool finite = tn == tn && tf == tf && ax == ax && bx == bx && ay == ay && by == by && az == az && bz == bz;
    return finite && !(tn <= tf && tf > 0.0f);
}

RT_DEV void trav_init(TravState& s, uint32_t root) {
    s.t = kRayMax;
    s.hitIdx = -1;
    s.hitU = 0.0f; s.hitV = 0.0f; s.hitErrT = 1e-7f;
    s.u = 0.0f; s.v = 0.0f; s.errT = 1e-7f;
    s.top = -1;
    s.cur = root;
    s.visits = 0; s.tests = 0; s.dropped = 0; s.iters = 0;
}

// the state TraverseBvh ends in for a ray root_surely_missed settles (one root visit, no hit)
RT_DEV void trav_root_miss(TravState& s, uint32_t root) {
    trav_init(s, root);
    s.iters = 1;
    s.visits = 1;
}

// The deepest entries of the 16-entry stack when the LDS holds fewer (trav_step<kLds < 16>):
// entries kLds .. 15 live in registers, written and read through select chains (no indexed private
// array, no scratch).  Only rays whose stack grows past kLds entries ever touch them.
struct DeepStack {
    uint2 e0, e1, e2, e3, e4, e5;
};
RT_DEV void deep_set(DeepStack& d, int k, uint2 v) {
    d.e0 = k == 0 ? v : d.e0;
    d.e1 = k == 1 ? v : d.e1;
    d.e2 = k == 2 ? v : d.e2;
    d.e3 = k == 3 ? v : d.e3;
    d.e4 = k == 4 ? v : d.e4;
    d.e5 = k == 5 ? v : d.e5;
}
RT_DEV unsigned long long deep_get(const DeepStack& d, int k) {
    const uint2 v = k == 0 ? d.e0 : k == 1 ? d.e1 : k == 2 ? d.e2 : k == 3 ? d.e3 : k == 4 ? d.e4 : d.e5;
    return ((unsigned long long)v.y << 32) | v.x;
}

// The record an iteration processes, loaded by the iteration before it (or by trav_first_rec):
// internal node (TLAS or BLAS) its 64-B record, BLAS leaf its triangle record, TLAS leaf the root
// record of that batch's BLAS (that iteration reads nothing; the next one reads this again).
struct TravRec {
    float4 a, b, c;
    uint4 d;
};

RT_DEV TravRec trav_load(const SceneView& sc, uint32_t word) {
    const float4* p = sc.arena + 4u * (word & kIdxMask);
    TravRec rec;
    rec.a = p[0];
    rec.b = p[1];
    rec.c = p[2];
    rec.d = *(const uint4*)(p + 3);
    return rec;
}

RT_DEV TravRec trav_first_rec(const SceneView& sc) { return trav_load(sc, sc.root); }

// measurement hook of tools/probe/lat_probe.hip (iteration start, record arrival); empty in the product
#ifndef RTX_TRAV_HOOK
#define RTX_TRAV_HOOK(k, s, rec)
#endif

// One TraverseBvh iteration (traverse.h:120-160); returns true when the stack ran empty
// (TestForFinish, traverse.h:88-105).  The caller stops at 1024 iterations as well.  On entry rec
// holds the record of s.cur; on return, that of the new s.cur.
//
// A lone ray's iteration is a dependent chain of instructions (tools/probe/lat_probe.hip: its
// record load is covered, the ~100 instructions are not), so the iteration runs as straight-line
// code wherever the reference's branches allow it:
//   - the box tests run on every iteration's record (a leaf's results are masked off);
//   - the stack top is read at the start whether or not the iteration pops;
//   - the would-be pushed entry is stored one slot above the top unconditionally (the stack
//     column has kLds + 1 slots; a slot above the top is dead), when kLds is 16;
//   - the next record is loaded unconditionally (a TLAS leaf's iteration re-reads its BLAS root);
//     issuing it before the triangle test instead (in place, the vertices copied out) measured
//     slower: 0.369 -> 0.405 us per lone-ray iteration, trace<3> 266 -> 270 us;
// branches remain for the triangle test and for pops past entries farther than the closest hit.
// The iterations — which node or triangle each one tests, pushes, drops (a push onto a full
// stack), pops, counters — are TraverseBvh's.
//
// kLds: stack entries kept in LDS (the others, up to the reference's 16, in `deep`); the camera
// and primary-ray kernels keep 10 there, so that six of their workgroups fit a CU's LDS.
// kCarry false: the iteration loads its own record at its start instead (rec is scratch, nothing
// is carried from one iteration to the next: 14 fewer registers live across the loop, for kernels
// whose occupancy the registers set — the camera rays, the fused chain).
// kStats false: the node-visit, triangle-test and dropped-push counters are not kept (launches
// without per-pixel statistics; the iteration count, which the 1024 cap reads, always is).
template <int kLds, bool kCarry = true, bool kStats = true>
RT_DEV bool trav_step(const SceneView& sc, const TravRay& r, TravState& s, TravRec& rec, uint2* stk, int stride,
                      DeepStack* deep) {
    static_assert(kLds >= 10 && kLds <= 16, "LDS stack depth: 10..16 entries (at most 6 in registers)");
    if (!kCarry) rec = trav_load(sc, s.cur);
    RTX_TRAV_HOOK(0, s, rec);
    RTX_TRAV_HOOK(1, s, rec);
    ++s.iters;
    const uint32_t cur = s.cur;
    const bool isNode = !(cur & kLeafBit);
    const bool isTri = cur >= (kLeafBit | kBlasBit);
    const int tp = s.top;
    // the stack top, read whether or not this iteration pops (kLds 16; with a register part the
    // pops read where they happen: fewer registers live through the box tests)
    const unsigned long long e = kLds == 16 ? *(volatile LdsU64*)(&stk[(tp < 0 ? 0 : tp) * stride]) : 0ull;
    Node nd;
    nd.q0 = rec.a; nd.q1 = rec.b; nd.q2 = rec.c; nd.q3 = rec.d;
    float t1, t2;
    bool i1, i2;
    box_test2(r.h, nd, i1, i2, t1, t2);
    i1 = i1 && isNode;
    i2 = i2 && isNode;
    // one child hit: go there; both: nearer first (tie -> right), push the other
    const bool both = i1 && i2;
    const bool goLeft = i1 && (!i2 || t1 < t2);
    const bool push = both && tp < 15;  // a push onto a full stack is dropped
    if (kStats) {
        s.dropped += (both && !push) ? 1u : 0u;
        s.visits += isNode ? 1u : 0u;
    }
    const uint2 pushed = make_uint2(goLeft ? rec.d.y : rec.d.x, __float_as_uint(goLeft ? t2 : t1));
    if (kLds == 16) {
        stk[(tp + 1) * stride] = pushed;
    } else if (push) {
        if (tp + 1 < kLds) stk[(tp + 1) * stride] = pushed;
        else deep_set(*deep, tp + 1 - kLds, pushed);
    }
    // the next node: the chosen child, or at a TLAS leaf (10 -> 01) its BLAS root; as mask
    // arithmetic on the leaf bit (a ternary on isNode became a branch)
    const uint32_t nodeNext = goLeft ? rec.d.x : rec.d.y;
    uint32_t next = nodeNext ^ ((nodeNext ^ cur ^ (kLeafBit | kBlasBit)) & (uint32_t)((int)cur >> 31));
    const bool pop = isTri || (isNode && !i1 && !i2);
    bool done = kLds == 16 && pop && tp < 0;
    // (a push needs both children hit at a node, so it never coincides with a pop)
    int top = (pop && kLds == 16) ? tp - 1 : (push ? tp + 1 : tp);
    next = (pop && kLds == 16) ? (uint32_t)e : next;
    // kLds 16: the popped entry is e, and the loop pops on past entries farther than the closest
    // hit; otherwise the loop makes every pop (a +inf start enters it)
    float et = pop ? (kLds == 16 ? __uint_as_float((uint32_t)(e >> 32)) : __builtin_inff()) : -kFltMax;
    if (isTri) {  // after the box tests' values are spent: fewer registers live through it
        if (kStats) ++s.tests;
        float tt;
        if (watertight(r.tr, r.org, f3_of(rec.a), f3_of(rec.b), f3_of(rec.c), s.t, tt, s.u, s.v, s.errT) && tt < s.t) {
            s.t = tt;
            s.hitIdx = (int)((cur & kIdxMask) - sc.triBase);
            s.hitU = s.u; s.hitV = s.v; s.hitErrT = s.errT;
        }
    }
    while (!done && et > s.t) {  // pop (past entries farther than the closest hit)
        if (top < 0) {
            done = true;
            break;
        }
        const unsigned long long f = (kLds == 16 || top < kLds) ? *(volatile LdsU64*)(&stk[top * stride])
                                                                : deep_get(*deep, top - kLds);
        next = (uint32_t)f;
        et = __uint_as_float((uint32_t)(f >> 32));
        --top;
    }
    next = done ? cur : next;  // a finished ray loads a record that exists
    if (kCarry) rec = trav_load(sc, next);
    s.top = top;
    s.cur = next;
    return done;
}

// Wave-level leaf batching for the lanes of one wave that each run their own traversal: a lane
// whose next step is a BLAS leaf (a triangle test, ~1 iteration in 20) waits until enough lanes
// are at leaves, so the triangle-test code runs for many lanes at once instead of in nearly
// every trip of the loop.  Each ray's own sequence of steps is unchanged (a waiting lane only
// pauses), hence its hits, counters and 1024-step cap.  Returns whether this lane steps now.
RT_DEV bool trav_lane_steps(bool active, const TravState& s) {
    const bool atLeaf = active && s.cur >= (kLeafBit | kBlasBit);
    const unsigned long long lm = __ballot(atLeaf), am = __ballot(active);
    const int nl = __popcll(lm), na = __popcll(am);
    const bool doLeaf = nl >= 16 || nl * 4 >= na;
    return active && (!atLeaf || doLeaf);
}

// hit finalisation (traverse.h:161-174, traverse.cuh:192-217), once for the closest hit
RT_DEV void finalize_hit(const SceneView& sc, F3 org, F3 dir, float t, int hitIdx, float hitU, float hitV,
                         float hitErrT, HitInfo& out) {
    F3 nrm = f3(0.0f), pos = f3(kRayMax), fake = f3(0.0f);
    float offset = 1e-7f;
    if (hitIdx >= 0) {
        const float4* tp = sc.tris + 4 * hitIdx;
        const F3 v1 = f3_of(tp[0]), v2 = f3_of(tp[1]), v3 = f3_of(tp[2]);
        nrm = normalize(cross(v2 - v1, v3 - v1));
        const float w = -dot(nrm, v1);
        const F3 p = org + dir * t;
        pos = p - (dot(nrm, p) + w) * nrm;
        const F3 ap = abs3(pos);
        const float errorP = fmx(fmx(ap.x, ap.y), ap.z) * err_gamma(6);
        offset = hitErrT + errorP;
        const F3 n1 = normalize(f3_of(sc.triNrm[3 * hitIdx]));
        const F3 n2 = normalize(f3_of(sc.triNrm[3 * hitIdx + 1]));
        const F3 n3 = normalize(f3_of(sc.triNrm[3 * hitIdx + 2]));
        fake = normalize(n3 * (1.0f - hitU - hitV) + n1 * hitU + n2 * hitV);
    }
    float ndr = dot(nrm, dir);
    const bool into = ndr < 0.0f;
    if (!into) { nrm = -nrm; ndr = -ndr; }
    if (dot(fake, nrm) < 0.0f) fake = -fake;
    const bool hit = t < kRayMax;
    if (!hit) { nrm = f3(0.0f, -1.0f, 0.0f); fake = f3(0.0f, -1.0f, 0.0f); }
    out.t = t;
    out.objectIdx = hitIdx;
    out.normal = nrm;
    out.fakeNormal = fake;
    out.pos = pos;
    out.offset = offset;
    out.ndr = ndr;
    out.into = into;
    out.hit = hit;
}

// One ray's closest hit (RaySceneIntersect): scene cull, then trav_step to the end.  stk: this
// thread's stack column (kLds + 1 slots when kLds is 16).
template <int kLds = 16, bool kStats = true>
RT_DEV void intersect(const SceneView& sc, F3 org, F3 dir, uint2* stk, int stride, HitInfo& out) {
    TravState s;
    if (root_surely_missed(sc, org, dir)) {
        trav_root_miss(s, sc.root);
    } else {
        TravRay r;
        trav_setup(sc, org, dir, r);
        trav_init(s, sc.root);
        DeepStack deep;
        TravRec rec = trav_first_rec(sc);
        for (int it = 0; it < 1024; ++it)
            if (trav_step<kLds, true, kStats>(sc, r, s, rec, stk, stride, &deep)) break;
    }
    finalize_hit(sc, org, dir, s.t, s.hitIdx, s.hitU, s.hitV, s.hitErrT, out);
    out.u = s.u;
    out.v = s.v;
    out.visits = s.visits; out.tests = s.tests; out.dropped = s.dropped; out.iters = s.iters;
}

}  // namespace rtd
