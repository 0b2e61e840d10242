// ORACLE (test infrastructure only; see ocommon.h) — two-level BVH traversal.
//
// Restates:
//   CreateRayBoxIntersectionHelper   geometry.cuh:519-583 (Woop/Ize conservative rounding)
//   RayAABBIntersect / pair test     geometry.cuh:585-629
//   RayTriangleWatertight            geometry.cuh:375-472 (fp64 fallback when U,V or W == 0)
//   GetRayPlaneIntersectPoint        geometry.cuh:252-262
//   BvhNodeStack / TestForFinish     traverse.h:9-105   (16 entries, dropped pushes)
//   TraverseBvh                      traverse.h:107-253 (1024-iteration cap)
//   RaySceneIntersect (geometry)     traverse.cuh:64-222
#include <atomic>
#include <thread>
#include <vector>

#include "oracle.h"
#include "ocommon.h"

namespace orc {

static inline float err_gamma(int n) { return (n * kMachineEps) / (1.0f - n * kMachineEps); }
static const float kP = 1.0f + 1.1920928955078125e-07f;  // 1 + 2^-23
static const float kM = 1.0f - 1.1920928955078125e-07f;
static inline float Up(float a) { return a * kP; }
static inline float Dn(float a) { return a * kM; }
static inline float up_(float a) { return a > 0.0f ? a * kP : a * kM; }
static inline float dn_(float a) { return a > 0.0f ? a * kM : a * kP; }

static inline int max_dim(F3 d) {
    if (d.x > d.y) return d.z > d.x ? 2 : 0;
    return d.z > d.y ? 2 : 1;
}

struct BoxHelper {
    int nearX, nearY, nearZ, farX, farY, farZ;
    float onx, ony, onz, ofx, ofy, ofz;
    float rnx, rny, rnz, rfx, rfy, rfz;
};

static BoxHelper make_helper(F3 org, F3 dir, const AABB& sceneBox, F3 inv) {
    int kz = max_dim(abs3(dir));
    int kx = kz + 1; if (kx == 3) kx = 0;
    int ky = kx + 1; if (ky == 3) ky = 0;
    if (dir[kz] < 0.0f) { int t = kx; kx = ky; ky = t; }
    BoxHelper h;
    h.nearX = kx; h.farX = 3 + kx;
    h.nearY = ky; h.farY = 3 + ky;
    h.nearZ = kz; h.farZ = 3 + kz;
    if (dir[kx] < 0.0f) { int t = h.nearX; h.nearX = h.farX; h.farX = t; }
    if (dir[ky] < 0.0f) { int t = h.nearY; h.nearY = h.farY; h.farY = t; }
    if (dir[kz] < 0.0f) { int t = h.nearZ; h.nearZ = h.farZ; h.farZ = t; }
    const float eps = 5.0f * 5.9604644775390625e-08f;  // 5 * 2^-24
    F3 lo = abs3(org - sceneBox.min), hi = abs3(org - sceneBox.max);
    F3 lower = f3(Dn(lo.x), Dn(lo.y), Dn(lo.z));
    F3 upper = f3(Up(hi.x), Up(hi.y), Up(hi.z));
    float max_z = fmx(lower[kz], upper[kz]);
    float err_near_x = Up(lower[kx] + max_z);
    float err_near_y = Up(lower[ky] + max_z);
    h.onx = up_(org[kx] + Up(eps * err_near_x));
    h.ony = up_(org[ky] + Up(eps * err_near_y));
    h.onz = org[kz];
    float err_far_x = Up(upper[kx] + max_z);
    float err_far_y = Up(upper[ky] + max_z);
    h.ofx = dn_(org[kx] - Up(eps * err_far_x));
    h.ofy = dn_(org[ky] - Up(eps * err_far_y));
    h.ofz = org[kz];
    if (dir[kx] < 0.0f) { float t = h.onx; h.onx = h.ofx; h.ofx = t; }
    if (dir[ky] < 0.0f) { float t = h.ony; h.ony = h.ofy; h.ofy = t; }
    h.rnx = Dn(Dn(inv[kx])); h.rny = Dn(Dn(inv[ky])); h.rnz = Dn(Dn(inv[kz]));
    h.rfx = Up(Up(inv[kx])); h.rfy = Up(Up(inv[ky])); h.rfz = Up(Up(inv[kz]));
    return h;
}

static inline bool box_test(const AABB& b, const BoxHelper& h, float& tNear, float& tFar) {
    float tnx = (aabb_at(b, h.nearX) - h.onx) * h.rnx;
    float tny = (aabb_at(b, h.nearY) - h.ony) * h.rny;
    float tnz = (aabb_at(b, h.nearZ) - h.onz) * h.rnz;
    float tfx = (aabb_at(b, h.farX) - h.ofx) * h.rfx;
    float tfy = (aabb_at(b, h.farY) - h.ofy) * h.rfy;
    float tfz = (aabb_at(b, h.farZ) - h.ofz) * h.rfz;
    tNear = fmx(fmx(tnx, tny), tnz);
    tFar = fmn(fmn(tfx, tfy), tfz);
    bool hit = tNear <= tFar && (tFar > 0);
    tNear = fmx(tNear, 0.0f);
    return hit;
}

static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float xorf(float a, uint32_t b) { uint32_t c = fbits(a) ^ b; float d; memcpy(&d, &c, 4); return d; }

static bool watertight(F3 org, F3 dir, const float* tri, float tCur, float& t, float& u, float& v, float& e) {
    int kz = max_dim(abs3(dir));
    int kx = kz + 1; if (kx == 3) kx = 0;
    int ky = kx + 1; if (ky == 3) ky = 0;
    if (dir[kz] < 0.0f) { int tt = kx; kx = ky; ky = tt; }
    float Sx = dir[kx] / dir[kz];
    float Sy = dir[ky] / dir[kz];
    float Sz = 1.0f / dir[kz];
    F3 A = f3(tri[0], tri[1], tri[2]) - org;
    F3 B = f3(tri[3], tri[4], tri[5]) - org;
    F3 C = f3(tri[6], tri[7], tri[8]) - org;
    const float Ax = A[kx] - Sx * A[kz];
    const float Ay = A[ky] - Sy * A[kz];
    const float Bx = B[kx] - Sx * B[kz];
    const float By = B[ky] - Sy * B[kz];
    const float Cx = C[kx] - Sx * C[kz];
    const float Cy = C[ky] - Sy * C[kz];
    float U = Cx * By - Cy * Bx;
    float V = Ax * Cy - Ay * Cx;
    float W = Bx * Ay - By * Ax;
    if (U == 0.0f || V == 0.0f || W == 0.0f) {
        double CxBy = (double)Cx * (double)By, CyBx = (double)Cy * (double)Bx;
        U = (float)(CxBy - CyBx);
        double AxCy = (double)Ax * (double)Cy, AyCx = (double)Ay * (double)Cx;
        V = (float)(AxCy - AyCx);
        double BxAy = (double)Bx * (double)Ay, ByAx = (double)By * (double)Ax;
        W = (float)(BxAy - ByAx);
    }
    if ((U < 0.0f || V < 0.0f || W < 0.0f) && (U > 0.0f || V > 0.0f || W > 0.0f)) return false;
    float det = U + V + W;
    if (det == 0.0f) return false;
    const float Az = Sz * A[kz];
    const float Bz = Sz * B[kz];
    const float Cz = Sz * C[kz];
    const float T = U * Az + V * Bz + W * Cz;
    uint32_t ds = fbits(det) & 0x80000000u;
    if ((xorf(T, ds) < 0.0f) || (xorf(T, ds) > tCur * xorf(det, ds))) return false;
    const float rcp = 1.0f / det;
    u = U * rcp;
    v = V * rcp;
    t = T * rcp;
    e = err_gamma(16) * fabsf(t);
    return true;
}

struct StackEntry { uint32_t idx, blasOffset, isBlas, isLeaf; float t; };

void intersect_one(const OrcScene* sc, F3 org, F3 dir, OrcHit& out) {
    const Node* nodes = (const Node*)sc->nodes;
    const Node* tlas = (const Node*)sc->tlasNodes;
    F3 inv = f3(safe_divide(1.0f, dir.x), safe_divide(1.0f, dir.y), safe_divide(1.0f, dir.z));
    float t = kRayMax;
    int objectIdx = -1;
    F3 nrm = f3(0.0f), pos = f3(kRayMax), fake = f3(0.0f);
    float u = 0.0f, v = 0.0f;
    float errorP = 1e-7f, errorT = 1e-7f, offset = 1e-7f;
    uint32_t visits = 0, tests = 0, dropped = 0, iters = 0, maxDepth = 0;

    AABB sceneBox = node_merged(tlas[0]);
    BoxHelper h = make_helper(org, dir, sceneBox, inv);
    StackEntry stack[16];
    int top = -1;
    StackEntry cur = {0, 0, 0, 0, -kFltMax};
    auto pop_until = [&](void) -> bool {  // TestForFinish: true when finished
        do {
            if (top < 0) return true;
            cur = stack[top--];
        } while (cur.t > t);
        return false;
    };
    auto push = [&](uint32_t idx, uint32_t off, uint32_t isBlas, uint32_t isLeaf, float tt) {
        if (top >= 15) { ++dropped; return; }
        StackEntry s = {idx & 0x7FFFu, off & 0x7FFFu, isBlas, isLeaf, tt};
        stack[++top] = s;
        if ((uint32_t)(top + 1) > maxDepth) maxDepth = (uint32_t)(top + 1);
    };
    for (int i = 0; i < 1024; ++i) {
        ++iters;
        if (cur.isLeaf) {
            if (cur.isBlas) {
                uint32_t li = cur.blasOffset * 1024u + cur.idx;
                const float* tri = sc->triangles + (size_t)li * 18;
                ++tests;
                float tt = kRayMax, ttmp;
                if (watertight(org, dir, tri, t, ttmp, u, v, errorT)) tt = ttmp;
                if (tt < t) {
                    t = tt;
                    objectIdx = (int)li;
                    F3 v1 = f3(tri[0], tri[1], tri[2]), v2 = f3(tri[3], tri[4], tri[5]), v3 = f3(tri[6], tri[7], tri[8]);
                    nrm = normalize(cross(v2 - v1, v3 - v1));
                    float w = -dot(nrm, v1);
                    F3 p = org + dir * t;
                    pos = p - (dot(nrm, p) + w) * nrm;
                    F3 ap = abs3(pos);
                    errorP = fmx(fmx(ap.x, ap.y), ap.z) * err_gamma(6);
                    offset = errorT + errorP;
                    F3 n1 = normalize(f3(tri[9], tri[10], tri[11]));
                    F3 n2 = normalize(f3(tri[12], tri[13], tri[14]));
                    F3 n3 = normalize(f3(tri[15], tri[16], tri[17]));
                    fake = normalize(n3 * (1.0f - u - v) + n1 * u + n2 * v);
                }
                if (pop_until()) break;
            } else {
                cur.isLeaf = 0;
                cur.isBlas = 1;
                cur.blasOffset = cur.idx;
                cur.idx = 0;
            }
        } else {
            const Node& nd = cur.isBlas ? nodes[cur.blasOffset * 1024u + cur.idx] : tlas[cur.idx];
            ++visits;
            float t1, t2, f1, f2;
            bool i1 = box_test(node_left(nd), h, t1, f1);
            bool i2 = box_test(node_right(nd), h, t2, f2);
            if (!i1 && !i2) {
                if (pop_until()) break;
            } else if (i1 && !i2) {
                cur.idx = nd.idxLeft; cur.isLeaf = nd.isLeftLeaf; cur.t = t1;
            } else if (!i1 && i2) {
                cur.idx = nd.idxRight; cur.isLeaf = nd.isRightLeaf; cur.t = t2;
            } else if (t1 < t2) {
                push(nd.idxRight, cur.blasOffset, cur.isBlas, nd.isRightLeaf, t2);
                cur.idx = nd.idxLeft; cur.isLeaf = nd.isLeftLeaf; cur.t = t1;
            } else {
                push(nd.idxLeft, cur.blasOffset, cur.isBlas, nd.isLeftLeaf, t1);
                cur.idx = nd.idxRight; cur.isLeaf = nd.isRightLeaf; cur.t = t2;
            }
        }
    }
    // RaySceneIntersect tail (traverse.cuh:192-217)
    float ndr = dot(nrm, dir);
    const bool into = ndr < 0;
    if (!into) { nrm = -nrm; ndr = -ndr; }
    if (dot(fake, nrm) < 0) fake = -fake;
    bool hit = t < kRayMax;
    if (!hit) { nrm = f3(0.0f, -1.0f, 0.0f); fake = f3(0.0f, -1.0f, 0.0f); }
    out.t = t;
    out.objectIdx = objectIdx;
    out.u = u; out.v = v;
    out.normal[0] = nrm.x; out.normal[1] = nrm.y; out.normal[2] = nrm.z;
    out.fakeNormal[0] = fake.x; out.fakeNormal[1] = fake.y; out.fakeNormal[2] = fake.z;
    out.pos[0] = pos.x; out.pos[1] = pos.y; out.pos[2] = pos.z;
    out.offset = offset;
    out.hit = hit ? 1u : 0u;
    out.intoSurface = into ? 1u : 0u;
    out.ndr = ndr;
    out.nodeVisits = visits; out.triTests = tests; out.droppedPushes = dropped; out.iterations = iters;
    out.maxDepth = maxDepth;
}

}  // namespace orc

using namespace orc;

extern "C" void orc_intersect(const OrcScene* scene, const float* rays, uint32_t n, OrcHit* hits, int threads) {
    if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
    if (threads < 1) threads = 1;
    auto work = [&](uint32_t lo, uint32_t hi) {
        for (uint32_t r = lo; r < hi; ++r) {
            const float* ry = rays + (size_t)r * 6;
            intersect_one(scene, f3(ry[0], ry[1], ry[2]), f3(ry[3], ry[4], ry[5]), hits[r]);
        }
    };
    if (threads == 1 || n < 1024) { work(0, n); return; }
    std::vector<std::thread> pool;
    const uint32_t chunk = 256;
    std::atomic_uint next(0);
    for (int k = 0; k < threads; ++k)
        pool.emplace_back([&]() {
            for (;;) {
                uint32_t lo = next.fetch_add(chunk);
                if (lo >= n) break;
                work(lo, lo + chunk < n ? lo + chunk : n);
            }
        });
    for (auto& th : pool) th.join();
}
