// pathtrace.hip — the per-pixel path tracer (PathTrace, pathtrace.cuh:11-128) for gfx950.
//
// One thread per pixel; a 256-thread workgroup covers 16x16 pixels and each wave64 an 8x8
// tile so primary rays stay coherent.  The three RaySceneIntersect calls per path share one
// 16-entry LDS stack column per thread (32 KB / workgroup).  With spp > 1 the thread loops
// over its samples (frame index spp*(frameNum-1)+1+s) and averages demodulated colour and
// albedo in fp32 before the half store; the other G-buffers come from sample 0.
// Traced-ray totals are reduced per workgroup and added with one 64-bit atomic.
#include "frame_kernels.h"
#include "pt_common.h"
#include "shade.h"
#include "traverse.h"

using namespace rtd;

namespace {

struct RayState {
    F3 orig, dir, pos, normal, fakeNormal, albedo, centerRaydir;
    int matId, matType, lightIdx, objectIdx;
    bool isRayIntoSurface, hitLight, hit, isDiffuseRay, isDiffuse, isHitProcessed, isOccluded, isShadowRay;
    float offset, normalDotRayDir, depth, rayConeWidth, rayConeSpread;
};

struct Ctx {
    const PathTraceParams& P;
    SceneView sc;
    uint32_t* stkA;
    float* stkT;
    F3 sunDir;
    uint32_t rays, visits, tests, diffuse;
};

RT_DEV void update_material(const Ctx& c, RayState& rs) {
    if (!rs.hit) {
        rs.matType = MAT_SKY;
        rs.matId = 99999;
    } else {
        if (c.P.materialOverride >= 0) rs.matId = c.P.materialOverride;
        else rs.matId = (rs.objectIdx >= 0 && rs.objectIdx < (int)c.P.triCount) ? 3 : 6;  // SAFE_LOAD(.., 6)
        rs.matType = (rs.matId >= 0 && rs.matId < 10) ? mat_type(rs.matId) : PERFECT_REFLECTION;
    }
    if (rs.isShadowRay) {
        if ((rs.matType == EMISSIVE && rs.lightIdx == rs.objectIdx) || (rs.matType == MAT_SKY && rs.lightIdx == kEnvLightId))
            rs.hitLight = true;
        else
            rs.isOccluded = true;
    } else {
        rs.hitLight = rs.matType == EMISSIVE || rs.matType == MAT_SKY;
    }
    rs.isDiffuse = (rs.matType == LAMBERTIAN) || (rs.matType == MICROFACET);
}

// RaySceneIntersect (traverse.cuh:64-225)
RT_DEV void scene_intersect(Ctx& c, RayState& rs) {
    if (rs.hitLight || !rs.isHitProcessed || rs.isOccluded) return;
    rs.isHitProcessed = false;
    ++c.rays;
    HitInfo h;
    intersect(c.sc, rs.orig, rs.dir, c.stkA, c.stkT, 256, h);
    c.visits += h.visits;
    c.tests += h.tests;
    rs.offset = h.offset;
    rs.objectIdx = h.objectIdx;
    rs.pos = h.pos;
    rs.normal = h.normal;
    rs.fakeNormal = h.fakeNormal;
    rs.normalDotRayDir = h.ndr;
    rs.isRayIntoSurface = h.into;
    rs.hit = h.hit;
    rs.depth = h.t;
    if (rs.hit) rs.rayConeWidth += rs.rayConeSpread * h.t;
    update_material(c, rs);
}

// GlossySurfaceInteraction (surfaceInteraction.cuh:11-34, bsdf.cuh:130-165)
RT_DEV void glossy(RayState& rs, float rnd) {
    if (rs.hitLight || rs.isDiffuse || rs.isOccluded) return;
    rs.isHitProcessed = true;
    if (rs.matType == PERFECT_REFLECTION) {
        rs.dir = normalize(rs.dir - rs.normal * dot(rs.dir, rs.normal) * 2.0f);
        rs.orig = rs.pos + rs.offset * rs.normal;
    } else if (rs.matType == FRESNEL_RR) {
        float etaI = 1.0f, etaT = 1.33f;
        if (!rs.isRayIntoSurface) { const float t = etaI; etaI = etaT; etaT = t; }
        const float eta = etaI / etaT;
        const float ndr = rs.normalDotRayDir;
        const float cosI = -ndr;
        const float sin2I = max1f(0.0f, (float)(1.0 - (double)(cosI * cosI)));
        const float sin2T = eta * eta * sin2I;
        const float cosT = __builtin_sqrtf(max1f(0.0f, (float)(1.0 - (double)sin2T)));
        F3 next;
        float off = rs.offset;
        if (sin2T >= 1.0f) {
            next = rs.dir - rs.normal * ndr * 2.0f;
        } else {
            const float R1 = etaT * cosI, R2 = etaI * cosT, R3 = etaI * cosI, R4 = etaT * cosT;
            const float Rparl = (R1 - R2) / (R1 + R2), Rperp = (R3 - R4) / (R3 + R4);
            const float fres = (Rparl * Rparl + Rperp * Rperp) / 2.0f;
            if (rnd < fres) {
                next = rs.dir - rs.normal * ndr * 2.0f;
            } else {
                next = eta * rs.dir + (eta * cosI - cosT) * rs.normal;
                off = -off;
            }
        }
        rs.dir = normalize(next);
        rs.orig = rs.pos + off * rs.normal;
    }
}

// one triplanar projection of DiffuseSurfaceInteraction's texture block
RT_DEV void tri_plane(const PathTraceParams& P, F2 uv, float lod, F3 normal, F3 w, F3& alb, F3& nrm) {
    uv.x *= 0.5f;
    uv.y *= 0.5f;
    const F4 t0 = sample_lod(P.texAlbedo, uv, lod);
    alb = f3(rt_powf(t0.x, 2.2f), rt_powf(t0.y, 2.2f), rt_powf(t0.z, 2.2f));
    const F4 t1 = sample_lod(P.texNormal, uv, lod);
    const F3 n = f3(t1.x - 0.5f, t1.y - 0.5f, t1.z - 0.5f);
    const F3 u = cross(normal, w);
    const F3 v = cross(normal, u);
    nrm = normalize(u * n.x + v * n.y + normal * n.z);
}

// DiffuseSurfaceInteraction (surfaceInteraction.cuh:36-310)
RT_DEV void diffuse(Ctx& c, int bounce, RayState& rs, F3& beta, const float r[4], const float r2[4]) {
    if (rs.hitLight || !rs.isDiffuse || rs.isOccluded) return;
    const PathTraceParams& P = c.P;
    ++c.diffuse;
    rs.isDiffuseRay = true;
    rs.lightIdx = kDefaultLightId;
    rs.isHitProcessed = true;
    F3 normal = rs.fakeNormal;
    const F3 surfaceNormal = rs.normal;
    F3 albedo;
    {
        const float lod = rt_log2f(rs.rayConeWidth * 0.5f * __builtin_sqrtf(1024.0f * 1024.0f + 1024.0f * 1024.0f));
        const float wx = surfaceNormal.x * surfaceNormal.x, wy = surfaceNormal.y * surfaceNormal.y,
                    wz = surfaceNormal.z * surfaceNormal.z;
        F3 accA = f3(0.0f), accN = f3(0.0f);
#pragma unroll 1
        for (int pl = 0; pl < 3; ++pl) {  // projections onto the x, y and z planes, summed in order
            const F2 uv = pl == 0 ? F2{rs.pos.y, rs.pos.z} : pl == 1 ? F2{rs.pos.x, rs.pos.z} : F2{rs.pos.x, rs.pos.y};
            F3 wv;
            if (pl == 0) wv = fabsf(normal.y) > 0.999f ? f3(0, 0, 1) : f3(0, 1, 0);
            else if (pl == 1) wv = fabsf(normal.x) > 0.999f ? f3(0, 0, 1) : f3(1, 0, 0);
            else wv = fabsf(normal.y) > 0.999f ? f3(1, 0, 0) : f3(0, 1, 0);
            F3 a, n;
            tri_plane(P, uv, lod, normal, wv, a, n);
            const float wgt = pl == 0 ? wx : pl == 1 ? wy : wz;
            accA = pl == 0 ? a * wgt : accA + a * wgt;
            accN = pl == 0 ? n * wgt : accN + n * wgt;
        }
        albedo = accA;
        normal = normalize(accN);
        rs.fakeNormal = normal;
    }
    if (bounce == 0) rs.albedo = albedo * (1.0f + fabsf(dot(normal, rs.centerRaydir)));
    const F3 rayDir = rs.dir;
    F3 lDir;
    float lPdf = 1.0f;
    int lIdx;
    sample_light(P, c.sunDir, lDir, lPdf, lIdx, r2[0], r2[1]);
    F3 sDir, sBsdf, lBsdf, tmp;
    float sPdf = 0.0f;
    if (rs.matType == LAMBERTIAN) {
        lambertian_sample(F2{r[0], r[1]}, sDir, normal);
        sBsdf = albedo / kPi;
        sPdf = fmx(dot(sDir, normal), kSafeCos) / kPi;
        lBsdf = albedo / kPi;
    } else {  // MICROFACET
        const F3 F0 = mat_F0(rs.matId);
        const float alpha = mat_alpha(rs.matId), alpha2 = alpha * alpha;
        const F3 sn = ggx_normal(F2{r[0], r[1]}, alpha2, normal);
        sDir = normalize(reflect3(rayDir, sn));
        if (dot(sDir, surfaceNormal) < 0.0f) {
            const F3 sn2 = ggx_normal(F2{r[2], r[3]}, alpha2, normal);
            sDir = normalize(reflect3(rayDir, sn2));
            if (dot(sDir, surfaceNormal) < 0.0f) sDir = normalize(reflect3(rayDir, normal));
        }
        float lsPdf;
        microfacet_terms(-rayDir, sDir, sn, normal, F0, albedo, alpha2, tmp, sBsdf, sPdf);
        microfacet_terms(-rayDir, lDir, normalize(lDir + -rayDir), normal, F0, albedo, alpha2, tmp, lBsdf, lsPdf);
    }
    if (isnan3(lBsdf)) lBsdf = f3(0.0f);
    if (isnan3(sBsdf)) sBsdf = f3(0.0f);
    if (sPdf != sPdf) sPdf = 0.0f;
    if (lPdf != lPdf) lPdf = 0.0f;
    const float ph = (sPdf * sPdf) / (sPdf * sPdf + lPdf * lPdf);
    const float minPdf = 1e-5f;
    if (r[3] < ph) {
        if (dot(rs.normal, sDir) < 0.0f) { rs.isOccluded = true; return; }
        const float cwi = fmx(kSafeCos, dot(sDir, normal));
        beta = sBsdf * cwi / fmx(sPdf, minPdf);
        rs.dir = sDir;
    } else {
        if (dot(rs.normal, lDir) < 0.0f) { rs.isOccluded = true; return; }
        const float cwi = fmx(kSafeCos, dot(lDir, normal));
        beta = lBsdf * cwi / fmx(lPdf, minPdf);
        rs.dir = lDir;
        rs.lightIdx = lIdx;
        rs.isShadowRay = true;
    }
    if (isnan3(beta)) beta = f3(0.0f);
    rs.orig = rs.pos + rs.offset * rs.normal;
}

// GetRayConeWidth (raygen.cuh:45-63)
RT_DEV float ray_cone_width(const PathTraceParams& P, int ix, int iy) {
    const F2 pc = {((float)ix + 0.5f) - P.res[0] / 2, ((float)iy + 0.5f) - P.res[1] / 2};
    const F2 po = {copysignf(0.5f, pc.x), copysignf(0.5f, pc.y)};
    const F2 un = {(pc.x - po.x) * P.cam.invRes[0] * 2, (pc.y - po.y) * P.cam.invRes[1] * 2};
    const F2 uf = {(pc.x + po.x) * P.cam.invRes[0] * 2, (pc.y + po.y) * P.cam.invRes[1] * 2};
    const F2 pn = {un.x * P.tanHalfFov[0], un.y * P.tanHalfFov[1]};
    const F2 pf = {uf.x * P.tanHalfFov[0], uf.y * P.tanHalfFov[1]};
    const float an = rt_atanf(__builtin_sqrtf(pn.x * pn.x + pn.y * pn.y));
    const float af = rt_atanf(__builtin_sqrtf(pf.x * pf.x + pf.y * pf.y));
    return af - an;
}

struct SampleOut {
    F3 L2, albedo, normal;
    float depth;
    F2 motion;
    uint32_t mask;
};

RT_DEV void path_sample(Ctx& c, int x, int y, int frameIdx, SampleOut& o) {
    const PathTraceParams& P = c.P;
    RayState rs;
    F3 beta0 = f3(1.0f), beta1 = f3(1.0f);
    rs.isDiffuseRay = false;
    rs.hitLight = false;
    rs.lightIdx = kDefaultLightId;
    rs.isHitProcessed = true;
    rs.isOccluded = false;
    rs.isShadowRay = false;
    rs.isDiffuse = false;
    rs.hit = false;
    rs.matType = MAT_SKY;
    rs.matId = 0;
    rs.objectIdx = -1;
    rs.normal = f3(0.0f, -1.0f, 0.0f);
    rs.fakeNormal = f3(0.0f);
    rs.albedo = f3(1.0f);
    rs.rayConeWidth = 0.0f;
    rs.rayConeSpread = ray_cone_width(P, x, y);
    float rn[4][4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int d = 0; d < 4; ++d) rn[k][d] = bluenoise(P.bluenoise, x, y, frameIdx * 4 + k, d);
    F2 sampleUv;
    generate_ray(P.cam, x, y, F2{rn[0][0], rn[0][1]}, F2{rn[0][2], rn[0][3]}, rs.orig, rs.dir, rs.centerRaydir,
                 sampleUv);
    // The reference's straight-line sequence (pathtrace.cuh:61-101)
    //   I G0 I G1 I G2 D0 [normal] I G3 D1 I
    // as one loop so traversal, glossy and diffuse each have a single call site.
    float outDepth = 0.0f;
    uint32_t mask = 0u;
    F2 mv = {0.0f, 0.0f};
    F3 outNormal = f3(0.0f);
#pragma unroll 1
    for (int k = 0; k < 5; ++k) {
        scene_intersect(c, rs);
        if (k == 0) {
            outDepth = rs.depth;
            mask = (uint32_t)rs.matId & 0xFFFFu;
            if (rs.hit) {  // HistoryCamera::WorldToScreenSpace (kernel.cuh:144-151)
                const F3 d = rs.pos - load3(P.hist.pos);
                const F3 v = f3(dot(load3(P.hist.left), d), dot(load3(P.hist.up), d), dot(load3(P.hist.dir), d));
                const F2 s = {v.x / v.z, v.y / v.z};
                const F2 ndc = {s.x / P.tanHalfFov[0], s.y / P.tanHalfFov[1]};
                mv = F2{(0.5f - ndc.x * 0.5f) - sampleUv.x, (0.5f - ndc.y * 0.5f) - sampleUv.y};
            }
            mv = F2{mv.x + 0.5f, mv.y + 0.5f};
        }
        if (k == 4) break;
        glossy(rs, k == 0 ? rn[0][0] : k == 1 ? rn[0][1] : k == 2 ? rn[0][2] : rn[0][3]);
        if (k >= 2) {
            const bool first = k == 2;
            const float r[4] = {first ? rn[0][0] : rn[2][0], first ? rn[0][1] : rn[2][1], first ? rn[0][2] : rn[2][2],
                                first ? rn[0][3] : rn[2][3]};
            const float r2[4] = {first ? rn[1][0] : rn[3][0], first ? rn[1][1] : rn[3][1], first ? rn[1][2] : rn[3][2],
                                 first ? rn[1][3] : rn[3][3]};
            F3 beta = f3(1.0f);
            diffuse(c, first ? 0 : 1, rs, beta, r, r2);
            if (first) {
                beta1 = beta;
                outNormal = rs.fakeNormal;
            } else {
                beta0 = beta;
            }
        }
    }
    F3 L0 = f3(0.0f);
    if (rs.hitLight && !rs.isOccluded && rs.matType == MAT_SKY) L0 = env_light(P, c.sunDir, rs.dir);
    F3 L2 = L0 * beta0 * beta1;
    if (isnan3(L2)) L2 = f3(0.0f);
    if (isnan3(outNormal)) outNormal = f3(0.0f);
    if (outDepth != outDepth) outDepth = 0.0f;
    if (mv.x != mv.x || mv.y != mv.y) mv = F2{0.0f, 0.0f};
    L2 = f3(clampf(L2.x, 0.0f, 10.0f), clampf(L2.y, 0.0f, 10.0f), clampf(L2.z, 0.0f, 10.0f));
    o.L2 = L2 / rs.albedo;
    o.albedo = rs.albedo;
    o.normal = outNormal;
    o.depth = outDepth;
    o.motion = mv;
    o.mask = mask;
}

RT_DEV uint2 pack_h4(float a, float b, float c, uint32_t d16) {
    return make_uint2((uint32_t)rt_f2h(a) | ((uint32_t)rt_f2h(b) << 16), (uint32_t)rt_f2h(c) | (d16 << 16));
}

}  // namespace

__global__ __launch_bounds__(256) void k_pathtrace(PathTraceParams P) {
    __shared__ uint32_t stkA[16 * 256];
    __shared__ float stkT[16 * 256];
    __shared__ unsigned long long wgRays[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int x = blockIdx.x * 16 + (w & 1) * 8 + (lane & 7);
    const int yl = blockIdx.y * 16 + (w >> 1) * 8 + (lane >> 3);
    const bool active = x < (int)P.width && yl < (int)P.rows;
    uint32_t rays = 0;
    if (active) {
        const int y = (int)P.y0 + yl;
        Ctx c{P, SceneView{}, stkA + tid, stkT + tid, f3(P.sunDir[0], P.sunDir[1], P.sunDir[2]), 0u, 0u, 0u, 0u};
        c.sc.triPos = P.triPos;
        c.sc.triNrm = P.triNrm;
        c.sc.nodes = (const Node*)P.nodes;
        c.sc.tlas = (const Node*)P.tlasNodes;
        SampleOut s0;
        F3 L = f3(0.0f), A = f3(0.0f);
#pragma unroll 1
        for (uint32_t s = 0; s < P.spp; ++s) {  // fp32 running sums in sample order, one divide
            SampleOut so;
            path_sample(c, x, y, (int)P.spp * (P.frameNum - 1) + 1 + (int)s, so);
            if (s == 0) s0 = so;
            L = L + so.L2;
            A = A + so.albedo;
        }
        if (P.spp == 1) {
            L = s0.L2;
            A = s0.albedo;
        } else {
            L = L / (float)P.spp;
            A = A / (float)P.spp;
        }
        const size_t p = (size_t)y * P.width + x;
        P.colorOut[p] = pack_h4(L.x, L.y, L.z, s0.mask);
        P.normalOut[p] = pack_h4(s0.normal.x, s0.normal.y, s0.normal.z, 0u);
        P.albedoOut[p] = pack_h4(A.x, A.y, A.z, 0u);
        P.depthOut[p] = rt_f2h(s0.depth);
        P.motionOut[p] = (uint32_t)rt_f2h(s0.motion.x) | ((uint32_t)rt_f2h(s0.motion.y) << 16);
        if (P.raysOut) P.raysOut[p] = c.rays;
        if (P.statsOut) P.statsOut[p] = make_uint4(c.rays, c.visits, c.tests, c.diffuse);
        rays = c.rays;
    }
    if (P.rayCounter) {
        unsigned long long r = rays;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o);
        if (lane == 0) wgRays[w] = r;
        __syncthreads();
        if (tid == 0) atomicAdd(P.rayCounter, wgRays[0] + wgRays[1] + wgRays[2] + wgRays[3]);
    }
}

extern "C" hipError_t rtk_launch_pathtrace(const PathTraceParams* p, hipStream_t stream) {
    if (p->spp < 1) return hipErrorInvalidValue;
    dim3 grid((p->width + 15) / 16, (p->rows + 15) / 16);
    hipLaunchKernelGGL(k_pathtrace, grid, dim3(256), 0, stream, *p);
    return hipGetLastError();
}
