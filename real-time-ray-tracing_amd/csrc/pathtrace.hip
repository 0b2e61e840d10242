// pathtrace.hip — the per-pixel path tracer (PathTrace, pathtrace.cuh:11-128) for gfx950,
// run as a wavefront pipeline:
//
//   k_pt_camera     one thread per (pixel, sample): blue noise, GenerateRay and the step-0
//                   RaySceneIntersect; a lean kernel (traversal state only) so the coherent
//                   camera rays trace at 4 waves/SIMD.  Writes the closest-hit record.
//   k_pt_shade0     one thread per pixel, looping over its samples: regenerates the camera
//                   ray, applies its hit and runs G0 I1 G1 I2 G2 D0 of the reference's
//                   straight-line sequence (I1/I2 trace inline only when the material table
//                   holds mirror or glass).  A sample whose next step is an intersection (I3:
//                   the BSDF bounce or the shadow ray) is appended to queue 3 with the state
//                   the rest of the path needs; every other sample is finished here.
//   k_trace_queue   (trace_queue.hip) traces a queue with persistent, refilling waves.
//   k_pt_resume<3>  applies the I3 hit, runs G3 D1 and appends the I4 rays to queue 4.
//   k_trace_queue   traces queue 4.
//   k_pt_resume<4>  applies the I4 hit and finishes those samples.
//   k_pt_resolve    averages the samples of the pixels that had a deferred sample.
//
// Every step runs the same code as the reference's sequence, in the same order per sample, so
// the G-buffers are bit-identical to the single-kernel evaluation (and to the CPU oracle).
// With spp > 1 sample s uses frame index spp*(frameNum-1)+1+s and the demodulated colour and
// albedo are averaged in fp32, in sample order, before the half store;
// the other G-buffers come from sample 0.
#include "frame_kernels.h"
#include "pt_common.h"
#include "queue_fetch.h"
#include "shade.h"
#include "traverse.h"

using namespace rtd;

namespace {

// queue-entry flags (PtQueue rayD.w)
constexpr uint32_t kQShadow = kQShadowFlag;  // isShadowRay
constexpr int kQSampleShift = 1;           // sample index s (6 bits, spp <= 64)
constexpr int kQLightShift = 16;           // lightIdx (16 bits: 7777 or 9999)

struct RayState {
    F3 orig, dir, pos, normal, fakeNormal, albedo, centerRaydir;
    int matId, matType, lightIdx, objectIdx;
    bool isRayIntoSurface, hitLight, hit, isDiffuse, isHitProcessed, isOccluded, isShadowRay;
    float offset, normalDotRayDir, depth, rayConeWidth, rayConeSpread;
};

struct PathCtx {
    const PathTraceParams& P;
    F3 sunDir;
    const uint32_t* sob;   // LDS copy of sobol dims 0..3
    BnPixel bp;
    int frameIdx;
    uint32_t rays, visits, tests, diffuse;
    const float* skyTree = nullptr;  // LDS copies of the light-CDF probe heaps (stage_cdf_trees)
    const float* sunTree = nullptr;
};

// copy the light-CDF probe heaps into LDS (all threads of the workgroup; caller syncs)
RT_DEV void stage_cdf_trees(const PathTraceParams& P, float* sky, float* sun, int tid, int nthreads) {
    for (int i = tid; i < kSkyTreeNodes / 4; i += nthreads) reinterpret_cast<float4*>(sky)[i] = reinterpret_cast<const float4*>(P.skyTree)[i];
    for (int i = tid; i < kSunTreeNodes / 4; i += nthreads) reinterpret_cast<float4*>(sun)[i] = reinterpret_cast<const float4*>(P.sunTree)[i];
}

// blue-noise sample (frameIdx * 4 + k, dim d) of this pixel (pathtrace.cuh:116-129)
RT_DEV float rnd(const PathCtx& c, int k, int d) { return bn_value(c.sob, c.bp, c.frameIdx * 4 + k, d); }

struct PathVars {
    RayState rs;
    F3 beta0, beta1;
    // sample-0 G-buffer values, set by steps 0 and 2 (always run in k_pt_shade0)
    float outDepth;
    uint32_t mask;
    F2 mv, sampleUv;
    F3 outNormal;
};

RT_DEV void update_material(const PathTraceParams& P, RayState& rs) {
    // values first, one store each: stores sunk behind a branch became a private array
    const int id = P.materialOverride >= 0 ? P.materialOverride
                   : (rs.objectIdx >= 0 && rs.objectIdx < (int)P.triCount) ? 3 : 6;  // SAFE_LOAD(.., 6)
    const int type = (id >= 0 && id < 10) ? mat_type(id) : PERFECT_REFLECTION;
    rs.matId = rs.hit ? id : 99999;
    rs.matType = rs.hit ? type : MAT_SKY;
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

// RaySceneIntersect (traverse.cuh:64-225): does this step trace?
RT_DEV bool needs_trace(const RayState& rs) { return !(rs.hitLight || !rs.isHitProcessed || rs.isOccluded); }

// ... and what it does with the hit
RT_DEV void apply_hit(const PathTraceParams& P, RayState& rs, const HitInfo& h) {
    rs.isHitProcessed = false;
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
    update_material(P, rs);
}

// GlossySurfaceInteraction (surfaceInteraction.cuh:11-34, bsdf.cuh:130-165); random number rn[0][k]
RT_DEV void glossy(const PathCtx& c, RayState& rs, int k) {
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
            if (rnd(c, 0, k) < fres) {
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
    // scheduling fences: the gamma chain and the normal-map fetches would otherwise interleave,
    // and the live texels of both maps set the register peak of the shading kernels
    __builtin_amdgcn_sched_barrier(0);
    alb = f3(rt_powf_div(t0.x, 2.2f), rt_powf_div(t0.y, 2.2f), rt_powf_div(t0.z, 2.2f));  // rtmath.h log2_pair_t
    __builtin_amdgcn_sched_barrier(0);
    const F4 t1 = sample_lod(P.texNormal, uv, lod);
    const F3 n = f3(t1.x - 0.5f, t1.y - 0.5f, t1.z - 0.5f);
    const F3 u = cross(normal, w);
    const F3 v = cross(normal, u);
    nrm = normalize(u * n.x + v * n.y + normal * n.z);
}

// DiffuseSurfaceInteraction (surfaceInteraction.cuh:36-310); random numbers rn[2*bounce] and
// rn[2*bounce+1].  kMF: the material table can hold the microfacet material (id 4, only through
// materialOverride); without it the GGX branch, whose live values set the kernels' register peak,
// is not compiled in.
template <bool kMF>
RT_DEV void diffuse(PathCtx& c, int bounce, RayState& rs, F3& beta) {
    if (rs.hitLight || !rs.isDiffuse || rs.isOccluded) return;
    const PathTraceParams& P = c.P;
    ++c.diffuse;
    rs.lightIdx = kDefaultLightId;
    rs.isHitProcessed = true;
    F3 normal = rs.fakeNormal;
    const F3 surfaceNormal = rs.normal;
    F3 albedo;
    {
        const float lod = rt_log2f_div(rs.rayConeWidth * 0.5f * __builtin_sqrtf(1024.0f * 1024.0f + 1024.0f * 1024.0f));
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
    float r[4], r2[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        r[d] = rnd(c, 2 * bounce, d);
        r2[d] = rnd(c, 2 * bounce + 1, d);
    }
    const F3 rayDir = rs.dir;
    F3 lDir;
    float lPdf = 1.0f;
    int lIdx;
    sample_light(P, c.sunDir, lDir, lPdf, lIdx, r2[0], r2[1], c.skyTree, c.sunTree);
    F3 sDir, sBsdf, lBsdf, tmp;
    float sPdf = 0.0f;
    if (!kMF || rs.matType == LAMBERTIAN) {
        lambertian_sample(F2{r[0], r[1]}, sDir, normal);
        sBsdf = f3(div_pi(albedo.x), div_pi(albedo.y), div_pi(albedo.z));  // albedo / kPi
        sPdf = div_pi(fmx(dot(sDir, normal), kSafeCos));
        lBsdf = sBsdf;  // albedo / kPi
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
    const F2 pc = {((float)ix + 0.5f) - P.halfRes[0], ((float)iy + 0.5f) - P.halfRes[1]};  // res / 2
    const F2 po = {copysignf(0.5f, pc.x), copysignf(0.5f, pc.y)};
    const F2 un = {(pc.x - po.x) * P.cam.invRes[0] * 2, (pc.y - po.y) * P.cam.invRes[1] * 2};
    const F2 uf = {(pc.x + po.x) * P.cam.invRes[0] * 2, (pc.y + po.y) * P.cam.invRes[1] * 2};
    const F2 pn = {un.x * P.tanHalfFov[0], un.y * P.tanHalfFov[1]};
    const F2 pf = {uf.x * P.tanHalfFov[0], uf.y * P.tanHalfFov[1]};
    const float an = rt_atanf(__builtin_sqrtf(pn.x * pn.x + pn.y * pn.y));
    const float af = rt_atanf(__builtin_sqrtf(pf.x * pf.x + pf.y * pf.y));
    return af - an;
}

// step 0's G-buffer values: depth, material mask and the motion vector
// (HistoryCamera::WorldToScreenSpace, kernel.cuh:144-151)
RT_DEV void gbuffer_step0(const PathCtx& c, PathVars& v) {
    const RayState& rs = v.rs;
    v.outDepth = rs.depth;
    v.mask = (uint32_t)rs.matId & 0xFFFFu;
    F2 mv = {0.0f, 0.0f};
    if (rs.hit) {
        const PathTraceParams& P = c.P;
        const F3 d = rs.pos - load3(P.hist.pos);
        const F3 q = f3(dot(load3(P.hist.left), d), dot(load3(P.hist.up), d), dot(load3(P.hist.dir), d));
        const F2 s = {q.x / q.z, q.y / q.z};
        const F2 ndc = {s.x / P.tanHalfFov[0], s.y / P.tanHalfFov[1]};
        mv = F2{(0.5f - ndc.x * 0.5f) - v.sampleUv.x, (0.5f - ndc.y * 0.5f) - v.sampleUv.y};
    }
    v.mv = F2{mv.x + 0.5f, mv.y + 0.5f};
}

// Steps k0..4 of the reference's straight-line sequence (pathtrace.cuh:61-101)
//   I G0 I G1 I G2 D0 [normal] I G3 D1 I
// as one loop so traversal, glossy and diffuse each have a single call site.  With `hit`
// set, step k0's intersection result is *hit (a deferred ray that came back from the queue
// tracer), applied before the loop so that the record is dead by the first interaction.  An
// intersection at a step >= kDeferFrom is not traced here: the step is returned and the caller
// queues the ray.  Returns 5 when the path is complete.
template <int kDeferFrom, bool kMF>
RT_DEV int run_path(PathCtx& c, PathVars& v, int k0, const HitInfo* hit, const SceneView& sc, uint2* stk) {
    RayState& rs = v.rs;
    if (hit) apply_hit(c.P, rs, *hit);
#pragma unroll 1
    for (int k = k0; k < 5; ++k) {
        if ((k != k0 || !hit) && needs_trace(rs)) {
            if (k >= kDeferFrom) return k;
            ++c.rays;
            HitInfo h;
            intersect(sc, rs.orig, rs.dir, stk, 256, h);
            c.visits += h.visits;
            c.tests += h.tests;
            apply_hit(c.P, rs, h);
        }
        if (k == 0) gbuffer_step0(c, v);
        if (k == 4) break;
        glossy(c, rs, k);
        if (k >= 2) {
            const bool first = k == 2;
            F3 beta = f3(1.0f);
            diffuse<kMF>(c, first ? 0 : 1, rs, beta);
            if (first) {
                v.beta1 = beta;
                v.outNormal = rs.fakeNormal;
            } else {
                v.beta0 = beta;
            }
        }
    }
    return 5;
}

// run_path<1, kMF>(c, v, 0, &hit, ..) for a material table without mirror or glass, in straight
// line.  glossy() then returns at once for every state (an emissive or sky hit sets hitLight or
// isOccluded, a lambertian or microfacet one isDiffuse), so step 1 never traces, step 2 is D0, and
// step 3 traces exactly when D0 produced a ray (D0 either returns before touching the state, which
// D1 then does too, or sets isOccluded, or sets a direction with isHitProcessed).  Without the
// step loop the camera hit record, the loop state and glossy's operands are not live across D0:
// k_pt_shade0 fits 3 waves per SIMD.
template <bool kMF>
RT_DEV int run_shade0_diffuse(PathCtx& c, PathVars& v, const HitInfo& hit) {
    RayState& rs = v.rs;
    apply_hit(c.P, rs, hit);
    gbuffer_step0(c, v);
    F3 beta = f3(1.0f);
    diffuse<kMF>(c, 0, rs, beta);
    v.beta1 = beta;
    v.outNormal = rs.fakeNormal;
    return needs_trace(rs) ? 3 : 5;
}

// end of PathTrace (pathtrace.cuh:103-128): the sample's demodulated colour
RT_DEV F3 finish(const PathCtx& c, const PathVars& v) {
    const RayState& rs = v.rs;
    F3 L0 = f3(0.0f);
    if (rs.hitLight && !rs.isOccluded && rs.matType == MAT_SKY) L0 = env_light(c.P, c.sunDir, rs.dir);
    F3 L2 = L0 * v.beta0 * v.beta1;
    if (isnan3(L2)) L2 = f3(0.0f);
    L2 = f3(clampf(L2.x, 0.0f, 10.0f), clampf(L2.y, 0.0f, 10.0f), clampf(L2.z, 0.0f, 10.0f));
    return L2 / rs.albedo;
}

RT_DEV uint2 pack_h4(float a, float b, float c, uint32_t d16) {
    return make_uint2((uint32_t)rt_f2h(a) | ((uint32_t)rt_f2h(b) << 16), (uint32_t)rt_f2h(c) | (d16 << 16));
}

// v / spp: the product with 1 / spp when spp is a power of two (P.invSpp, set by the host), which is
// the same real number and so the same correctly rounded result; the division otherwise
RT_DEV F3 div_spp(const PathTraceParams& P, F3 v) { return P.invSpp != 0.0f ? v * P.invSpp : v / (float)P.spp; }

// wave sum of a per-lane count into a counter: one atomic per wave (every lane of the wave calls)
RT_DEV void wave_add(uint32_t v, uint32_t* dst) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (__lane_id() == 0 && v) atomicAdd(dst, v);
}

// set bits of the wave mask m below this lane (v_mbcnt: no per-lane 64-bit mask kept live)
RT_DEV uint32_t lane_rank(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// wave-aggregated append: one atomic per wave, slots in lane order
RT_DEV uint32_t wave_append(bool want, uint32_t* counter) {
    const unsigned long long m = __ballot(want);
    if (m == 0ull) return 0u;
    const int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0u;
    if ((int)__lane_id() == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    return base + lane_rank(m);
}

RT_DEV void enqueue(const PtQueue& q, uint32_t slot, const PathVars& v, uint32_t pixel, uint32_t s) {
    const RayState& rs = v.rs;
    const uint32_t flags = (rs.isShadowRay ? kQShadow : 0u) | (s << kQSampleShift) |
                           ((uint32_t)rs.lightIdx << kQLightShift);
    q.rayO[slot] = make_float4(rs.orig.x, rs.orig.y, rs.orig.z, __uint_as_float(pixel));
    q.rayD[slot] = make_float4(rs.dir.x, rs.dir.y, rs.dir.z, __uint_as_float(flags));
    q.st0[slot] = make_float4(rs.albedo.x, rs.albedo.y, rs.albedo.z, rs.rayConeWidth);
    q.st1[slot] = make_float4(v.beta1.x, v.beta1.y, v.beta1.z, rs.rayConeSpread);
    q.st2[slot] = make_float4(v.beta0.x, v.beta0.y, v.beta0.z, 0.0f);
}

RT_DEV SceneView scene_of(const PathTraceParams& P) { return scene_view(P.nodes, P.tlasNodes, P.triPos, P.triNrm); }

// workgroup sum of traced rays into the frame counter (one atomic per workgroup)
// w: the calling wave's index in the workgroup (wave-uniform); the lane comes from v_mbcnt, so a
// caller need not keep threadIdx.x live until its end
// kBits: every lane's count is 0 or 1 (the camera kernel's one round), so the wave's sum is a
// popcount of a ballot; otherwise a 32-bit butterfly (a lane's count stays far below 2^26)
template <bool kBits = false>
RT_DEV void add_rays(const PathTraceParams& P, unsigned long long* wgSlots, uint32_t rays, int w) {
    if (!P.rayCounter) return;
    uint32_t r = rays;
    if (kBits) {
        r = (uint32_t)__popcll(__ballot(rays != 0u));
    } else {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o);
    }
    const bool lane0 = __lane_id() == 0;
    if (lane0) wgSlots[w] = r;
    __syncthreads();
    const uint32_t slot = (blockIdx.y * gridDim.x + blockIdx.x) % kRayCounterSlots;
    if (w == 0 && lane0)
        atomicAdd(&P.rayCounter[slot * kRayCounterStride], wgSlots[0] + wgSlots[1] + wgSlots[2] + wgSlots[3]);
}
template <bool kBits = false>
RT_DEV void add_rays(const PathTraceParams& P, unsigned long long* wgSlots, uint32_t rays) {
    add_rays<kBits>(P, wgSlots, rays, __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6));
}

// per-sample init of PathTrace (pathtrace.cuh:20-60) and GenerateRay (raygen.cuh:7-38)
RT_DEV void start_sample(PathCtx& c, PathVars& v, int x, int y, float coneSpread, F3 centerDir) {
    RayState& rs = v.rs;
    v.beta0 = f3(1.0f);
    v.beta1 = f3(1.0f);
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
    rs.rayConeSpread = coneSpread;
    rs.centerRaydir = centerDir;
    generate_ray_jittered(c.P.cam, x, y, F2{rnd(c, 0, 0), rnd(c, 0, 1)}, F2{rnd(c, 0, 2), rnd(c, 0, 3)}, rs.orig,
                          rs.dir, v.sampleUv);
    v.outDepth = 0.0f;
    v.mask = 0u;
    v.mv = F2{0.0f, 0.0f};
    v.outNormal = f3(0.0f);
}

}  // namespace

// Pixel block of one k_pt_camera workgroup: four waves = (4 / nSW) 8x8 tiles x nSW sample
// lanes, nSW = min(spp, 4) rounded down to 1, 2 or 4.
__host__ __device__ inline int cam_sample_waves(uint32_t spp) { return spp >= 4 ? 4 : (spp >= 2 ? 2 : 1); }
// one round of nSW sample waves covers every sample (spp 1, 2 and 4)
inline bool one_round(uint32_t spp) { return spp >= 1 && ((int)spp + cam_sample_waves(spp) - 1) / cam_sample_waves(spp) == 1; }

// Step 0 of every sample: the camera ray's RaySceneIntersect.  A sample that misses is complete
// right here (its path is GenerateRay -> miss -> EnvLight2, pathtrace.cuh:61-128, with every
// other step a no-op), so a pixel whose samples all miss — the sky, most of the default view —
// gets its G-buffer texels from this kernel and never reaches the shading kernels.  The other
// pixels keep their samples' hit records and are appended to the surface list for k_pt_shade0.
//
// kOneRound: every sample wave runs one round (spp <= 4 except 3: the launcher checks), so the
// round loop and its carried state compile away.
// kStats: the launch keeps per-pixel statistics (P.statsOut), so the traversal counts visits and tests
template <bool kOneRound, bool kStats>
__global__ __launch_bounds__(256, kOneRound ? 6 : 4) void k_pt_camera(PathTraceParams P) {
    // stack entries in LDS (the rest in registers): 26 KB per workgroup, 6 workgroups per CU
    // (measured: 16 entries 4 per CU 0.948 ms/frame, 12 entries 5 per CU 0.918, 10 entries 6 per CU
    // 0.900; the default scene's rays hold at most 11 entries)
    constexpr int kCamLds = 10;
    __shared__ uint2 stk[kCamLds * 256];
    __shared__ uint32_t sob[256];
    __shared__ float4 fold[4][64];   // this round's samples: sky colour xyz, w = 1 when it hit
    __shared__ uint32_t surf[4][64]; // pixel has a sample that hit (set by its folding thread)
    __shared__ unsigned long long wgRays[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    bn_stage_sobol(P.bluenoise, sob, tid, 256);
    __syncthreads();
    const int nSW = cam_sample_waves(P.spp);
    const int sw = w % nSW, g = w / nSW, tilesX = nSW == 4 ? 1 : 2;
    const int BW = 8 * tilesX, BH = nSW == 1 ? 16 : 8;
    const int x = blockIdx.x * BW + (g % tilesX) * 8 + (lane & 7);
    const int yl = blockIdx.y * BH + (g / tilesX) * 8 + (lane >> 3);
    const bool active = x < (int)P.width && yl < (int)P.rows;
    const int y = (int)row_of(P.y0, P.nStrips, P.strip, (uint32_t)yl);
    const uint32_t p = (uint32_t)y * P.width + (uint32_t)x;
    const uint32_t pl = (uint32_t)yl * P.width + (uint32_t)x;
    const size_t plane = (size_t)P.rows * P.width;
    const SceneView sc = scene_of(P);
    PathCtx c{P, f3(P.sunDir[0], P.sunDir[1], P.sunDir[2]), sob, BnPixel{0u, 0u}, 0, 0u, 0u, 0u, 0u};
    if (active) c.bp = bn_pixel(P.bluenoise, x, y);
    const int rounds = kOneRound ? 1 : ((int)P.spp + nSW - 1) / nSW;
    F3 L = f3(0.0f), A = f3(0.0f);  // folding thread (sw == 0): running sums of an all-sky pixel
    bool anyHit = false;
    float4 rec = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float recErr = 0.0f;
    uint32_t rays = 0, camV = 0, camT = 0, camCull = 0;
#pragma unroll 1
    for (int r = 0; r < rounds; ++r) {  // uniform trip count: every thread reaches the barriers
        const int s = r * nSW + sw;
        float4 out = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (active && s < (int)P.spp) {
            c.frameIdx = (int)P.spp * (P.frameNum - 1) + 1 + s;
            F3 org, dir;
            F2 uv;
            generate_ray_jittered(P.cam, x, y, F2{rnd(c, 0, 0), rnd(c, 0, 1)}, F2{rnd(c, 0, 2), rnd(c, 0, 3)}, org,
                                  dir, uv);
            TravState st;
            if (root_surely_missed(sc, org, dir)) {  // most sky rays: settled without the ray-box helper
                trav_root_miss(st, sc.root);
                ++camCull;
            } else {
                TravRay tr;
                trav_setup(sc, org, dir, tr);
                trav_init(st, sc.root);
                DeepStack deep;
                TravRec trec;  // each iteration loads its own record (kCarry false: occupancy)
                for (int it = 0; it < 1024; ++it)
                    if (trav_step<kCamLds, false, kStats>(sc, tr, st, trec, stk + tid, 256, &deep)) break;
            }
            ++rays;
            if (P.statsOut) {  // the pixel's counters are added after the round loop
                camV += st.visits;
                camT += st.tests;
            }
            rec = make_float4(st.t, __uint_as_float((uint32_t)st.hitIdx), st.hitU, st.hitV);
            recErr = st.hitErrT;
            if (rounds > 1) {  // several rounds: the pixel's status is not known yet
                P.ws.hit0Rec[(size_t)s * plane + pl] = rec;
                P.ws.hit0Err[(size_t)s * plane + pl] = recErr;
            }
            if (st.t < kRayMax) {
                out.w = 1.0f;
            } else {  // the whole path: finish() of a miss (beta 1, albedo 1)
                PathVars v;
                v.rs.dir = dir;
                v.rs.hitLight = true;
                v.rs.isOccluded = false;
                v.rs.matType = MAT_SKY;
                v.rs.albedo = f3(1.0f);
                v.beta0 = f3(1.0f);
                v.beta1 = f3(1.0f);
                const F3 Ls = finish(c, v);
                out = make_float4(Ls.x, Ls.y, Ls.z, 0.0f);
            }
        }
        fold[w][lane] = out;
        __syncthreads();
        if (sw == 0 && active) {
#pragma unroll 1
            for (int k = 0; k < nSW; ++k) {  // fold this round's samples in sample order
                const int sk = r * nSW + k;
                if (sk >= (int)P.spp) break;
                const float4 o = fold[g * nSW + k][lane];
                anyHit = anyHit || o.w != 0.0f;
                if (P.spp == 1) {
                    L = f3(o.x, o.y, o.z);
                    A = f3(1.0f);
                } else {
                    L = L + f3(o.x, o.y, o.z);
                    A = A + f3(1.0f);
                }
            }
        }
        __syncthreads();
    }
    if (sw == 0) surf[g][lane] = (active && anyHit) ? 1u : 0u;
    __syncthreads();
    const bool surface = active && surf[g][lane] != 0u;
    if (surface && rounds == 1 && sw < (int)P.spp) {
        P.ws.hit0Rec[(size_t)sw * plane + pl] = rec;
        P.ws.hit0Err[(size_t)sw * plane + pl] = recErr;
    }
    if (active && rays) {
        if (P.raysOut) atomicAdd(&P.raysOut[p], rays);
        if (P.statsOut) {
            atomicAdd(&P.statsOut[p].x, rays);
            if (camV) atomicAdd(&P.statsOut[p].y, camV);
            if (camT) atomicAdd(&P.statsOut[p].z, camT);
        }
    }
    if (P.statsOut) {
        wave_add(camV, &P.ws.counters[kCntVisCam]);
        wave_add(camT, &P.ws.counters[kCntTstCam]);
        wave_add(camCull, &P.ws.counters[kCntCulledCam]);
    }
    const uint32_t slot = wave_append(sw == 0 && surface, &P.ws.counters[kCntSurface]);
    if (sw == 0 && active) {
        if (surface) {
            P.ws.surface[slot] = pl;
        } else {  // G-buffer of an all-sky pixel: sample 0 missed (matId 99999, miss normal/depth)
            if (P.spp > 1) {
                L = div_spp(P, L);
                A = div_spp(P, A);
            }
            P.colorOut[p] = pack_h4(L.x, L.y, L.z, 99999u & 0xFFFFu);
            P.normalOut[p] = pack_h4(0.0f, -1.0f, 0.0f, 0u);
            P.albedoOut[p] = pack_h4(A.x, A.y, A.z, 0u);
            P.depthOut[p] = rt_f2h(kRayMax);
            P.motionOut[p] = (uint32_t)rt_f2h(0.5f) | ((uint32_t)rt_f2h(0.5f) << 16);
        }
    }
    add_rays<kOneRound>(P, wgRays, rays);
}

// Batches of k_pt_shade0.  Synchronous frames (PtWorkspace::shadeClaim) claim them dynamically:
// the batches are cut into kParts contiguous parts, one counter each (64 B apart, in the
// workspace's fetch block); a workgroup claims from its home part (blockIdx % kParts) and moves
// on to the next part once that is drained, thread 0 publishing the batch through LDS.  A batch's
// time is a chain of dependent loads that varies with its pixels, and the static split (batch b,
// then b + grid) left the last round to a fraction of the workgroups: serial shade 197 -> 184 us.
// Pipelined frames keep the static split over the larger grid: there the shade runs beside the
// previous frame's tracers, and workgroups that stay resident until the list is drained measured
// 0.79 -> 0.82 ms per frame.  Block-uniform calls, each ending with a barrier.
struct ShadeClaim {
    uint32_t batches, partLen, drained, next;
    int home;
    bool dyn;
};
RT_DEV void claim_init(ShadeClaim& c, uint32_t batches, bool dyn) {
    c.batches = batches;
    c.partLen = (batches + kParts - 1) / kParts;
    c.drained = batches == 0u ? (1u << kParts) - 1u : 0u;
    c.home = (int)(blockIdx.x % kParts);
    c.dyn = dyn;
    c.next = blockIdx.x;
}
// the next batch index, or >= batches when every part is drained
RT_DEV uint32_t claim_next(ShadeClaim& c, uint32_t* counters, uint32_t& slot) {
    if (!c.dyn) {
        const uint32_t b = c.next;
        c.next += gridDim.x;
        return b;
    }
    __syncthreads();  // the previous batch's readers of `slot` are done
    if (threadIdx.x == 0) {
        uint32_t b = c.batches;
        while (c.drained != (1u << kParts) - 1u) {
            int part = c.home;
            while (c.drained & (1u << part)) part = (part + 1) % kParts;
            const uint32_t got = atomicAdd(&counters[part * 16], 1u);
            const uint32_t lo = (uint32_t)part * c.partLen;
            const uint32_t len = lo >= c.batches ? 0u : (c.batches - lo < c.partLen ? c.batches - lo : c.partLen);
            if (got < len) {
                b = lo + got;
                break;
            }
            c.drained |= 1u << part;
        }
        slot = b;
    }
    __syncthreads();
    return slot;
}

// Steps 0 (hit from k_pt_camera) .. 3 of every sample of the surface pixels.  kGlossy: the
// material table holds mirror/glass, so steps 1 and 2 may trace (inline, LDS stack).
//
// Work layout as in k_pt_camera: a workgroup takes 64-pixel groups of the surface list, and
// each of its nSW sample waves shades one sample of those pixels per round, so a lane runs one
// sample's dependent chain (hit, textures, light-CDF searches, BSDF) rather than all spp of
// them back to back.  The folding thread (sample wave 0) then combines the round's samples in
// sample order through LDS — colour and albedo sums, the first deferred sample, the per-sample
// colours the resolve kernel needs — exactly as the sequential loop of PathTrace's caller does.
//
// kOneRound as in k_pt_camera: with one round per sample wave the fold state around the sample loop
// is not carried across rounds (one GPU 0.970 -> 0.945 ms/frame in round 3).  Without mirror or
// glass the sample runs run_shade0_diffuse, so the one-round kernel fits 168 VGPRs without
// scratch: 3 waves per SIMD instead of 2 (229 VGPRs through the step loop; serial 0.212 ->
// 0.190 ms, synchronous draw 1.089 -> 1.069 ms, profiles/r05_ab/shade0_straight/).
template <bool kGlossy, bool kMF, bool kOneRound>
#ifndef RTX_SHADE_WAVES  // A/B builds only (tools/abl_build.sh): waves per SIMD of the default-material variant
#define RTX_SHADE_WAVES 3
#endif
__global__ __launch_bounds__(256, (kGlossy || !kOneRound) ? 2 : RTX_SHADE_WAVES) void k_pt_shade0(PathTraceParams P) {
    __shared__ uint2 stk[kGlossy ? 17 * 256 : 1];  // 16 entries + trav_step's dead slot
    __shared__ uint32_t sob[256];
    __shared__ float4 foldL[4][64];  // this round's samples: finished colour xyz, w = 1 when deferred
    __shared__ float4 foldA[4][64];  // their albedo
    __shared__ unsigned long long wgRays[4];
    __shared__ __align__(16) float sSkyTree[kSkyTreeNodes];
    __shared__ __align__(16) float sSunTree[kSunTreeNodes];
    __shared__ uint32_t wgBatch;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wS = __builtin_amdgcn_readfirstlane(w);  // for add_rays: threadIdx.x need not live to the end
    bn_stage_sobol(P.bluenoise, sob, tid, 256);
    stage_cdf_trees(P, sSkyTree, sSunTree, tid, 256);
    __syncthreads();
    const uint32_t n = P.ws.counters[kCntSurface];
    const int nSW = cam_sample_waves(P.spp), sw = w % nSW, g = w / nSW;
    const uint32_t perWg = 64u * (uint32_t)(4 / nSW);
    const int rounds = kOneRound ? 1 : ((int)P.spp + nSW - 1) / nSW;
    const SceneView sc = scene_of(P);
    const size_t plane = (size_t)P.rows * P.width;
    uint32_t raysWg = 0, shV = 0, shT = 0, shD = 0;
    ShadeClaim claim;  // batches of perWg surface pixels (claim_next)
    claim_init(claim, (n + perWg - 1) / perWg, P.ws.shadeClaim != 0);
#pragma unroll 1
    for (uint32_t base; (base = claim_next(claim, P.ws.fetch + 2 * kParts * 16, wgBatch) * perWg) < n;) {
        const uint32_t i = base + (uint32_t)g * 64u + (uint32_t)lane;
        const bool active = i < n;
        const uint32_t pl = active ? P.ws.surface[i] : 0u;
        const int x = (int)(pl % P.width), yl = (int)(pl / P.width);
        const int y = (int)row_of(P.y0, P.nStrips, P.strip, (uint32_t)yl);
        const uint32_t p = (uint32_t)y * P.width + (uint32_t)x;
        PathCtx c{P, f3(P.sunDir[0], P.sunDir[1], P.sunDir[2]), sob, BnPixel{0u, 0u}, 0, 0u, 0u, 0u, 0u};
        c.skyTree = sSkyTree;
        c.sunTree = sSunTree;
        float coneSpread = 0.0f;
        F3 centerDir = f3(0.0f);
        if (active) {  // per-pixel invariants of the sample loop
            c.bp = bn_pixel(P.bluenoise, x, y);
            coneSpread = ray_cone_width(P, x, y);
            centerDir = center_dir(P.cam, x, y);
        }
        // folding thread (sw == 0) state; sample 0 runs on this same thread in round 0
        F3 L = f3(0.0f), A = f3(0.0f), L0s = f3(0.0f), A0s = f3(0.0f), N0 = f3(0.0f);
        float D0 = 0.0f;
        F2 M0 = {0.0f, 0.0f};
        uint32_t mask0 = 0u;
        int sd = -1;  // first deferred sample
#pragma unroll 1
        for (int r = 0; r < rounds; ++r) {  // uniform trip count: every thread reaches the barriers
            const int s = r * nSW + sw;
            const bool run = active && s < (int)P.spp;
            PathVars v;
            int kd = 5;
            if (run) {
                c.frameIdx = (int)P.spp * (P.frameNum - 1) + 1 + s;
                start_sample(c, v, x, y, coneSpread, centerDir);
                const size_t q = (size_t)s * plane + pl;
                const float4 hr = P.ws.hit0Rec[q];
                HitInfo h;
                finalize_hit(sc, v.rs.orig, v.rs.dir, hr.x, (int)__float_as_uint(hr.y), hr.z, hr.w, P.ws.hit0Err[q],
                             h);
                if constexpr (kGlossy) kd = run_path<3, kMF>(c, v, 0, &h, sc, stk + tid);
                else kd = run_shade0_diffuse<kMF>(c, v, h);
                if (kd < 3) {  // cannot happen without mirror/glass materials: flag it, finish the sample
                    atomicAdd(&P.ws.counters[kCntError], 1u);
                    kd = 5;
                }
            }
            const uint32_t slot3 = wave_append(kd == 3, &P.ws.counters[kCntQ3]);
            const uint32_t slot4 = wave_append(kd == 4, &P.ws.counters[kCntQ4]);
            float4 outL = make_float4(0.0f, 0.0f, 0.0f, 0.0f), outA = outL;
            if (run) {
                outA = make_float4(v.rs.albedo.x, v.rs.albedo.y, v.rs.albedo.z, 0.0f);
                if (s == 0) {
                    N0 = v.outNormal;
                    D0 = v.outDepth;
                    M0 = v.mv;
                    mask0 = v.mask;
                }
                if (kd < 5) {
                    ++c.rays;  // the deferred RaySceneIntersect
                    enqueue(kd == 3 ? P.ws.q3 : P.ws.q4, kd == 3 ? slot3 : slot4, v, p, (uint32_t)s);
                    outL.w = 1.0f;
                } else {
                    const F3 Ls = finish(c, v);
                    outL = make_float4(Ls.x, Ls.y, Ls.z, 0.0f);
                }
            }
            foldL[w][lane] = outL;
            foldA[w][lane] = outA;
            __syncthreads();
            if (sw == 0 && active) {
#pragma unroll 1
                for (int k = 0; k < nSW; ++k) {  // this round's samples in sample order
                    const int sk = r * nSW + k;
                    if (sk >= (int)P.spp) break;
                    const float4 o = foldL[g * nSW + k][lane];
                    const float4 a = foldA[g * nSW + k][lane];
                    A = A + f3(a.x, a.y, a.z);
                    if (sk == 0) A0s = f3(a.x, a.y, a.z);
                    if (o.w != 0.0f) {
                        if (sd < 0) {
                            sd = sk;
                            if (sk > 0) P.ws.pathL[(size_t)pl * P.spp + sk - 1] = make_float4(L.x, L.y, L.z, 0.0f);
                        }
                    } else {
                        const F3 Ls = f3(o.x, o.y, o.z);
                        if (sk == 0) L0s = Ls;
                        if (sd < 0) L = L + Ls;
                        else P.ws.pathL[(size_t)pl * P.spp + sk] = make_float4(Ls.x, Ls.y, Ls.z, 0.0f);
                    }
                }
            }
            __syncthreads();
        }
        const uint32_t pslot = wave_append(sw == 0 && active && sd >= 0, &P.ws.counters[kCntPending]);
        if (sw == 0 && active) {
            if (P.spp == 1) {
                L = L0s;
                A = A0s;
            } else {
                L = div_spp(P, L);
                A = div_spp(P, A);
            }
            if (N0.x != N0.x || N0.y != N0.y || N0.z != N0.z) N0 = f3(0.0f);
            if (D0 != D0) D0 = 0.0f;
            if (M0.x != M0.x || M0.y != M0.y) M0 = F2{0.0f, 0.0f};
            if (sd >= 0) {
                P.ws.pending[pslot] = pl | ((uint32_t)sd << 26);
                P.colorOut[p] = make_uint2(0u, mask0 << 16);  // colour resolved by k_pt_resolve
            } else {
                P.colorOut[p] = pack_h4(L.x, L.y, L.z, mask0);
            }
            P.normalOut[p] = pack_h4(N0.x, N0.y, N0.z, 0u);
            P.albedoOut[p] = pack_h4(A.x, A.y, A.z, 0u);
            P.depthOut[p] = rt_f2h(D0);
            P.motionOut[p] = (uint32_t)rt_f2h(M0.x) | ((uint32_t)rt_f2h(M0.y) << 16);
        }
        if (active && c.rays) {
            if (P.raysOut) atomicAdd(&P.raysOut[p], c.rays);
            if (P.statsOut) atomicAdd(&P.statsOut[p].x, c.rays);
        }
        if (active && P.statsOut) {
            if (c.visits) atomicAdd(&P.statsOut[p].y, c.visits);
            if (c.tests) atomicAdd(&P.statsOut[p].z, c.tests);
            if (c.diffuse) atomicAdd(&P.statsOut[p].w, c.diffuse);
            shV += c.visits;
            shT += c.tests;
            shD += c.diffuse;
        }
        raysWg += c.rays;
    }
    if (P.statsOut) {
        wave_add(shV, &P.ws.counters[kCntVisShade]);
        wave_add(shT, &P.ws.counters[kCntTstShade]);
        wave_add(shD, &P.ws.counters[kCntDiffShade]);
    }
    add_rays(P, wgRays, raysWg, wS);
}

// run_path<0, kMF>(c, v, kStep, &hit, ..) in straight line where no glossy interaction can run:
// step 4 (it ends the path) for any table, step 3 without mirror or glass (as run_shade0_diffuse:
// G3 returns at once, so step 3 is D1 and step 4 traces exactly when D1 produced a ray)
template <int kStep, bool kMF>
RT_DEV int resume_diffuse(PathCtx& c, PathVars& v, const HitInfo& hit) {
    apply_hit(c.P, v.rs, hit);
    if (kStep == 4) return 5;
    F3 beta = f3(1.0f);
    diffuse<kMF>(c, 1, v.rs, beta);
    v.beta0 = beta;
    return needs_trace(v.rs) ? 4 : 5;
}

// Entry i of queue kStep (3 or 4): reloads the sample's state, applies the hit the tracer found
// (t, triangle index bits, u, v; errorT) and runs the rest of its sequence.  Returns 4 when the
// I4 ray must be traced (kStep == 3 only), else 5 (the sample is complete).  kGlossy: the material
// table holds mirror or glass.
template <int kStep, bool kMF, bool kGlossy>
RT_DEV int resume_entry(PathCtx& c, const PtQueue& q, const SceneView& sc, uint32_t i, float4 hr, float herr,
                        PathVars& v, uint32_t& p, uint32_t& s) {
    const PathTraceParams& P = c.P;
    const float4 o = q.rayO[i], d = q.rayD[i], s0 = q.st0[i], s1 = q.st1[i], s2 = q.st2[i];
    p = __float_as_uint(o.w);
    const uint32_t flags = __float_as_uint(d.w);
    s = (flags >> kQSampleShift) & 63u;
    const int x = (int)(p % P.width), y = (int)(p / P.width);
    c.bp = bn_pixel(P.bluenoise, x, y);
    c.frameIdx = (int)P.spp * (P.frameNum - 1) + 1 + (int)s;
    RayState& rs = v.rs;
    rs.orig = f3(o.x, o.y, o.z);
    rs.dir = f3(d.x, d.y, d.z);
    rs.isShadowRay = (flags & kQShadow) != 0u;
    rs.lightIdx = (int)(flags >> kQLightShift);
    rs.albedo = f3(s0.x, s0.y, s0.z);
    rs.rayConeWidth = s0.w;
    v.beta1 = f3(s1.x, s1.y, s1.z);
    rs.rayConeSpread = s1.w;
    v.beta0 = f3(s2.x, s2.y, s2.z);
    rs.hitLight = false;  // a traced ray had neither flag set
    rs.isOccluded = false;
    rs.isHitProcessed = true;
    rs.isDiffuse = false;
    rs.centerRaydir = f3(0.0f);  // read by D0 only
    rs.matId = 0;
    rs.matType = MAT_SKY;
    HitInfo h;
    finalize_hit(sc, rs.orig, rs.dir, hr.x, (int)__float_as_uint(hr.y), hr.z, hr.w, herr, h);
    if constexpr (kGlossy && kStep == 3) return run_path<0, kMF>(c, v, kStep, &h, sc, nullptr);
    else return resume_diffuse<kStep, kMF>(c, v, h);
}

// a completed sample of a queue entry: its radiance goes to the late-resolve slot
RT_DEV void store_path_L(const PathCtx& c, const PathVars& v, uint32_t p, uint32_t s) {
    const PathTraceParams& P = c.P;
    const F3 Ls = finish(c, v);
    const uint32_t pl = local_row(P.y0, P.nStrips, p / P.width) * P.width + p % P.width;
    P.ws.pathL[(size_t)pl * P.spp + s] = make_float4(Ls.x, Ls.y, Ls.z, 0.0f);
}

// Resumes the samples of queue kStep (3 or 4) once k_trace_queue has written their hits.
template <int kStep, bool kMF, bool kGlossy>
__global__ __launch_bounds__(256, kStep == 3 ? (kGlossy ? 2 : 3) : 4) void k_pt_resume(PathTraceParams P) {
    __shared__ uint32_t sob[256];
    __shared__ unsigned long long wgRays[4];
    // step 4 ends the path before any diffuse interaction: no light sampling there
    __shared__ __align__(16) float sSkyTree[kStep == 3 ? kSkyTreeNodes : 4];
    __shared__ __align__(16) float sSunTree[kStep == 3 ? kSunTreeNodes : 4];
    const uint32_t n = P.ws.counters[kStep == 3 ? kCntQ3 : kCntQ4];
    // a workgroup past the queue (queue 4 holds a few thousand entries against a grid sized for
    // queue 3) leaves before staging its tables; block-uniform, no ray counted
    if (blockIdx.x * 256u >= n) return;
    const int tid = threadIdx.x;
    bn_stage_sobol(P.bluenoise, sob, tid, 256);
    if (kStep == 3) stage_cdf_trees(P, sSkyTree, sSunTree, tid, 256);
    __syncthreads();
    const PtQueue& q = kStep == 3 ? P.ws.q3 : P.ws.q4;
    const SceneView sc = scene_of(P);
    uint32_t rays = 0, rsD = 0;
#pragma unroll 1
    for (uint32_t base = blockIdx.x * 256u; base < n; base += gridDim.x * 256u) {  // block-uniform
        const uint32_t i = base + (uint32_t)tid;
        const bool active = i < n;
        PathCtx c{P, f3(P.sunDir[0], P.sunDir[1], P.sunDir[2]), sob, BnPixel{0u, 0u}, 0, 0u, 0u, 0u, 0u};
        c.skyTree = sSkyTree;
        c.sunTree = sSunTree;
        PathVars v;
        int kd = 5;
        uint32_t p = 0, s = 0;
        if (active) kd = resume_entry<kStep, kMF, kGlossy>(c, q, sc, i, P.ws.hitRec[i], P.ws.hitErr[i], v, p, s);
        const uint32_t slot = wave_append(kd == 4, &P.ws.counters[kCntQ4]);
        if (active) {
            if (kd < 5) {  // kStep == 3 only: the I4 ray
                ++c.rays;
                enqueue(P.ws.q4, slot, v, p, s);
            } else {
                store_path_L(c, v, p, s);
            }
            if (P.raysOut && c.rays) atomicAdd(&P.raysOut[p], c.rays);
            if (P.statsOut) {
                if (c.rays) atomicAdd(&P.statsOut[p].x, c.rays);
                if (c.diffuse) atomicAdd(&P.statsOut[p].w, c.diffuse);
                rsD += c.diffuse;
            }
            rays += c.rays;
        }
    }
    if (kStep == 3 && P.statsOut) wave_add(rsD, &P.ws.counters[kCntDiffRes3]);
    add_rays(P, wgRays, rays);
}

constexpr int kChainRanges = 32;  // queue-3 reserves a wave records before it resumes them
#ifndef RTX_CHAIN_STATIC
#define RTX_CHAIN_STATIC 0
#endif
constexpr bool kChainStaticFirst = RTX_CHAIN_STATIC != 0;  // ablation: static first batch per wave

// The bounce chain of the default materials in one launch: trace<3> -> resume<3> -> trace<4> ->
// resume<4>.  As separate kernels every stage ends on its slowest wave, so a frame
// paid the longest queue-3 traversal plus the longest queue-4 traversal one after the other.
// Here each wave resumes the queue-3 entries it traced itself, then traces and finishes the I4
// rays those produced, while other waves are still in their queue-3 tails; the launch ends on
// the wave whose chain is longest, not on the sum of two tails.
//
//   phase 1  k_trace_queue<3>'s refilling traversal loop (same Fetch), plus a per-wave list of
//            the reserves [lo, hi) the wave took; every entry of a reserve is traced by its lanes.
//   phase 2  (every lane idle) the wave resumes its reserves 64 entries at a time — resume<3> —
//            appends the I4 rays to queue 4 and to a per-wave slot list, and once 64 slots could
//            overflow, or at the end, traces them one per lane and finishes them (resume<4>).
//   repeat   when the reserve list was full before the queue drained.
// Per sample the code is the one the separate kernels run (resume_entry, trav_step), so the
// G-buffers are identical.  The hit records a wave reads in phase 2 are ones its own lanes wrote
// (a workgroup-scope fence orders them), so no record crosses workgroups inside the launch.
template <bool kStats>
RT_DEV bool chain_step(const SceneView& sc, const TravRay& r, TravState& s, TravRec& rec, uint2* stk) {
    return trav_step<16, false, kStats>(sc, r, s, rec, stk, 256, nullptr);  // no carried record: 168 VGPRs, no scratch
}

#ifndef RTX_CHAIN_WAVES
#define RTX_CHAIN_WAVES 3
#endif
template <bool kStats>  // as k_pt_camera's
__global__ __launch_bounds__(256, RTX_CHAIN_WAVES) void k_pt_chain(PathTraceParams P) {
    __shared__ uint2 stk[17 * 256];  // 16 entries + trav_step's dead slot
    __shared__ uint32_t sob[256];
    __shared__ uint2 ranges[4][kChainRanges];
    __shared__ uint32_t q4list[4][64];
    __shared__ unsigned long long wgRays[4];
    // w: the wave's index, wave-uniform (an SGPR); lane ranks come from v_mbcnt (lane_rank)
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    bn_stage_sobol(P.bluenoise, sob, tid, 256);
    __syncthreads();
    const uint32_t n = P.ws.counters[kCntQ3];
    const SceneView sc = scene_of(P);
    const PtQueue& q = P.ws.q3;
    const uint32_t allParts = (1u << kParts) - 1u;
    Fetch f;
    fetch_init(f, n, gridDim.x * 4u, blockIdx.x * 4u + (uint32_t)w, kChainStaticFirst);
    uint32_t rays = 0;
#pragma unroll 1
    while (true) {  // wave-uniform
        // ---- phase 1: trace queue-3 entries, recording the reserves taken
        uint32_t nRanges = 0;
        if (f.resLo < f.resHi) {  // the rest of a reserve (the static first batch, or one cut short)
            if (lane == 0) ranges[w][0] = make_uint2(f.resLo, f.resHi);
            nRanges = 1;
        }
        bool active = false, exhausted = false, occlusion = false;
        uint32_t idx = 0;
        TravRay r;
        TravState s;
        TravRec rec;  // scratch of chain_step (each iteration loads its own record)
        r.org = f3(0.0f);
        trav_init(s, sc.root);
#pragma unroll 1
        while (true) {
            const unsigned long long need = __ballot(!active && !exhausted);
            const unsigned long long busy = __ballot(active);
            if (need != 0ull && (__popcll(need) >= kRefillMin || busy == 0ull)) {
                const uint32_t k = (uint32_t)__popcll(need);
                if (f.resLo == f.resHi && nRanges < (uint32_t)kChainRanges) {
                    fetch_topup(f, n, P.ws.fetch, lane);
                    if (f.resLo < f.resHi) {
                        if (lane == 0) ranges[w][nRanges] = make_uint2(f.resLo, f.resHi);
                        ++nRanges;
                    }
                }
                const uint32_t avail = f.resHi - f.resLo;
                const bool none = avail == 0u;  // drained, or the reserve list is full
                if (!active && !exhausted) {
                    const uint32_t rank = lane_rank(need);
                    if (rank < avail) {
                        idx = f.resLo + rank;
                        const float4 o = q.rayO[idx], d = q.rayD[idx];
                        trav_setup(sc, f3(o.x, o.y, o.z), f3(d.x, d.y, d.z), r);
                        trav_init(s, sc.root);
                        active = true;
                        occlusion = (__float_as_uint(d.w) & kQShadowFlag) != 0u;
                    } else if (none) {
                        exhausted = true;
                    }
                }
                f.resLo += k < avail ? k : avail;
            }
            if (__ballot(active) == 0ull) break;
            // tail (no lane can be refilled: queue drained or reserve list full): plain per-lane
            // loop, as in k_trace_queue
            const bool tail = f.resLo == f.resHi && (f.drained == allParts || nRanges >= (uint32_t)kChainRanges);
            if (tail ? active : trav_lane_steps(active, s)) {
                bool done = false;
                do {
                    done = chain_step<kStats>(sc, r, s, rec, stk + tid) || s.iters >= 1024u || (occlusion && s.hitIdx >= 0);
                } while (tail && !done);
                if (done) {
                    P.ws.hitRec[idx] = make_float4(s.t, __uint_as_float((uint32_t)s.hitIdx), s.hitU, s.hitV);
                    P.ws.hitErr[idx] = s.hitErrT;
                    if (P.statsOut) {
                        const uint32_t p = __float_as_uint(q.rayO[idx].w);
                        atomicAdd(&P.statsOut[p].y, s.visits);
                        atomicAdd(&P.statsOut[p].z, s.tests);
                        atomicMax(&P.ws.counters[kCntMaxIter3], s.iters);
                        atomicAdd(&P.ws.counters[kCntVisQ3], s.visits);  // detail launches only
                        atomicAdd(&P.ws.counters[kCntTstQ3], s.tests);
                    }
                    active = false;
                }
            }
        }
        // ---- phase 2: resume this wave's entries, trace and finish their I4 rays
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // the hit records this wave wrote
        PathCtx c{P, f3(P.sunDir[0], P.sunDir[1], P.sunDir[2]), sob, BnPixel{0u, 0u}, 0, 0u, 0u, 0u, 0u};
        c.skyTree = P.skyTree;  // the light-CDF heaps from L2: LDS holds the traversal stacks
        c.sunTree = P.sunTree;
        uint32_t ri = 0, nq4 = 0;
#pragma unroll 1
        while (true) {
            const bool more = ri < nRanges;
            const uint2 rg = more ? ranges[w][ri] : make_uint2(0u, 0u);
            if (nq4 > 0u && (!more || nq4 + (rg.y - rg.x) > 64u)) {
                // trace the listed I4 rays (one per lane) to their first hit, then finish them
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // queue-4 records, slot list
                bool act = (uint32_t)lane < nq4;
                const uint32_t slot = act ? q4list[w][lane] : 0u;
                TravRay r4;
                TravState s4;
                {
                    const float4 o = P.ws.q4.rayO[slot], d = P.ws.q4.rayD[slot];  // slot 0 for idle lanes
                    trav_setup(sc, f3(o.x, o.y, o.z), f3(d.x, d.y, d.z), r4);
                }
                trav_init(s4, sc.root);
                TravRec rec4;
                const bool mine = act;
                if (nq4 < 16u) {  // few rays: plain per-lane loop (no ballots, no leaf batching)
#pragma unroll 1
                    while (act)
                        if (chain_step<kStats>(sc, r4, s4, rec4, stk + tid) || s4.iters >= 1024u || s4.hitIdx >= 0) act = false;
                } else {
#pragma unroll 1
                    while (__ballot(act) != 0ull) {
                        if (trav_lane_steps(act, s4)) {
                            if (chain_step<kStats>(sc, r4, s4, rec4, stk + tid) || s4.iters >= 1024u || s4.hitIdx >= 0)
                                act = false;
                        }
                    }
                }
                if (mine) {
                    PathVars v;
                    uint32_t p = 0, smp = 0;
                    c.rays = 0;
                    (void)resume_entry<4, false, false>(c, P.ws.q4, sc, slot,
                                                 make_float4(s4.t, __uint_as_float((uint32_t)s4.hitIdx), s4.hitU, s4.hitV),
                                                 s4.hitErrT, v, p, smp);
                    store_path_L(c, v, p, smp);
                    if (P.statsOut) {
                        atomicAdd(&P.statsOut[p].y, s4.visits);
                        atomicAdd(&P.statsOut[p].z, s4.tests);
                        atomicMax(&P.ws.counters[kCntMaxIter4], s4.iters);
                        atomicAdd(&P.ws.counters[kCntVisQ4], s4.visits);
                        atomicAdd(&P.ws.counters[kCntTstQ4], s4.tests);
                    }
                }
                nq4 = 0u;
                continue;
            }
            if (!more) break;
            const uint32_t i = rg.x + (uint32_t)lane;
            const bool act = i < rg.y;
            PathVars v;
            int kd = 5;
            uint32_t p = 0, smp = 0;
            c.rays = 0;
            c.diffuse = 0;
            if (act) kd = resume_entry<3, false, false>(c, q, sc, i, P.ws.hitRec[i], P.ws.hitErr[i], v, p, smp);
            const bool i4 = kd == 4;
            const uint32_t slot = wave_append(i4, &P.ws.counters[kCntQ4]);
            const unsigned long long m4 = __ballot(i4);
            if (act) {
                if (i4) {
                    ++c.rays;
                    enqueue(P.ws.q4, slot, v, p, smp);
                    q4list[w][nq4 + lane_rank(m4)] = slot;
                } else {
                    store_path_L(c, v, p, smp);
                }
                if (P.raysOut && c.rays) atomicAdd(&P.raysOut[p], c.rays);
                if (P.statsOut) {
                    if (c.rays) atomicAdd(&P.statsOut[p].x, c.rays);
                    if (c.diffuse) {
                        atomicAdd(&P.statsOut[p].w, c.diffuse);
                        atomicAdd(&P.ws.counters[kCntDiffRes3], c.diffuse);
                    }
                }
                rays += c.rays;
            }
            nq4 += (uint32_t)__popcll(m4);
            ++ri;
        }
        if (f.resLo == f.resHi && f.drained == allParts) break;  // queue 3 drained
    }
    add_rays(P, wgRays, rays, w);
}

// colour of the pixels with a deferred sample: the fp32 sample average in sample order
__global__ __launch_bounds__(256) void k_pt_resolve(PathTraceParams P) {
    const uint32_t n = P.ws.counters[kCntPending];
    if (P.ws.zeroNext && blockIdx.x == 0)  // the next serial frame's counter block (frame.cpp)
        for (int i = (int)threadIdx.x; i < kWsCounterWords; i += 256) P.ws.zeroNext[i] = 0u;
    // serial frames: queue 3's length into pinned host memory for the next frame's chain choice
    // (frame.cpp), a vector store over the bus instead of a copy on the stream
    if (P.ws.q3HostOut && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(P.ws.q3HostOut, ((unsigned long long)P.ws.q3Tag << 32) | P.ws.counters[kCntQ3], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll 1
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        const uint32_t e = P.ws.pending[i];
        const uint32_t pl = e & 0x3FFFFFFu, sd = e >> 26;
        const float4* ls = P.ws.pathL + (size_t)pl * P.spp;
        F3 L;
        if (P.spp == 1) {
            L = f3(ls[0].x, ls[0].y, ls[0].z);
        } else {
            L = f3(0.0f);
            if (sd > 0) L = f3(ls[sd - 1].x, ls[sd - 1].y, ls[sd - 1].z);  // prefix sum of samples < sd
            for (uint32_t s = sd; s < P.spp; ++s) L = L + f3(ls[s].x, ls[s].y, ls[s].z);
            L = div_spp(P, L);
        }
        const uint32_t p = row_of(P.y0, P.nStrips, P.strip, pl / P.width) * P.width + pl % P.width;
        const uint32_t mask = P.colorOut[p].y >> 16;
        P.colorOut[p] = pack_h4(L.x, L.y, L.z, mask);
    }
}


// src is zeroed for the next launches ahead; dst null: zero src only (they were dropped)
__global__ __launch_bounds__(256) void k_fold_ray_counts(unsigned long long* dst, unsigned long long* src) {
    const int k = (int)threadIdx.x;
    if (k >= kRayCounterSlots) return;
    if (dst) atomicAdd(&dst[k * kRayCounterStride], src[k * kRayCounterStride]);  // beside a frame's own counts
    src[k * kRayCounterStride] = 0ull;
}

extern "C" hipError_t rtk_fold_ray_counts(unsigned long long* dst, unsigned long long* src, hipStream_t stream) {
    static_assert(kRayCounterSlots <= 256, "one workgroup");
    hipLaunchKernelGGL(k_fold_ray_counts, dim3(1), dim3(256), 0, stream, dst, src);
    return hipGetLastError();
}

extern "C" hipError_t rtk_launch_pt_camera(const PathTraceParams* p, hipStream_t stream, hipEvent_t* marks) {
    if (p->spp < 1 || p->spp > 64 || p->ws.persistBlocks < 1) return hipErrorInvalidValue;
    if ((size_t)p->rows * p->width >= (1u << 26) || (size_t)p->rows * p->width * p->spp > p->ws.cap)
        return hipErrorInvalidValue;
    hipError_t e = p->ws.countersZeroed ? hipSuccess  // zeroed by the previous serial frame's resolve
                                        : hipMemsetAsync(p->ws.counters, 0, kWsCounterWords * sizeof(uint32_t), stream);
    if (e == hipSuccess && marks && marks[0]) e = hipEventRecord(marks[0], stream);  // begin / end of kernel 0
    if (e != hipSuccess) return e;
    const int nSW = cam_sample_waves(p->spp);
    const int BW = nSW == 4 ? 8 : 16, BH = nSW == 1 ? 16 : 8;
    const dim3 grid((p->width + BW - 1) / BW, (p->rows + BH - 1) / BH);
    const bool stats = p->statsOut != nullptr;
    void (*k)(PathTraceParams) = one_round(p->spp) ? (stats ? k_pt_camera<true, true> : k_pt_camera<true, false>)
                                                   : (stats ? k_pt_camera<false, true> : k_pt_camera<false, false>);
    hipLaunchKernelGGL(k, grid, dim3(256), 0, stream, *p);
    if (marks && marks[1] && (e = hipEventRecord(marks[1], stream)) != hipSuccess) return e;
    return hipGetLastError();
}

// hook (optional): called on the host right after each kernel is enqueued; the frame pipeline
// issues the previous frame's denoise and gates the next frame's camera rays there (frame.cpp).
namespace {
// the shade kernel's grid: with dynamic claims ws.shadeBlocksPerCu, or its residency (queried
// once per variant); the static split keeps persistBlocks
template <typename K>
dim3 shade_grid(const PathTraceParams* p, K kernel, int& cached) {
    if (cached == 0) {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, 256, 0) != hipSuccess || b < 1) b = 2;
        cached = b;
    }
    if (!p->ws.shadeClaim) return dim3(p->ws.persistBlocks);  // the static split's grid
    const uint32_t perCu = p->ws.shadeBlocksPerCu ? p->ws.shadeBlocksPerCu : (uint32_t)cached;
    return dim3(perCu * (p->ws.cus ? p->ws.cus : 256u));
}

template <bool kOneRound>
void launch_shade_rounds(const PathTraceParams* p, hipStream_t stream) {
    static int occ[3];
    const dim3 pb(256);
    if (p->ws.glossy) {
        auto k = k_pt_shade0<true, false, kOneRound>;
        hipLaunchKernelGGL(k, shade_grid(p, k, occ[0]), pb, 0, stream, *p);
    } else if (p->ws.microfacet) {
        auto k = k_pt_shade0<false, true, kOneRound>;
        hipLaunchKernelGGL(k, shade_grid(p, k, occ[1]), pb, 0, stream, *p);
    } else {
        auto k = k_pt_shade0<false, false, kOneRound>;
        hipLaunchKernelGGL(k, shade_grid(p, k, occ[2]), pb, 0, stream, *p);
    }
}

void launch_shade(const PathTraceParams* p, hipStream_t stream) {
    if (one_round(p->spp)) launch_shade_rounds<true>(p, stream);
    else launch_shade_rounds<false>(p, stream);
}

hipError_t launch_rest(const PathTraceParams* p, hipStream_t stream, hipEvent_t* marks, const PtLaunchHook* hook,
                       bool withShade);
}  // namespace

extern "C" hipError_t rtk_launch_pt_shade(const PathTraceParams* p, hipStream_t stream, hipEvent_t* marks) {
    hipError_t e;
    if (marks && marks[2] && (e = hipEventRecord(marks[2], stream)) != hipSuccess) return e;
    launch_shade(p, stream);
    if (marks && marks[3] && (e = hipEventRecord(marks[3], stream)) != hipSuccess) return e;
    return hipGetLastError();
}

extern "C" hipError_t rtk_launch_pt_rest(const PathTraceParams* p, hipStream_t stream, hipEvent_t* marks,
                                         const PtLaunchHook* hook) {
    return launch_rest(p, stream, marks, hook, true);
}

extern "C" hipError_t rtk_launch_pt_rest_after_shade(const PathTraceParams* p, hipStream_t stream, hipEvent_t* marks,
                                                     const PtLaunchHook* hook) {
    return launch_rest(p, stream, marks, hook, false);
}

namespace {
hipError_t launch_rest(const PathTraceParams* p, hipStream_t stream, hipEvent_t* marks, const PtLaunchHook* hook,
                       bool withShade) {
    hipError_t e = hipSuccess;  // the counters were zeroed before the camera kernel (rtk_launch_pt_camera)
    int k = 1;  // kernel 1 = shade; marks[2k] / marks[2k + 1] bracket kernel k on this stream
    // a null entry: that kernel is not bracketed (rt_frame_marks_begin's kernel mask)
    auto begin = [&]() { return marks && marks[2 * k] ? hipEventRecord(marks[2 * k], stream) : hipSuccess; };
    auto end = [&]() {  // the mark first: a hook that blocks the host must not delay it
        const hipError_t me = marks && marks[2 * k + 1] ? hipEventRecord(marks[2 * k + 1], stream) : hipSuccess;
        if (me != hipSuccess) return me;
        if (hook && hook->fn) {
            const hipError_t he = hook->fn(hook->arg, k);
            if (he != hipSuccess) return he;
        }
        ++k;
        return hipSuccess;
    };
    const dim3 pg(p->ws.persistBlocks), pb(256);
    if (withShade) {
        if ((e = begin()) != hipSuccess) return e;
        launch_shade(p, stream);
        if ((e = end()) != hipSuccess) return e;
    } else {  // enqueued by the caller on another stream: only the hook runs for kernel 1
        if (hook && hook->fn && (e = hook->fn(hook->arg, k)) != hipSuccess) return e;
        ++k;
    }
    if ((e = begin()) != hipSuccess) return e;
    if (p->ws.chain && !p->ws.glossy && !p->ws.microfacet) {
        // kernel 2 = the fused bounce chain (trace<3> .. resume<4>); slots 3-5 stay empty, so the
        // hook's kernel numbers and the per-kernel timing slots keep their meaning
        hipLaunchKernelGGL(p->statsOut ? k_pt_chain<true> : k_pt_chain<false>, dim3(p->ws.traceBlocks), pb, 0, stream, *p);
        for (int j = 0; j < 4; ++j)
            if ((e = end()) != hipSuccess || (e = begin()) != hipSuccess) return e;
    } else {
        if ((e = rtk_launch_trace_queue(p, 3, stream)) != hipSuccess || (e = end()) != hipSuccess) return e;
        if ((e = begin()) != hipSuccess) return e;
        if (p->ws.microfacet) hipLaunchKernelGGL((k_pt_resume<3, true, false>), pg, pb, 0, stream, *p);
        else if (p->ws.glossy) hipLaunchKernelGGL((k_pt_resume<3, false, true>), pg, pb, 0, stream, *p);
        else hipLaunchKernelGGL((k_pt_resume<3, false, false>), pg, pb, 0, stream, *p);
        if ((e = end()) != hipSuccess || (e = begin()) != hipSuccess) return e;
        if ((e = rtk_launch_trace_queue(p, 4, stream)) != hipSuccess || (e = end()) != hipSuccess) return e;
        if ((e = begin()) != hipSuccess) return e;
        hipLaunchKernelGGL((k_pt_resume<4, false, false>), pg, pb, 0, stream, *p);  // step 4 shades nothing
        if ((e = end()) != hipSuccess || (e = begin()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_pt_resolve, dim3(p->ws.persistBlocks), dim3(256), 0, stream, *p);
    if ((e = end()) != hipSuccess) return e;
    return hipGetLastError();
}
}  // namespace
