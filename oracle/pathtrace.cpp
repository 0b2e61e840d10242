// ORACLE (test infrastructure only; see ocommon.h) — per-pixel PathTrace.
//
// Restates PathTrace (pathtrace.cuh:11-128) with RayState (kernel.cuh:233-284):
//   RaySceneIntersect + UpdateMaterial          traverse.cuh:9-225 (geometry in traverse.cpp)
//   HistoryCamera::WorldToScreenSpace           kernel.cuh:135-155
//   GlossySurfaceInteraction                    surfaceInteraction.cuh:11-34, bsdf.cuh:131-166
//   DiffuseSurfaceInteraction                   surfaceInteraction.cuh:36-310 (triplanar textures,
//                                               SampleBicubicSmoothStepLod sampler.cuh:498-584)
//   LambertianSample / Macrofacet* / cosines    bsdf.cuh:36-354
//   SampleLight / BinarySearch / EnvLight2       light.cuh:9-305
//   NAN_DETECTER, clamp, demodulation, stores    pathtrace.cuh:113-127, debugUtil.h:158-168
// S samples per pixel (a build extension; S = 1 is the reference): sample s evaluates the
// reference PathTrace with frame index S*(frameNum-1)+1+s; demodulated colour and albedo are
// averaged in fp32 before the half store; normal/depth/motion/mask come from sample 0.
#include <atomic>
#include <thread>
#include <vector>

#include "oracle.h"
#include "ocommon.h"
#include "opath.h"

namespace orc {

F3 equal_area_map(float u, float v);
F3 equal_area_map_cone(F3 sunDir, float u, float v, float cosThetaMax);
void localize_sample(F3 n, F3& u, F3& v);

enum MatType { LAMBERTIAN = 0, PERFECT_REFLECTION = 1, FRESNEL_RR = 2, MICROFACET = 3, EMISSIVE = 4, MAT_SKY = 5 };
struct Material { F3 albedo; int type; F3 F0; float alpha; };

// init.cu:215-251 on top of the SurfaceMaterial defaults (kernel.cuh:184-189)
static void default_materials(Material* m) {
    for (int i = 0; i < 10; ++i) m[i] = {f3(0.8f), PERFECT_REFLECTION, f3(0.56f, 0.57f, 0.58f), 0.05f};
    m[0].type = EMISSIVE; m[0].albedo = f3(0.1f, 0.2f, 0.9f);
    m[1].type = FRESNEL_RR;
    m[2].type = EMISSIVE; m[2].albedo = f3(0.9f, 0.2f, 0.1f);
    m[3].type = LAMBERTIAN; m[3].albedo = f3(0.9f);
    m[4].type = MICROFACET; m[4].albedo = f3(0.9f); m[4].F0 = f3(0.56f, 0.57f, 0.58f); m[4].alpha = 0.05f;
    m[5].type = PERFECT_REFLECTION;
    m[6].type = LAMBERTIAN;
    m[7].type = LAMBERTIAN; m[7].albedo = f3(0.9f, 0.2f, 0.1f);
    m[8].type = LAMBERTIAN; m[8].albedo = f3(0.2f, 0.9f, 0.1f);
    m[9].type = LAMBERTIAN; m[9].albedo = f3(0.1f, 0.2f, 0.9f);
}

static const int ENV_LIGHT_ID = 9999, DEFAULT_LIGHT_ID = 7777;
static const float kInvTwoPi = 0.15915494309f;

struct RayState {
    F3 orig, dir, pos, normal, fakeNormal, beta0, beta1, albedo, centerRaydir;
    int matId, matType, lightIdx, objectIdx;
    bool isRayIntoSurface, hitLight, hit, isDiffuseRay, isDiffuse, isHitProcessed, isOccluded, isShadowRay;
    float offset, normalDotRayDir, depth, rayConeWidth, rayConeSpread;
    F2 uv;
};

struct Ctx {
    const OrcFrame* f;
    Material mats[10];
    Camera cam, hcam;
    F3 sunDir;
    uint32_t rays;
};

static bool isnan3(F3 v) { return v.x != v.x || v.y != v.y || v.z != v.z; }
static float clampf(float a, float lo = 0.0f, float hi = 1.0f) { return a < lo ? lo : a > hi ? hi : a; }
static F3 clamp3(F3 a, F3 lo, F3 hi) { return f3(clampf(a.x, lo.x, hi.x), clampf(a.y, lo.y, hi.y), clampf(a.z, lo.z, hi.z)); }

// ------------------------------------------------------------------ RaySceneIntersect
static void update_material(Ctx& c, RayState& rs) {
    if (!rs.hit) {
        rs.matType = MAT_SKY;
        rs.matId = 99999;
    } else {
        int n = (int)c.f->triCount;
        if (c.f->materialOverride >= 0) rs.matId = c.f->materialOverride;
        else rs.matId = (rs.objectIdx >= 0 && rs.objectIdx < n) ? 3 : 6;  // SAFE_LOAD default 6
        rs.matType = (rs.matId >= 0 && rs.matId < 10) ? c.mats[rs.matId].type : PERFECT_REFLECTION;
    }
    if (rs.isShadowRay) {
        if ((rs.matType == EMISSIVE && rs.lightIdx == rs.objectIdx) || (rs.matType == MAT_SKY && rs.lightIdx == ENV_LIGHT_ID))
            rs.hitLight = true;
        else
            rs.isOccluded = true;
    } else {
        rs.hitLight = rs.matType == EMISSIVE || rs.matType == MAT_SKY;
    }
    rs.isDiffuse = (rs.matType == LAMBERTIAN) || (rs.matType == MICROFACET);
}

static void scene_intersect(Ctx& c, RayState& rs) {
    if (rs.hitLight || !rs.isHitProcessed || rs.isOccluded) return;
    rs.isHitProcessed = false;
    ++c.rays;
    OrcHit h;
    intersect_one(&c.f->scene, rs.orig, rs.dir, h);
    rs.offset = h.offset;
    rs.objectIdx = h.objectIdx;
    rs.pos = f3(h.pos[0], h.pos[1], h.pos[2]);
    rs.uv = F2{h.u, h.v};
    rs.normal = f3(h.normal[0], h.normal[1], h.normal[2]);          // flipped; (0,-1,0) on a miss
    rs.fakeNormal = f3(h.fakeNormal[0], h.fakeNormal[1], h.fakeNormal[2]);
    rs.normalDotRayDir = h.ndr;
    rs.isRayIntoSurface = h.intoSurface != 0;
    rs.hit = h.hit != 0;
    rs.depth = h.t;
    if (rs.hit) rs.rayConeWidth += rs.rayConeSpread * h.t;
    update_material(c, rs);
}

// ------------------------------------------------------------------ textures
static float tex_channel(const uint16_t* tex, int level, int x, int y, int ch) {
    size_t off = 0;
    for (int l = 0; l < level; ++l) off += (size_t)(1024 >> l) * (1024 >> l);
    int n = 1024 >> level;
    return (float)tex[(off + (size_t)y * n + x) * 4 + ch] / 65535.0f;
}

static int wrap(int v, int size) {  // BoundaryFuncRepeat (sampler.cuh:313-326) + surface clamp
    if (v >= size) v %= size;
    if (v < 0) v = size - (-v) % size;  // yields `size` for multiples of -size ...
    return v < size ? v : size - 1;     // ... which surf2Dread's cudaBoundaryModeClamp clamps
}

struct F4 { float x, y, z, w; };

static F4 bicubic_smoothstep_tex(const uint16_t* tex, int level, F2 uv) {
    const int n = 1024 >> level;
    F2 UV = {uv.x * (float)n, uv.y * (float)n};
    F2 tc = {floorf(UV.x - 0.5f) + 0.5f, floorf(UV.y - 0.5f) + 0.5f};
    F2 f = {UV.x - tc.x, UV.y - tc.y};
    F2 f2 = {f.x * f.x, f.y * f.y};
    F2 f3v = {f2.x * f.x, f2.y * f.y};
    F2 w1 = {f3v.x * -2.0f + f2.x * 3.0f, f3v.y * -2.0f + f2.y * 3.0f};
    F2 w0 = {1.0f - w1.x, 1.0f - w1.y};
    int t0x = (int)floorf(UV.x - 0.5f), t0y = (int)floorf(UV.y - 0.5f);
    int t1x = t0x + 1, t1y = t0y + 1;
    int sx[4] = {t0x, t1x, t0x, t1x}, sy[4] = {t0y, t0y, t1y, t1y};
    float wts[4] = {w0.x * w0.y, w1.x * w0.y, w0.x * w1.y, w1.x * w1.y};
    F4 o = {0, 0, 0, 0};
    float sw = 0.0f;
    for (int i = 0; i < 4; ++i) {
        sw += wts[i];
        int x = wrap(sx[i], n), y = wrap(sy[i], n);
        o.x += tex_channel(tex, level, x, y, 0) * wts[i];
        o.y += tex_channel(tex, level, x, y, 1) * wts[i];
        o.z += tex_channel(tex, level, x, y, 2) * wts[i];
        o.w += tex_channel(tex, level, x, y, 3) * wts[i];
    }
    o.x /= sw; o.y /= sw; o.z /= sw; o.w += sw;  // Float4::operator/= (linearMath.h:433)
    return o;
}

static F4 sample_lod(const uint16_t* tex, F2 uv, float lod) {
    float low = floorf(lod);
    float fr = lod - low;
    int lo = (int)low, hi = lo + 1;
    lo = lo < 0 ? 0 : lo > 10 ? 10 : lo;
    hi = hi < 0 ? 0 : hi > 10 ? 10 : hi;
    F4 a = bicubic_smoothstep_tex(tex, lo, uv), b = bicubic_smoothstep_tex(tex, hi, uv);
    float ia = 1.0f - fr;
    return F4{a.x * ia + b.x * fr, a.y * ia + b.y * fr, a.z * ia + b.z * fr, a.w * ia + b.w * fr};
}

// ------------------------------------------------------------------ env lookups
static F3 sky_texel(const float* buf, int x, int y) {  // BoundaryFuncRepeatXClampY, 512x256
    if (x >= 512) x %= 512;
    if (x < 0) x = 512 - (-x) % 512;
    if (x >= 512) x = 511;
    if (y >= 256) y = 255;
    if (y < 0) y = 0;
    const float* p = buf + ((size_t)y * 512 + x) * 4;
    return f3(p[0], p[1], p[2]);
}
static F3 sun_texel(const float* buf, int x, int y) {
    // BoundaryFuncDefault + surface clamp on the 512x256 allocation the reference uses for
    // SunBuffer (init.cu:496): only 32x32 is written, the rest reads as zero.
    if (x < 0) x = 0;
    if (y < 0) y = 0;
    if (x >= 32 || y >= 32) return f3(0.0f);
    const float* p = buf + ((size_t)y * 32 + x) * 4;
    return f3(p[0], p[1], p[2]);
}

template <typename Fetch>
static F3 bicubic_smoothstep_env(Fetch fetch, F2 uv, int W, int H) {
    F2 UV = {uv.x * (float)W, uv.y * (float)H};
    F2 tc = {floorf(UV.x - 0.5f) + 0.5f, floorf(UV.y - 0.5f) + 0.5f};
    F2 f = {UV.x - tc.x, UV.y - tc.y};
    F2 f2 = {f.x * f.x, f.y * f.y};
    F2 f3v = {f2.x * f.x, f2.y * f.y};
    F2 w1 = {f3v.x * -2.0f + f2.x * 3.0f, f3v.y * -2.0f + f2.y * 3.0f};
    F2 w0 = {1.0f - w1.x, 1.0f - w1.y};
    int t0x = (int)floorf(UV.x - 0.5f), t0y = (int)floorf(UV.y - 0.5f);
    int sx[4] = {t0x, t0x + 1, t0x, t0x + 1}, sy[4] = {t0y, t0y, t0y + 1, t0y + 1};
    float wts[4] = {w0.x * w0.y, w1.x * w0.y, w0.x * w1.y, w1.x * w1.y};
    F3 o = f3(0.0f);
    float sw = 0.0f;
    for (int i = 0; i < 4; ++i) {
        sw += wts[i];
        o = o + fetch(sx[i], sy[i]) * wts[i];
    }
    return o / sw;
}

static F2 equal_area_inverse(F3 d) {
    float u = rt_atan2f(-d.z, -d.x) / kTwoPi + 0.5f;
    float v = fmx(d.y, 0.05f);
    return F2{u, v};
}

static bool equal_area_cone_inverse(F2& uv, F3 sunDir, F3 rd, float cosMax) {
    F3 t, b;
    localize_sample(sunDir, t, b);
    // transpose(Mat3(t, sunDir, b)) * rd: rows t, sunDir, b
    F3 c = f3(inner3(t.x, rd.x, t.y, rd.y, t.z, rd.z), inner3(sunDir.x, rd.x, sunDir.y, rd.y, sunDir.z, rd.z),
              inner3(b.x, rd.x, b.y, rd.y, b.z, rd.z));
    float cosTheta = c.y;
    if (cosTheta < cosMax) return false;
    float u = (1.0f - cosTheta) / (1.0f - cosMax);
    float sinTheta = sqrtf(1.0f - cosTheta * cosTheta);
    if (sinTheta < 1e-5f || (c.x / sinTheta) < -1.0f || (c.x / sinTheta) > 1.0f) return false;
    float v = rt_acosf(c.x / sinTheta) * kInvTwoPi;
    uv = F2{u, v};
    return true;
}

static F3 env_light(const Ctx& c, F3 rd) {
    const OrcFrame* f = c.f;
    F3 color = f3(0.0f);
    {
        F3 sky = bicubic_smoothstep_env([&](int x, int y) { return sky_texel(f->skyBuffer, x, y); },
                                        equal_area_inverse(rd), 512, 256);
        F3 mist = f3(0.2f);
        float w = clampf((rd.y + 0.4f) * (1.0f / 0.5f));
        color = color + (mist + (w * w * (3.0f - 2.0f * w)) * (sky - mist));
    }
    F2 uv;
    if (equal_area_cone_inverse(uv, c.sunDir, rd, f->sunAngleCosThetaMax))
        color = color + bicubic_smoothstep_env([&](int x, int y) { return sun_texel(f->sunBuffer, x, y); }, uv, 32, 32);
    return color;
}

static int binary_search(const float* a, int left, int right, float target) {
    while (right - left > 1) {
        int mid = (left + right) / 2;
        if (a[mid] < target) left = mid;
        else right = mid;
    }
    return left;
}

static void sample_light(const Ctx& c, F3& dir, float& pdf, int& lightIdx, const float r[4]) {
    const OrcFrame* f = c.f;
    const float maxSky = f->skyCdf[131072 - 1], maxSun = f->sunCdf[1024 - 1];
    const float totalSky = maxSky * kTwoPi / 131072;
    const float totalSun = maxSun * kTwoPi * (1.0f - f->sunAngleCosThetaMax) / 1024;
    const float pSky = totalSky / (totalSky + totalSun);
    if (pSky > r[1]) {
        const int idx = binary_search(f->skyCdf, 0, 131072 - 2, r[0] * maxSky) + 1;
        float p = (f->skyCdf[idx] - f->skyCdf[idx - 1]) / maxSky;
        p = p * 131072 / kTwoPi;
        float u = ((float)(idx % 512) + 0.5f) / 512;
        float v = ((float)(idx / 512) + 0.5f) / 256;
        dir = equal_area_map(u, v);
        pdf = p * 1.0f * pSky;
    } else {
        const int idx = binary_search(f->sunCdf, 0, 1024 - 2, r[0] * maxSun) + 1;
        float p = (f->sunCdf[idx] - f->sunCdf[idx - 1]) / maxSun;
        p = p * 1024 / (kTwoPi * (1.0f - f->sunAngleCosThetaMax));
        float u = ((float)(idx % 32) + 0.5f) / 32;
        float v = ((float)(idx / 32) + 0.5f) / 32;
        dir = equal_area_map_cone(c.sunDir, u, v, f->sunAngleCosThetaMax);
        pdf = p * 1.0f;
    }
    lightIdx = ENV_LIGHT_ID;
}

// ------------------------------------------------------------------ BSDFs
static const float kSafeCos = 1e-5f;

static void lambertian_sample(F2 u, F3& wo, F3 n) {
    float r = sqrtf(u.x);
    float theta = kTwoPi * u.y;
    F2 d = {r * rt_cosf(theta), r * rt_sinf(theta)};
    float z = sqrtf(max1f(0.0f, 1.0f - d.x * d.x - d.y * d.y));
    F3 s = f3(d.x, z, d.y);
    F3 uu, vv;
    localize_sample(n, uu, vv);
    wo = s.x * uu + s.z * vv + s.y * n;
    wo = normalize(wo);
}

static F3 fresnel_schlick(F3 F0, float cosTheta) {
    float e = 1.0f - cosTheta;
    float e2 = e * e;
    float p5 = e2 * e2 * e;
    return F0 + (f3(1.0f) - F0) * p5;
}

static void microfacet_eval(F3& brdfOverPdf, F3& brdf, float& pdf, F3 wn, F3 wo, F3 wi, F3 F0, F3 albedo, float alpha) {
    float alpha2 = alpha * alpha;
    if (dot(wo, wn) <= 0 || dot(wi, wn) <= 0) { brdfOverPdf = f3(0.0f); brdf = f3(0.0f); pdf = 1; }
    F3 wh = normalize(wi + wo);
    float cWoWh = fmx(kSafeCos, dot(wh, wo));
    F3 F = fresnel_schlick(F0, cWoWh);
    float cWo = clampf(dot(wo, wn), kSafeCos, 1.0f - kSafeCos);
    float cWi = fmx(kSafeCos, dot(wi, wn));
    float tWo = sqrtf(1.0f - cWo * cWo) / cWo;
    float G = 1.0f / (1.0f + (sqrtf(1.0f + alpha2 * tWo * tWo) - 1.0f) / 2.0f);
    float cWh = fmx(kSafeCos, dot(wh, wn));
    float c2 = cWh * cWh;
    float t2 = (1.0f - c2) / c2;
    float e = t2 / alpha2 + 1.0f;
    float D = 1.0f / (kPi * (alpha2 * c2 * c2) * (e * e));
    brdf = (albedo * F) * (D * G) / (4.0f * cWo * cWi);
    pdf = (D * cWh) / (4.0f * cWoWh);
    brdfOverPdf = (albedo * F) * (G * cWoWh) / (cWh * cWo);
}

static F3 reflect3(F3 i, F3 n) { return i - 2.0f * n * dot(n, i); }

static void microfacet_sample(F2 r, F2 r2, F3 raydir, F3& nextdir, F3 normal, F3 surfaceNormal, F3& brdfOverPdf, F3& brdf,
                              float& pdf, F3 F0, F3 albedo, float alpha) {
    float alpha2 = alpha * alpha;
    // float/double mix of bsdf.cuh:187-190: 1.0f / sqrt(float) -> float sqrtf
    float cosTheta = 1.0f / sqrtf(1.0f + alpha2 * r.x / (1.0f - r.x));
    float sinTheta = sqrtf(1.0f - cosTheta * cosTheta);
    float phi = kTwoPi * r.y;
    F3 sl = f3(sinTheta * rt_cosf(phi), cosTheta, sinTheta * rt_sinf(phi));
    F3 t, b;
    localize_sample(normal, t, b);
    F3 sn = sl.x * t + sl.z * b + sl.y * normal;
    sn = normalize(sn);
    nextdir = normalize(reflect3(raydir, sn));
    if (dot(nextdir, surfaceNormal) < 0) {
        cosTheta = 1.0f / sqrtf(1.0f + alpha2 * r2.x / (1.0f - r2.x));
        sinTheta = sqrtf(1.0f - cosTheta * cosTheta);
        phi = kTwoPi * r2.y;
        sl = f3(sinTheta * rt_cosf(phi), cosTheta, sinTheta * rt_sinf(phi));
        F3 t2, b2;
        localize_sample(normal, t2, b2);
        F3 sn2 = sl.x * t2 + sl.z * b2 + sl.y * normal;
        sn2 = normalize(sn2);
        nextdir = normalize(reflect3(raydir, sn2));
        if (dot(nextdir, surfaceNormal) < 0) nextdir = normalize(reflect3(raydir, normal));
    }
    F3 wi = nextdir, wo = -raydir, wh = sn, wn = normal;  // wh: the FIRST sampled normal (bsdf.cuh:229)
    float cWoWh = fmx(kSafeCos, dot(wh, wo));
    F3 F = fresnel_schlick(F0, cWoWh);
    float cWo = clampf(dot(wo, wn), kSafeCos, 1.0f - kSafeCos);
    float cWi = fmx(kSafeCos, dot(wi, wn));
    float tWo = sqrtf(1.0f - cWo * cWo) / cWo;
    float G = 1.0f / (1.0f + (sqrtf(1.0f + alpha2 * tWo * tWo) - 1.0f) / 2.0f);
    float cWh = fmx(kSafeCos, dot(wh, wn));
    float c2 = cWh * cWh;
    float tt = (1.0f - c2) / c2;
    float e = tt / alpha2 + 1.0f;
    float D = 1.0f / (kPi * (alpha2 * c2 * c2) * (e * e));
    brdf = (albedo * F) * (D * G) / (4.0f * cWo * cWi);
    pdf = (D * cWh) / (4.0f * cWoWh);
    brdfOverPdf = (albedo * F) * (G * cWoWh) / (cWh * cWo);
}

static void glossy(Ctx& c, RayState& rs, float rnd) {
    if (rs.hitLight || rs.isDiffuse || rs.isOccluded) return;
    rs.isHitProcessed = true;
    if (rs.matType == PERFECT_REFLECTION) {
        rs.dir = normalize(rs.dir - rs.normal * dot(rs.dir, rs.normal) * 2.0f);
        rs.orig = rs.pos + rs.offset * rs.normal;
    } else if (rs.matType == FRESNEL_RR) {
        float etaI = 1.0f, etaT = 1.33f;
        if (!rs.isRayIntoSurface) { float t = etaI; etaI = etaT; etaT = t; }
        const float eta = etaI / etaT;
        float ndr = rs.normalDotRayDir;
        float cosI = -ndr;
        float sin2I = max1f(0, (float)(1.0 - (double)(cosI * cosI)));
        float sin2T = eta * eta * sin2I;
        float cosT = sqrtf(max1f(0, (float)(1.0 - (double)sin2T)));
        F3 next;
        float off = rs.offset;
        if (sin2T >= 1.0f) {
            next = rs.dir - rs.normal * ndr * 2.0f;
        } else {
            float R1 = etaT * cosI, R2 = etaI * cosT, R3 = etaI * cosI, R4 = etaT * cosT;
            float Rparl = (R1 - R2) / (R1 + R2), Rperp = (R3 - R4) / (R3 + R4);
            float fres = (float)((double)(Rparl * Rparl + Rperp * Rperp) / 2.0);
            if (rnd < fres) next = rs.dir - rs.normal * ndr * 2.0f;
            else { next = eta * rs.dir + (eta * cosI - cosT) * rs.normal; off = -off; }
        }
        rs.dir = normalize(next);
        rs.orig = rs.pos + off * rs.normal;
    }
}

static void diffuse(Ctx& c, int bounce, RayState& rs, F3& beta, const float r[4], const float r2[4]) {
    if (rs.hitLight || !rs.isDiffuse || rs.isOccluded) return;
    rs.isDiffuseRay = true;
    rs.lightIdx = DEFAULT_LIGHT_ID;
    rs.isHitProcessed = true;
    const Material& mat = c.mats[rs.matId];
    F3 normal = rs.fakeNormal, surfaceNormal = rs.normal;
    F3 albedo;
    {
        const float uvScale = 0.5f;
        float len = sqrtf(1024.0f * 1024.0f + 1024.0f * 1024.0f);
        float lod = rt_log2f_div(rs.rayConeWidth * uvScale * len);  // the path tracer's log2 variant (rtmath.h log2_pair_t)
        F3 aX, aY, aZ, nX, nY, nZ;
        const uint16_t* T0 = c.f->texAlbedoAo;
        const uint16_t* T1 = c.f->texNormalRough;
        auto plane = [&](F2 uv, F3 wDefault, bool alt, F3 wAlt, F3& alb, F3& nrm) {
            uv.x *= uvScale;
            uv.y *= uvScale;
            F4 t0 = sample_lod(T0, uv, lod);
            alb = f3(rt_powf_div(t0.x, 2.2f), rt_powf_div(t0.y, 2.2f), rt_powf_div(t0.z, 2.2f));
            F4 t1 = sample_lod(T1, uv, lod);
            F3 n = f3(t1.x - 0.5f, t1.y - 0.5f, t1.z - 0.5f);
            F3 w = alt ? wAlt : wDefault;
            F3 u = cross(normal, w);
            F3 v = cross(normal, u);
            nrm = normalize(u * n.x + v * n.y + normal * n.z);
        };
        plane(F2{rs.pos.y, rs.pos.z}, f3(0, 1, 0), fabsf(normal.y) > 0.999f, f3(0, 0, 1), aX, nX);
        plane(F2{rs.pos.x, rs.pos.z}, f3(1, 0, 0), fabsf(normal.x) > 0.999f, f3(0, 0, 1), aY, nY);
        plane(F2{rs.pos.x, rs.pos.y}, f3(0, 1, 0), fabsf(normal.y) > 0.999f, f3(1, 0, 0), aZ, nZ);
        float wx = surfaceNormal.x * surfaceNormal.x, wy = surfaceNormal.y * surfaceNormal.y,
              wz = surfaceNormal.z * surfaceNormal.z;
        albedo = aX * wx + aY * wy + aZ * wz;
        F3 texNormal = normalize(nX * wx + nY * wy + nZ * wz);
        normal = texNormal;
        rs.fakeNormal = normal;
    }
    if (bounce == 0) rs.albedo = albedo * (1.0f + fabsf(dot(normal, rs.centerRaydir)));
    F3 rayDir = rs.dir;
    F3 lDir;
    float lPdf = 1;
    int lIdx;
    sample_light(c, lDir, lPdf, lIdx, r2);
    F3 sDir, sBsdfOverPdf, sBsdf, lBsdfOverPdf, lBsdf;
    float sPdf = 0, lsPdf = 0;
    F2 u1 = {r[0], r[1]}, u2 = {r[2], r[3]};
    if (rs.matType == LAMBERTIAN) {
        lambertian_sample(u1, sDir, normal);
        sBsdfOverPdf = albedo;
        sBsdf = albedo / kPi;
        sPdf = fmx(dot(sDir, normal), kSafeCos) / kPi;
        lBsdfOverPdf = albedo;
        lBsdf = albedo / kPi;
        lsPdf = fmx(dot(lDir, normal), kSafeCos) / kPi;
    } else if (rs.matType == MICROFACET) {
        microfacet_sample(u1, u2, rayDir, sDir, normal, surfaceNormal, sBsdfOverPdf, sBsdf, sPdf, mat.F0, albedo, mat.alpha);
        microfacet_eval(lBsdfOverPdf, lBsdf, lsPdf, normal, -rayDir, lDir, mat.F0, albedo, mat.alpha);
    }
    if (isnan3(lBsdf)) lBsdf = f3(0.0f);
    if (isnan3(sBsdf)) sBsdf = f3(0.0f);
    if (sPdf != sPdf) sPdf = 0.0f;
    if (lPdf != lPdf) lPdf = 0.0f;
    float ph = (sPdf * sPdf) / (sPdf * sPdf + lPdf * lPdf);
    const float minPdf = 1e-5f;
    if (r[3] < ph) {
        if (dot(rs.normal, sDir) < 0) { rs.isOccluded = true; return; }
        float cwi = fmx(kSafeCos, dot(sDir, normal));
        beta = sBsdf * cwi / fmx(sPdf, minPdf);
        rs.dir = sDir;
    } else {
        if (dot(rs.normal, lDir) < 0) { rs.isOccluded = true; return; }
        float cwi = fmx(kSafeCos, dot(lDir, normal));
        beta = lBsdf * cwi / fmx(lPdf, minPdf);
        rs.dir = lDir;
        rs.lightIdx = lIdx;
        rs.isShadowRay = true;
    }
    if (isnan3(beta)) beta = f3(0.0f);
    rs.orig = rs.pos + rs.offset * rs.normal;
}

// HistoryCamera::WorldToScreenSpace (kernel.cuh:144-151)
static F2 world_to_screen(const Camera& h, F3 p, F2 tanHalfFov) {
    F3 d = p - h.pos;
    F3 v = f3(dot(h.left, d), dot(h.up, d), dot(h.dir, d));
    F2 s = {v.x / v.z, v.y / v.z};
    F2 ndc = {s.x / tanHalfFov.x, s.y / tanHalfFov.y};
    return F2{0.5f - ndc.x * 0.5f, 0.5f - ndc.y * 0.5f};
}

struct SampleOut {
    F3 L2, albedo, normal;
    float depth;
    F2 motion;
    uint16_t mask;
};

static void path_trace_sample(Ctx& c, int x, int y, int frameIdx, SampleOut& o) {
    const OrcFrame* f = c.f;
    RayState rs;
    memset(&rs, 0, sizeof(rs));
    rs.beta0 = f3(1.0f);
    rs.beta1 = f3(1.0f);
    rs.isDiffuseRay = false;
    rs.hitLight = false;
    rs.lightIdx = DEFAULT_LIGHT_ID;
    rs.isHitProcessed = true;
    rs.isOccluded = false;
    rs.isShadowRay = false;
    rs.normal = f3(0.0f, -1.0f, 0.0f);
    rs.albedo = f3(1.0f);
    rs.rayConeWidth = 0.0f;
    rs.rayConeSpread = ray_cone_width(c.cam, x, y);
    float rn[4][4];
    for (int k = 0; k < 4; ++k)
        for (int d = 0; d < 4; ++d) rn[k][d] = bluenoise(f->bluenoise, x, y, frameIdx * 4 + k, d);
    F2 sampleUv;
    generate_ray(c.cam, x, y, F2{rn[0][0], rn[0][1]}, F2{rn[0][2], rn[0][3]}, rs.orig, rs.dir, rs.centerRaydir, sampleUv);
    scene_intersect(c, rs);
    float outDepth = rs.depth;
    uint16_t mask = (uint16_t)rs.matId;
    F2 mv = {0.0f, 0.0f};
    if (rs.hit) {
        F2 last = world_to_screen(c.hcam, rs.pos, c.cam.tanHalfFov);
        mv = F2{last.x - sampleUv.x, last.y - sampleUv.y};
    }
    mv = F2{mv.x + 0.5f, mv.y + 0.5f};
    glossy(c, rs, rn[0][0]);
    scene_intersect(c, rs);
    glossy(c, rs, rn[0][1]);
    scene_intersect(c, rs);
    glossy(c, rs, rn[0][2]);
    diffuse(c, 0, rs, rs.beta1, rn[0], rn[1]);
    F3 outNormal = rs.fakeNormal;
    scene_intersect(c, rs);
    glossy(c, rs, rn[0][3]);
    diffuse(c, 1, rs, rs.beta0, rn[2], rn[3]);
    scene_intersect(c, rs);
    F3 L0 = f3(0.0f);
    if (rs.hitLight && !rs.isOccluded && rs.matType == MAT_SKY) L0 = env_light(c, rs.dir);
    F3 L2 = L0 * rs.beta0 * rs.beta1;
    if (isnan3(L2)) L2 = f3(0.0f);
    if (isnan3(outNormal)) outNormal = f3(0.0f);
    if (outDepth != outDepth) outDepth = 0.0f;
    if (mv.x != mv.x || mv.y != mv.y) mv = F2{0.0f, 0.0f};
    L2 = clamp3(L2, f3(0.0f), f3(10.0f));
    L2 = L2 / rs.albedo;
    o.L2 = L2;
    o.albedo = rs.albedo;
    o.normal = outNormal;
    o.depth = outDepth;
    o.motion = mv;
    o.mask = mask;
}

}  // namespace orc

using namespace orc;



extern "C" void orc_pathtrace(const OrcFrame* f, uint32_t W, uint32_t H, uint32_t y0, uint32_t rows, OrcGBuffer* out,
                              int threads) {
    if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
    if (threads < 1) threads = 1;
    Ctx proto;
    proto.f = f;
    default_materials(proto.mats);
    camera_update(f->cam, proto.cam);
    camera_update(f->histCam, proto.hcam);
    proto.sunDir = f3(f->sunDir[0], f->sunDir[1], f->sunDir[2]);
    std::atomic_uint next(0);
    const uint32_t n = W * rows;
    auto work = [&]() {
        Ctx c = proto;
        for (;;) {
            uint32_t lo = next.fetch_add(64);
            if (lo >= n) break;
            uint32_t hi = lo + 64 < n ? lo + 64 : n;
            for (uint32_t k = lo; k < hi; ++k) {
                int x = (int)(k % W), y = (int)(y0 + k / W);
                size_t p = (size_t)y * W + x;
                c.rays = 0;
                F3 sumL = f3(0.0f), sumA = f3(0.0f);
                SampleOut s0{};
                for (uint32_t s = 0; s < f->spp; ++s) {
                    SampleOut so;
                    int frameIdx = (int)f->spp * (f->frameNum - 1) + 1 + (int)s;
                    path_trace_sample(c, x, y, frameIdx, so);
                    if (s == 0) s0 = so;
                    sumL = sumL + so.L2;
                    sumA = sumA + so.albedo;
                }
                F3 L = f->spp == 1 ? s0.L2 : sumL / (float)f->spp;
                F3 A = f->spp == 1 ? s0.albedo : sumA / (float)f->spp;
                out->color[4 * p + 0] = rt_f2h(L.x);
                out->color[4 * p + 1] = rt_f2h(L.y);
                out->color[4 * p + 2] = rt_f2h(L.z);
                out->color[4 * p + 3] = s0.mask;
                out->normal[4 * p + 0] = rt_f2h(s0.normal.x);
                out->normal[4 * p + 1] = rt_f2h(s0.normal.y);
                out->normal[4 * p + 2] = rt_f2h(s0.normal.z);
                out->normal[4 * p + 3] = rt_f2h(0.0f);
                out->albedo[4 * p + 0] = rt_f2h(A.x);
                out->albedo[4 * p + 1] = rt_f2h(A.y);
                out->albedo[4 * p + 2] = rt_f2h(A.z);
                out->albedo[4 * p + 3] = rt_f2h(0.0f);
                out->depth[p] = rt_f2h(s0.depth);
                out->motion[2 * p + 0] = rt_f2h(s0.motion.x);
                out->motion[2 * p + 1] = rt_f2h(s0.motion.y);
                if (out->rays) out->rays[p] = c.rays;
            }
        }
    };
    if (threads == 1) { work(); return; }
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t) pool.emplace_back(work);
    for (auto& th : pool) th.join();
}
