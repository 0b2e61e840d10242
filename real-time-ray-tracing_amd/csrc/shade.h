// shade.h — device-side surface/light evaluation of the path tracer, with the reference's
// arithmetic order (one rounding per operation; -ffp-contract=off build).
//
//   material table / UpdateMaterial   init.cu:215-251, kernel.cuh:182-196, traverse.cuh:9-56
//   SampleBicubicSmoothStep(Lod)      sampler.cuh:498-584 (+ boundary functors 293-339)
//   EqualAreaMap / EqualAreaMapCone   sky.cuh:33-87
//   EnvLight2 / SampleLight           light.cuh:33-273
//   Lambertian / Microfacet / glass   bsdf.cuh:36-300
//   GlossySurfaceInteraction          surfaceInteraction.cuh:11-34
//   DiffuseSurfaceInteraction         surfaceInteraction.cuh:36-310 (triplanar soil textures)
#pragma once
#include "frame_kernels.h"
#include "pt_common.h"
#include "rtmath.h"

namespace rtd {

enum MatType : int { LAMBERTIAN = 0, PERFECT_REFLECTION = 1, FRESNEL_RR = 2, MICROFACET = 3, EMISSIVE = 4, MAT_SKY = 5 };
constexpr int kEnvLightId = 9999, kDefaultLightId = 7777;
constexpr float kInvTwoPi = 0.15915494309f;
constexpr float kSafeCos = 1e-5f;

// Reference material table (init.cu:215-251 over the SurfaceMaterial defaults).
RT_DEV int mat_type(int id) {
    // 0 E, 1 glass, 2 E, 3 L, 4 MF, 5 mirror, 6..9 L
    switch (id) {
        case 0: case 2: return EMISSIVE;
        case 1: return FRESNEL_RR;
        case 3: case 6: case 7: case 8: case 9: return LAMBERTIAN;
        case 4: return MICROFACET;
        default: return PERFECT_REFLECTION;
    }
}
RT_DEV F3 mat_F0(int) { return f3(0.56f, 0.57f, 0.58f); }
RT_DEV float mat_alpha(int) { return 0.05f; }

RT_DEV F3 f3_4(float4 a) { return f3(a.x, a.y, a.z); }
RT_DEV float clampf(float a, float lo = 0.0f, float hi = 1.0f) { return a < lo ? lo : a > hi ? hi : a; }
RT_DEV bool isnan3(F3 v) { return v.x != v.x || v.y != v.y || v.z != v.z; }

// ------------------------------------------------------------------ textures
struct F4 { float x, y, z, w; };

RT_DEV F4 load_u16x4(const uint2* tex, uint32_t texel) {
    // a 32-bit byte offset from the (uniform) chain base: one VGPR per address, not two
    const uint2 q = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(tex) + texel * 8u);
    return F4{rt_unorm16(q.x & 0xFFFFu), rt_unorm16(q.x >> 16), rt_unorm16(q.y & 0xFFFFu), rt_unorm16(q.y >> 16)};
}

// BoundaryFuncRepeat, then the surface read's clamp: v % size for v >= size, size - (-v) % size
// for v < 0 — which is `size` for multiples of -size, clamped to size - 1.  Mip sizes are powers
// of two, so both remainders are a mask.
RT_DEV int wrap_repeat(int v, int size) {
    const int r = v & (size - 1);
    return (v < 0 && r == 0) ? size - 1 : r;
}

// SampleBicubicSmoothStep<Load2DFuncUshort4<Float4>, Float4, BoundaryFuncRepeat> on one mip level
RT_DEV F4 bicubic_tex(const uint2* tex, int level, F2 uv) {
    const int n = kTexSize >> level;
    const uint32_t base = tex_level_offset(level);
    const F2 UV = {uv.x * (float)n, uv.y * (float)n};
    const float fx0 = floorf(UV.x - 0.5f), fy0 = floorf(UV.y - 0.5f);
    const F2 f = {UV.x - (fx0 + 0.5f), UV.y - (fy0 + 0.5f)};
    const F2 f2 = {f.x * f.x, f.y * f.y};
    const F2 f3v = {f2.x * f.x, f2.y * f.y};
    const F2 w1 = {f3v.x * -2.0f + f2.x * 3.0f, f3v.y * -2.0f + f2.y * 3.0f};
    const F2 w0 = {1.0f - w1.x, 1.0f - w1.y};
    const int t0x = (int)fx0, t0y = (int)fy0;
    const int xa = wrap_repeat(t0x, n), xb = wrap_repeat(t0x + 1, n);
    const int ya = wrap_repeat(t0y, n), yb = wrap_repeat(t0y + 1, n);
    const float wt[4] = {w0.x * w0.y, w1.x * w0.y, w0.x * w1.y, w1.x * w1.y};
    const F4 s0 = load_u16x4(tex, base + (uint32_t)(ya * n + xa));
    const F4 s1 = load_u16x4(tex, base + (uint32_t)(ya * n + xb));
    const F4 s2 = load_u16x4(tex, base + (uint32_t)(yb * n + xa));
    const F4 s3 = load_u16x4(tex, base + (uint32_t)(yb * n + xb));
    F4 o = {0.0f, 0.0f, 0.0f, 0.0f};
    float sw = 0.0f;
    const F4 s[4] = {s0, s1, s2, s3};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        sw += wt[i];
        o.x += s[i].x * wt[i];
        o.y += s[i].y * wt[i];
        o.z += s[i].z * wt[i];
        o.w += s[i].w * wt[i];
    }
    o.x /= sw; o.y /= sw; o.z /= sw; o.w += sw;  // Float4::operator/= (linearMath.h:433)
    return o;
}

RT_DEV F4 sample_lod(const uint2* tex, F2 uv, float lod) {
    const float low = floorf(lod);
    const float fr = lod - low;
    int lo = (int)low, hi = lo + 1;
    lo = lo < 0 ? 0 : lo > kTexLevels - 1 ? kTexLevels - 1 : lo;
    hi = hi < 0 ? 0 : hi > kTexLevels - 1 ? kTexLevels - 1 : hi;
    const F4 a = bicubic_tex(tex, lo, uv), b = bicubic_tex(tex, hi, uv);
    const float ia = 1.0f - fr;
    return F4{a.x * ia + b.x * fr, a.y * ia + b.y * fr, a.z * ia + b.z * fr, a.w * ia + b.w * fr};
}

// ------------------------------------------------------------------ environment
RT_DEV F3 equal_area_map(float u, float v) {
    const float z = v;
    const float r = __builtin_sqrtf(1.0f - v * v);
    const float phi = kTwoPi * u;
    return f3(r * rt_cosf(phi), z, r * rt_sinf(phi));
}

RT_DEV void localize_sample(F3 n, F3& u, F3& v) {
    F3 w = f3(1.0f, 0.0f, 0.0f);
    if (fabsf(n.x) > 0.707f) w = f3(0.0f, 1.0f, 0.0f);
    u = cross(n, w);
    v = cross(n, u);
}

RT_DEV F3 equal_area_map_cone(F3 sunDir, F3 t, F3 b, float u, float v, float cosThetaMax) {
    const float cosTheta = (1.0f - u) + u * cosThetaMax;
    const float sinTheta = __builtin_sqrtf(1.0f - cosTheta * cosTheta);
    const float phi = v * kTwoPi;
    const F3 c = f3(rt_cosf(phi) * sinTheta, cosTheta, rt_sinf(phi) * sinTheta);
    return f3(inner3(t.x, c.x, sunDir.x, c.y, b.x, c.z), inner3(t.y, c.x, sunDir.y, c.y, b.y, c.z),
              inner3(t.z, c.x, sunDir.z, c.y, b.z, c.z));
}

RT_DEV F3 equal_area_map_cone(F3 sunDir, float u, float v, float cosThetaMax) {
    F3 t, b;
    localize_sample(sunDir, t, b);
    return equal_area_map_cone(sunDir, t, b, u, v, cosThetaMax);
}

// SampleBicubicSmoothStep over a float4 env buffer.  sky: RepeatX/ClampY on 512x256.
// sun: the reference reads its 32x32 sun image from a 512x256 surface with the default
// (no-op) boundary and surface clamp at the low edge; texels beyond the 32x32 are zero.
template <bool kSun>
RT_DEV F3 bicubic_env(const float4* buf, F2 uv) {
    const int W = kSun ? kSunW : kSkyW, H = kSun ? kSunH : kSkyH;
    const F2 UV = {uv.x * (float)W, uv.y * (float)H};
    const float fx0 = floorf(UV.x - 0.5f), fy0 = floorf(UV.y - 0.5f);
    const F2 f = {UV.x - (fx0 + 0.5f), UV.y - (fy0 + 0.5f)};
    const F2 f2 = {f.x * f.x, f.y * f.y};
    const F2 f3v = {f2.x * f.x, f2.y * f.y};
    const F2 w1 = {f3v.x * -2.0f + f2.x * 3.0f, f3v.y * -2.0f + f2.y * 3.0f};
    const F2 w0 = {1.0f - w1.x, 1.0f - w1.y};
    const int t0x = (int)fx0, t0y = (int)fy0;
    const int sx[4] = {t0x, t0x + 1, t0x, t0x + 1}, sy[4] = {t0y, t0y, t0y + 1, t0y + 1};
    const float wt[4] = {w0.x * w0.y, w1.x * w0.y, w0.x * w1.y, w1.x * w1.y};
    F3 o = f3(0.0f);
    float sw = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        sw += wt[i];
        int x = sx[i], y = sy[i];
        F3 c;
        if (kSun) {
            if (x < 0) x = 0;
            if (y < 0) y = 0;
            c = (x >= kSunW || y >= kSunH) ? f3(0.0f) : f3_4(buf[y * kSunW + x]);
        } else {
            if (x >= kSkyW) x %= kSkyW;
            if (x < 0) x = kSkyW - (-x) % kSkyW;
            if (x >= kSkyW) x = kSkyW - 1;
            if (y >= kSkyH) y = kSkyH - 1;
            if (y < 0) y = 0;
            c = f3_4(buf[y * kSkyW + x]);
        }
        o = o + c * wt[i];
    }
    return o / sw;
}

RT_DEV F3 env_light(const PathTraceParams& P, F3 sunDir, F3 rd) {
    F3 color;
    {
        const F2 uv = {div_two_pi(rt_atan2f(-rd.z, -rd.x)) + 0.5f, fmx(rd.y, 0.05f)};
        const F3 sky = bicubic_env<false>(P.skyBuffer, uv);
        const F3 mist = f3(0.2f);
        const float w = clampf((rd.y + 0.4f) * (1.0f / 0.5f));
        color = f3(0.0f) + (mist + (w * w * (3.0f - 2.0f * w)) * (sky - mist));
    }
    // EqualAreaMapCone inverse (sky.cuh:64-87); the sun frame (t, b) = LocalizeSample(sunDir) is
    // per frame (P.sunT / P.sunB), and c.x is needed only inside the sun cone
    const float cosMax = P.cosThetaMax;
    const float cosTheta = inner3(sunDir.x, rd.x, sunDir.y, rd.y, sunDir.z, rd.z);
    if (cosTheta < cosMax) return color;
    const F3 c = f3(inner3(P.sunT[0], rd.x, P.sunT[1], rd.y, P.sunT[2], rd.z), cosTheta, 0.0f);
    const float u = (1.0f - cosTheta) / P.oneMinusCosThetaMax;  // (1 - cosMax), from the host
    const float sinTheta = __builtin_sqrtf(1.0f - cosTheta * cosTheta);
    if (sinTheta < 1e-5f || (c.x / sinTheta) < -1.0f || (c.x / sinTheta) > 1.0f) return color;
    const float v = rt_acosf(c.x / sinTheta) * kInvTwoPi;
    return color + bicubic_env<true>(P.sunBuffer, F2{u, v});
}

RT_DEV int cdf_search(const float* a, int left, int right, float target) {
    while (right - left > 1) {
        const int mid = (left + right) / 2;
        if (a[mid] < target) left = mid;
        else right = mid;
    }
    return left;
}

// BinarySearch (light.cuh:9-31) with its first probes read from the LDS heap `tree` (see
// kSkyTreeNodes): identical probes, identical result, fewer dependent global loads
RT_DEV int cdf_search_tree(const float* a, int right, float target, const float* tree, int nodes) {
    int left = 0, j = 1;
    while (right - left > 1) {
        const int mid = (left + right) / 2;
        const float v = j < nodes ? tree[j] : a[mid];
        if (v < target) {
            left = mid;
            j = 2 * j + 1;
        } else {
            right = mid;
            j = 2 * j;
        }
    }
    return left;
}

RT_DEV void sample_light(const PathTraceParams& P, F3 sunDir, F3& dir, float& pdf, int& lightIdx, float r0, float r1,
                         const float* skyTree, const float* sunTree) {
    // pSky = totalSky / (totalSky + totalSun) and the CDF totals, per frame (sky.hip k_light_select)
    const float pSky = P.lightSel[0], maxSky = P.lightSel[1], maxSun = P.lightSel[2], sunDen = P.lightSel[3];
    if (pSky > r1) {
        const int idx = cdf_search_tree(P.skyCdf, kSkySize - 2, r0 * maxSky, skyTree, kSkyTreeNodes) + 1;
        float p = (P.skyCdf[idx] - P.skyCdf[idx - 1]) / maxSky;
        p = div_two_pi(p * kSkySize);
        const float u = ((float)(idx % kSkyW) + 0.5f) / kSkyW;
        const float v = ((float)(idx / kSkyW) + 0.5f) / kSkyH;
        dir = equal_area_map(u, v);
        pdf = p * 1.0f * pSky;
    } else {
        const int idx = cdf_search_tree(P.sunCdf, kSunSize - 2, r0 * maxSun, sunTree, kSunTreeNodes) + 1;
        float p = (P.sunCdf[idx] - P.sunCdf[idx - 1]) / maxSun;
        p = p * kSunSize / sunDen;  // kTwoPi * (1 - cosThetaMax)
        const float u = ((float)(idx % kSunW) + 0.5f) / kSunW;
        const float v = ((float)(idx / kSunW) + 0.5f) / kSunH;
        dir = equal_area_map_cone(sunDir, f3(P.sunT[0], P.sunT[1], P.sunT[2]), f3(P.sunB[0], P.sunB[1], P.sunB[2]), u,
                                  v, P.cosThetaMax);
        pdf = p * 1.0f;
    }
    lightIdx = kEnvLightId;
}

// ------------------------------------------------------------------ BSDFs
RT_DEV void lambertian_sample(F2 u, F3& wo, F3 n) {
    const float r = __builtin_sqrtf(u.x);
    const float theta = kTwoPi * u.y;
    const F2 d = {r * rt_cosf(theta), r * rt_sinf(theta)};
    const float z = __builtin_sqrtf(max1f(0.0f, 1.0f - d.x * d.x - d.y * d.y));
    F3 uu, vv;
    localize_sample(n, uu, vv);
    wo = normalize(d.x * uu + d.y * vv + z * n);
}

RT_DEV F3 fresnel_schlick(F3 F0, float cosTheta) {
    const float e = 1.0f - cosTheta;
    const float e2 = e * e;
    return F0 + (f3(1.0f) - F0) * (e2 * e2 * e);
}

RT_DEV void microfacet_terms(F3 wo, F3 wi, F3 wh, F3 wn, F3 F0, F3 albedo, float alpha2, F3& brdfOverPdf, F3& brdf,
                             float& pdf) {
    const float cWoWh = fmx(kSafeCos, dot(wh, wo));
    const F3 F = fresnel_schlick(F0, cWoWh);
    const float cWo = clampf(dot(wo, wn), kSafeCos, 1.0f - kSafeCos);
    const float cWi = fmx(kSafeCos, dot(wi, wn));
    const float tWo = __builtin_sqrtf(1.0f - cWo * cWo) / cWo;
    const float G = 1.0f / (1.0f + (__builtin_sqrtf(1.0f + alpha2 * tWo * tWo) - 1.0f) / 2.0f);
    const float cWh = fmx(kSafeCos, dot(wh, wn));
    const float c2 = cWh * cWh;
    const float t2 = (1.0f - c2) / c2;
    const float e = t2 / alpha2 + 1.0f;
    const float D = 1.0f / (kPi * (alpha2 * c2 * c2) * (e * e));
    brdf = (albedo * F) * (D * G) / (4.0f * cWo * cWi);
    pdf = (D * cWh) / (4.0f * cWoWh);
    brdfOverPdf = (albedo * F) * (G * cWoWh) / (cWh * cWo);
}

RT_DEV F3 reflect3(F3 i, F3 n) { return i - 2.0f * n * dot(n, i); }

RT_DEV F3 ggx_normal(F2 r, float alpha2, F3 normal) {
    const float cosTheta = 1.0f / __builtin_sqrtf(1.0f + alpha2 * r.x / (1.0f - r.x));
    const float sinTheta = __builtin_sqrtf(1.0f - cosTheta * cosTheta);
    const float phi = kTwoPi * r.y;
    const F3 sl = f3(sinTheta * rt_cosf(phi), cosTheta, sinTheta * rt_sinf(phi));
    F3 t, b;
    localize_sample(normal, t, b);
    return normalize(sl.x * t + sl.z * b + sl.y * normal);
}

}  // namespace rtd
