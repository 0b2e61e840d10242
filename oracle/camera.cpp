// ORACLE (test infrastructure only; see ocommon.h) — camera, primary rays, blue noise,
// smooth normals, rtmath probes.
//
// Restates:
//   Camera::update                  kernel.cuh:103-121
//   GenerateRay / GetRayConeWidth   raygen.cuh:7-63, ConcentricSampleDisk bsdf.cuh:9-34
//   blue-noise sampler              blueNoiseRandGen.h:113-146 (OPTIMIZED_BLUE_NOISE_SPP 4)
//   GenerateSmoothNormals x2        kernel.cu:228-257, 313-327
#include <cstring>
#include <vector>

#include "oracle.h"
#include "ocommon.h"
#include "opath.h"

namespace orc {

void camera_update(const OrcCamera& in, Camera& c) {
    c.pos = f3(in.pos[0], in.pos[1], in.pos[2]);
    c.yaw = in.yaw;
    c.pitch = in.pitch;
    c.focal = in.focal;
    c.aperture = in.aperture;
    c.res = F2{in.resolution[0], in.resolution[1]};
    c.fov.x = in.fovX;
    c.dir = f3(rt_sinf(c.yaw) * rt_cosf(c.pitch), rt_sinf(c.pitch), rt_cosf(c.yaw) * rt_cosf(c.pitch));
    c.invRes = F2{1.0f / c.res.x, 1.0f / c.res.y};
    c.fov.y = c.fov.x / c.res.x * c.res.y;
    c.tanHalfFov = F2{rt_tanf(c.fov.x / 2), rt_tanf(c.fov.y / 2)};
    F3 upv = f3(0.0f, 1.0f, 0.0f);
    c.left = normalize(cross(upv, c.dir));
    c.up = normalize(cross(c.dir, c.left));
    c.adjustedFront = c.dir * c.focal;
    c.adjustedLeft = c.left * c.tanHalfFov.x * c.focal;
    c.adjustedUp = c.up * c.tanHalfFov.y * c.focal;
    c.apertureLeft = c.left * c.aperture;
    c.apertureUp = c.up * c.aperture;
}

float bluenoise(const uint8_t* tables, int px, int py, int sampleIdx, int dim) {
    const uint8_t* sobol = tables;
    const uint8_t* scr = tables + 256 * 256;
    const uint8_t* rnk = scr + 128 * 128 * 8;
    px &= 127;
    py &= 127;
    sampleIdx &= 255;
    int ranked = sampleIdx ^ rnk[dim + (px + py * 128) * 8];
    int value = sobol[dim + ranked * 256];
    value = value ^ scr[(dim % 8) + (px + py * 128) * 8];
    return ((float)value + 0.5f) / 256.0f;
}

F2 concentric_disk(F2 u) {
    F2 o = {2.0f * u.x - 1.0f, 2.0f * u.y - 1.0f};
    if (fabsf(o.x) < 1e-10f && fabsf(o.y) < 1e-10f) return F2{0.0f, 0.0f};
    float theta, r;
    if (fabsf(o.x) > fabsf(o.y)) {
        r = o.x;
        theta = kPiOver4 * (o.y / o.x);
    } else {
        r = o.y;
        theta = kPiOver2 - kPiOver4 * (o.x / o.y);
    }
    return F2{rt_cosf(theta) * r, rt_sinf(theta) * r};
}

void generate_ray(const Camera& c, int ix, int iy, F2 pix, F2 ap, F3& orig, F3& dir, F3& centerDir, F2& sampleUv) {
    F2 uv = {((float)ix + pix.x) * c.invRes.x, ((float)iy + pix.y) * c.invRes.y};
    F2 uvc = {((float)ix + 0.5f) * c.invRes.x, ((float)iy + 0.5f) * c.invRes.y};
    sampleUv = uv;
    uv = F2{uv.x * -2.0f + 1.0f, uv.y * -2.0f + 1.0f};
    uvc = F2{uvc.x * -2.0f + 1.0f, uvc.y * -2.0f + 1.0f};
    F3 p = c.adjustedFront + c.adjustedLeft * uv.x + c.adjustedUp * uv.y;
    F3 pc = c.adjustedFront + c.adjustedLeft * uvc.x + c.adjustedUp * uvc.y;
    F2 d = concentric_disk(ap);
    F3 pa = d.x * c.apertureLeft + d.y * c.apertureUp;
    orig = c.pos + pa;
    dir = normalize(p - pa);
    centerDir = normalize(pc);
}

float ray_cone_width(const Camera& c, int ix, int iy) {
    F2 pcen = {((float)ix + 0.5f) - c.res.x / 2, ((float)iy + 0.5f) - c.res.y / 2};
    F2 poff = {copysignf(0.5f, pcen.x), copysignf(0.5f, pcen.y)};
    F2 uvn = {(pcen.x - poff.x) * c.invRes.x * 2, (pcen.y - poff.y) * c.invRes.y * 2};
    F2 uvf = {(pcen.x + poff.x) * c.invRes.x * 2, (pcen.y + poff.y) * c.invRes.y * 2};
    F2 hf = {rt_tanf(c.fov.x / 2), rt_tanf(c.fov.y / 2)};
    F2 pn = {uvn.x * hf.x, uvn.y * hf.y};
    F2 pf = {uvf.x * hf.x, uvf.y * hf.y};
    float an = rt_atanf(sqrtf(pn.x * pn.x + pn.y * pn.y));
    float af = rt_atanf(sqrtf(pf.x * pf.x + pf.y * pf.y));
    return af - an;
}

}  // namespace orc

using namespace orc;

extern "C" float orc_bluenoise(const uint8_t* tables, int px, int py, int sampleIdx, int dim) {
    return bluenoise(tables, px, py, sampleIdx, dim);
}

extern "C" void orc_primary_rays(const OrcCamera* cam, uint32_t W, uint32_t H, int frameNum, const uint8_t* bn,
                                 float* rays, float* coneSpread) {
    Camera c;
    camera_update(*cam, c);
    for (uint32_t y = 0; y < H; ++y)
        for (uint32_t x = 0; x < W; ++x) {
            int s = frameNum * 4 + 0;
            F2 pix = {bluenoise(bn, (int)x, (int)y, s, 0), bluenoise(bn, (int)x, (int)y, s, 1)};
            F2 ap = {bluenoise(bn, (int)x, (int)y, s, 2), bluenoise(bn, (int)x, (int)y, s, 3)};
            F3 o, d, cd;
            F2 suv;
            generate_ray(c, (int)x, (int)y, pix, ap, o, d, cd, suv);
            float* r = rays + ((size_t)y * W + x) * 6;
            r[0] = o.x; r[1] = o.y; r[2] = o.z; r[3] = d.x; r[4] = d.y; r[5] = d.z;
            if (coneSpread) coneSpread[(size_t)y * W + x] = ray_cone_width(c, (int)x, (int)y);
        }
}

extern "C" void orc_smooth_normals(const float* vertices, uint32_t nverts, const uint32_t* indices,
                                   uint32_t triCountPadded, float* normals) {
    const F3* V = (const F3*)vertices;
    F3* N = (F3*)normals;
    for (uint32_t k = 0; k < nverts; ++k) N[k] = f3(0.0f);
    auto angle_between = [](F3 a, F3 b) { return rt_acosf(dot(a, b) / sqrtf(length2(a) * length2(b))); };
    for (int pass = 0; pass < 2; ++pass)
        for (uint32_t t = 0; t < triCountPadded; ++t) {
            uint32_t i0 = indices[3 * t], i1 = indices[3 * t + 1], i2 = indices[3 * t + 2];
            F3 v0 = V[i0], v1 = V[i1], v2 = V[i2];
            F3 pnma = cross(v2 - v0, v2 - v1) / 2.0f;
            float w0 = angle_between(v2 - v0, v1 - v0);
            float w1 = angle_between(v2 - v1, v0 - v1);
            float w2 = angle_between(v0 - v2, v1 - v2);
            N[i0] = N[i0] + pnma * w0;
            N[i1] = N[i1] + pnma * w1;
            N[i2] = N[i2] + pnma * w2;
        }
}

extern "C" float orc_rtmath(int fn, float x, float y) {
    switch (fn) {
        case 0: return rt_sinf(x);
        case 1: return rt_cosf(x);
        case 2: return rt_tanf(x);
        case 3: return rt_atanf(x);
        case 4: return rt_atan2f(x, y);
        case 5: return rt_acosf(x);
        case 6: return rt_asinf(x);
        case 7: return rt_expf(x);
        case 8: return rt_exp2f(x);
        case 9: return rt_logf(x);
        case 10: return rt_log2f(x);
        case 11: return rt_powf(x, y);
        case 12: return rt_log2f_div(x);
        case 13: return rt_powf_div(x, y);
        default: return 0.0f;
    }
}

// rtmath.h over arrays with one second argument (the denoiser's uniform sigmas): 0 rt_powf(x, y),
// 1 rt_expf(x), 2 rt_div_rcp(x, y, c) — the checker of the GPU's packed-pair forms
// (tests/test_gpu_pk_math.py)
extern "C" void orc_rtmath_n(int fn, const float* x, float y, float c, float* out, size_t n) {
    for (size_t i = 0; i < n; ++i)
        out[i] = fn == 0 ? rt_powf(x[i], y) : fn == 1 ? rt_expf(x[i]) : rt_div_rcp(x[i], y, c);
}

// the half conversions of the G-buffers and denoise buffers (rtmath.h rt_f2h / rt_h2f, host
// integer restatements), over arrays: tests/test_gpu_half.py checks the GPU's hardware conversions
// against them
extern "C" void orc_f2h_n(const float* f, uint16_t* h, size_t n) {
    for (size_t i = 0; i < n; ++i) h[i] = rt_f2h(f[i]);
}
extern "C" void orc_h2f_n(const uint16_t* h, float* f, size_t n) {
    for (size_t i = 0; i < n; ++i) f[i] = rt_h2f(h[i]);
}

// rt_unorm16 against the IEEE division it replaces, over every 16-bit value: the count of mismatches
extern "C" int orc_unorm16_mismatches() {
    int bad = 0;
    for (uint32_t x = 0; x < 65536u; ++x) {
        volatile float d = 65535.0f;  // a real division, not a constant-folded product
        const float ref = (float)x / d, got = rt_unorm16(x);
        if (memcmp(&ref, &got, 4) != 0) ++bad;
    }
    return bad;
}

// the shading path's x / d by x * RN(1/d) and one fma correction (pt_common.h div_by_const) against
// the IEEE division, over every stride-th float bit pattern with finite |x| >= 2^-100: mismatches
extern "C" long orc_div_const_mismatches(float d, uint32_t stride) {
    volatile float dv = d;
    const float c = 1.0f / dv;
    long bad = 0;
    for (uint64_t u = 0; u < (1ull << 32); u += stride) {
        const float x = rtm::bits_to_float((uint32_t)u);
        const float ax = fabsf(x);
        if (!(ax >= 0x1p-100f && ax <= 0x1.fffffep127f)) continue;
        const float q = x * c, got = fmaf(fmaf(-q, d, x), c, q), ref = x / dv;
        if (memcmp(&ref, &got, 4) != 0) ++bad;
    }
    return bad;
}

// rt_div_rcp(x, d, RN(1/d)) (the denoiser's depth weights, rtmath.h) against the IEEE division,
// over every stride-th float bit pattern x with x = 0 or 2^-30 <= |x| <= 2^30, plus +-inf and NaN:
// mismatches (NaN compared as NaN)
extern "C" long orc_div_rcp_mismatches(float d, uint32_t stride) {
    volatile float dv = d;
    const float c = 1.0f / dv;
    long bad = 0;
    auto check = [&](float x) {
        const float ref = x / dv, got = rt_div_rcp(x, d, c);
        if (memcmp(&ref, &got, 4) != 0 && !(ref != ref && got != got)) ++bad;
    };
    for (uint64_t u = 0; u < (1ull << 32); u += stride) {
        const float x = rtm::bits_to_float((uint32_t)u);
        const float ax = fabsf(x);
        if (ax >= 0x1p-30f && ax <= 0x1p30f) check(x);
    }
    for (float x : {0.0f, -0.0f, INFINITY, -INFINITY, NAN}) check(x);
    return bad;
}

// UpdateFrame's dynamic resolution (kernel.cu:77-100), restated: outside the targetFps +-2 band
// the width is scaled (int *= float) by sqrt(target frame time / dt); it is then snapped to the
// nearest multiple of 16 (ties of 8 round up), clamped by clampi to [minW, maxW], and the height
// is (w / 16) * 9.
extern "C" void orc_dynamic_resolution(int w, float dt, float targetFps, int minW, int maxW, int maxH, int* outW,
                                       int* outH) {
    const float high = 1000.0f / (targetFps - 2), low = 1000.0f / (targetFps + 2);
    if (high < dt || low > dt) {
        float ratio = (1000.0f / targetFps) / dt;
        ratio = sqrtf(ratio);
        w = (int)((float)w * ratio);
    }
    const int rem = w % 16;
    w = rem < 8 ? w - rem : w + (16 - rem);
    w = w < minW ? minW : (w > maxW ? maxW : w);
    const int h = (w / 16) * 9;
    *outW = w;
    *outH = h > maxH ? maxH : h;
}
