// pt_common.h — per-pixel sampling helpers shared by the primary-ray and path-trace kernels.
//
//   blue-noise sampler   blueNoiseRandGen.h:113-146 (Heitz 2019, OPTIMIZED_BLUE_NOISE_SPP 4)
//   ConcentricSampleDisk bsdf.cuh:9-34
//   GenerateRay          raygen.cuh:7-38
//   GetRayConeWidth      raygen.cuh:45-63
#pragma once
#include "bvh_kernels.h"
#include "rt_device.h"

namespace rtd {

constexpr float kPiOver4 = 0.7853981633974483096156608458198757210492f;   // linearMath.h:11-20
constexpr float kPiOver2 = 1.5707963267948966192313216916397514420985f;
constexpr float kPi = 3.1415926535897932384626422832795028841971f;
constexpr float kTwoPi = 6.2831853071795864769252867665590057683943f;

// x / kPi and x / kTwoPi, correctly rounded: x * RN(1/d) corrected by one fma step (Markstein).
// Equal to the IEEE quotient for every finite |x| >= 2^-100, checked exhaustively over all floats
// (tools/div_exhaustive.c; tests/test_rtmath.py samples it); smaller, infinite and NaN x take the
// division.  Three instructions instead of the division's ten on the shading path.
RT_DEV float div_by_const(float x, float d, float c) {
    const float q = x * c;
    const float fast = __builtin_fmaf(__builtin_fmaf(-q, d, x), c, q);
    const float ax = __builtin_fabsf(x);
    return (ax >= 0x1p-100f && ax <= 0x1.fffffep127f) ? fast : x / d;
}
RT_DEV float div_pi(float x) { return div_by_const(x, kPi, 0x1.45f306p-2f); }      // c = RN(1 / kPi)
RT_DEV float div_two_pi(float x) { return div_by_const(x, kTwoPi, 0x1.45f306p-3f); }  // c = RN(1 / kTwoPi)

// tables: sobol[256*256] | scrambling[128*128*8] | ranking[128*128*8]
RT_DEV float bluenoise(const uint8_t* tables, int px, int py, int sampleIdx, int dim) {
    const uint8_t* sobol = tables;
    const uint8_t* scr = tables + 256 * 256;
    const uint8_t* rnk = scr + 128 * 128 * 8;
    px &= 127;
    py &= 127;
    sampleIdx &= 255;
    const int cell = (px + py * 128) * 8;
    const int ranked = sampleIdx ^ (int)rnk[dim + cell];
    int value = sobol[dim + ranked * 256];
    value = value ^ (int)scr[(dim % 8) + cell];
    return ((float)value + 0.5f) / 256.0f;
}

// The same lookup split into its per-pixel half (ranking + scrambling bytes of dims 0..3, one
// dword each) and its per-sample half against an LDS copy of sobol dims 0..3 (row r at [r]).
// bn_value(...) == bluenoise(...) for dim < 4.
struct BnPixel {
    uint32_t rnk, scr;
};

RT_DEV BnPixel bn_pixel(const uint8_t* tables, int px, int py) {
    const uint8_t* scr = tables + 256 * 256;
    const uint8_t* rnk = scr + 128 * 128 * 8;
    const int cell = ((px & 127) + (py & 127) * 128) * 8;
    return BnPixel{*(const uint32_t*)(rnk + cell), *(const uint32_t*)(scr + cell)};
}

RT_DEV float bn_value(const uint32_t* sobolRows, BnPixel b, int sampleIdx, int dim) {
    const int sh = 8 * dim;
    const int ranked = (sampleIdx & 255) ^ (int)((b.rnk >> sh) & 255u);
    const int value = (int)((sobolRows[ranked] >> sh) & 255u) ^ (int)((b.scr >> sh) & 255u);
    return ((float)value + 0.5f) / 256.0f;
}

// workgroup-cooperative copy of sobol dims 0..3 into LDS (caller syncs)
RT_DEV void bn_stage_sobol(const uint8_t* tables, uint32_t* sobolRows, int tid, int nthreads) {
    for (int r = tid; r < 256; r += nthreads) sobolRows[r] = *(const uint32_t*)(tables + r * 256);
}

RT_DEV F2 concentric_disk(F2 u) {
    const F2 o = {2.0f * u.x - 1.0f, 2.0f * u.y - 1.0f};
    if (fabsf(o.x) < 1e-10f && fabsf(o.y) < 1e-10f) return F2{0.0f, 0.0f};
    // the two branches as selects around one division (a wave's lanes take both; each lane's
    // operations are the branch's own)
    const bool xMajor = fabsf(o.x) > fabsf(o.y);
    const float r = xMajor ? o.x : o.y;
    const float q = (xMajor ? o.y : o.x) / r;
    const float theta = xMajor ? kPiOver4 * q : kPiOver2 - kPiOver4 * q;
    float sn, cs;
    rt_sincosf(theta, &sn, &cs);
    return F2{cs * r, sn * r};
}

RT_DEV F3 load3(const float* a) { return f3(a[0], a[1], a[2]); }

// the pixel-centre direction of GenerateRay (raygen.cuh:7-38): the same for every sample
RT_DEV F3 center_dir(const TraceCamera& c, int ix, int iy) {
    F2 uvc = {((float)ix + 0.5f) * c.invRes[0], ((float)iy + 0.5f) * c.invRes[1]};
    uvc = F2{uvc.x * -2.0f + 1.0f, uvc.y * -2.0f + 1.0f};
    const F3 pc = load3(c.adjustedFront) + load3(c.adjustedLeft) * uvc.x + load3(c.adjustedUp) * uvc.y;
    return normalize(pc);
}

// GenerateRay without the centre direction
RT_DEV void generate_ray_jittered(const TraceCamera& c, int ix, int iy, F2 pix, F2 ap, F3& orig, F3& dir,
                                  F2& sampleUv) {
    F2 uv = {((float)ix + pix.x) * c.invRes[0], ((float)iy + pix.y) * c.invRes[1]};
    sampleUv = uv;
    uv = F2{uv.x * -2.0f + 1.0f, uv.y * -2.0f + 1.0f};
    const F3 p = load3(c.adjustedFront) + load3(c.adjustedLeft) * uv.x + load3(c.adjustedUp) * uv.y;
    const F2 d = concentric_disk(ap);
    const F3 pa = d.x * load3(c.apertureLeft) + d.y * load3(c.apertureUp);
    orig = load3(c.pos) + pa;
    dir = normalize(p - pa);
}

RT_DEV void generate_ray(const TraceCamera& c, int ix, int iy, F2 pix, F2 ap, F3& orig, F3& dir, F3& centerDir,
                         F2& sampleUv) {
    F2 uv = {((float)ix + pix.x) * c.invRes[0], ((float)iy + pix.y) * c.invRes[1]};
    F2 uvc = {((float)ix + 0.5f) * c.invRes[0], ((float)iy + 0.5f) * c.invRes[1]};
    sampleUv = uv;
    uv = F2{uv.x * -2.0f + 1.0f, uv.y * -2.0f + 1.0f};
    uvc = F2{uvc.x * -2.0f + 1.0f, uvc.y * -2.0f + 1.0f};
    const F3 front = load3(c.adjustedFront), left = load3(c.adjustedLeft), up = load3(c.adjustedUp);
    const F3 p = front + left * uv.x + up * uv.y;
    const F3 pc = front + left * uvc.x + up * uvc.y;
    const F2 d = concentric_disk(ap);
    const F3 pa = d.x * load3(c.apertureLeft) + d.y * load3(c.apertureUp);
    orig = load3(c.pos) + pa;
    dir = normalize(p - pa);
    centerDir = normalize(pc);
}

}  // namespace rtd
