// ORACLE (test infrastructure only; see ocommon.h) — sky/sun model, CDF scan, sun direction.
//
// Restates:
//   UpdateFrame sun direction          kernel.cu:119-123 (axis-angle quaternion rotate, linearMath.h:650-716)
//   UpdateSkyState / GetFittingData    sky.cuh:90-146
//   GetSkyRadiance / GetSunRadiance    sky.cuh:165-278 (incl. the double-precision sub-expressions)
//   Sky / SkySun kernels               sky.cuh:280-320, EqualAreaMap(Cone) sky.cuh:33-62
//   Scan (Blelloch, blocks + sums)     scan.cuh:31-298 — the intended inclusive scan; see DESIGN.md
//   draw's regeneration block          kernel.cu:289-308
#include <vector>

#include "oracle.h"
#include "ocommon.h"
#include "opath.h"

namespace orc {

struct Quat { F3 v; float w; };
static Quat qmul(const Quat& p, const Quat& q) {
    Quat r;
    r.v = p.w * q.v + q.w * p.v + cross(p.v, q.v);
    r.w = p.w * q.w - dot(p.v, q.v);
    return r;
}

F3 sun_direction(float timeOfDay, float sunAxisAngle) {
    F3 axis = normalize(f3(0.0f, rt_cosf(sunAxisAngle * kPiOver180), rt_sinf(sunAxisAngle * kPiOver180)));
    float angle = fmodf(timeOfDay * kPi, kTwoPi);
    F3 v = cross(f3(0.0f, 1.0f, 0.0f), axis);
    // Quat::axisAngle(axis, angle) = (axis.normalized() * sin(angle/2), cos(angle/2))
    Quat q = {normalize(axis) * rt_sinf(angle / 2), rt_cosf(angle / 2)};
    Quat qc = {-q.v, q.w};
    Quat pv = {v, 0.0f};
    Quat r = qmul(qmul(q, pv), qc);
    return normalize(r.v);
}

static float fitting(const float* m, float s, int i) {
    return (rt_powf(1.0f - s, 5.0f) * m[i] + 5.0f * rt_powf(1.0f - s, 4.0f) * s * m[i + 9] +
            10.0f * rt_powf(1.0f - s, 3.0f) * rt_powf(s, 2.0f) * m[i + 18] +
            10.0f * rt_powf(1.0f - s, 2.0f) * rt_powf(s, 3.0f) * m[i + 27] +
            5.0f * (1.0f - s) * rt_powf(s, 4.0f) * m[i + 36] + rt_powf(s, 5.0f) * m[i + 45]);
}
static float fitting2(const float* m, float s) {
    return (rt_powf(1.0f - s, 5.0f) * m[0] + 5.0f * rt_powf(1.0f - s, 4.0f) * s * m[1] +
            10.0f * rt_powf(1.0f - s, 3.0f) * rt_powf(s, 2.0f) * m[2] +
            10.0f * rt_powf(1.0f - s, 2.0f) * rt_powf(s, 3.0f) * m[3] + 5.0f * (1.0f - s) * rt_powf(s, 4.0f) * m[4] +
            rt_powf(s, 5.0f) * m[5]);
}

struct SkyState {
    float configs[90], radiances[10];
    const float* solar;   // 1800
    const float* limb;    // 60
    const float* cieX; const float* cieY; const float* cieZ;
};

static void sky_state(const F3& sunDir, const OrcSkyTables& t, SkyState& st) {
    float elevation = rt_acosf(sunDir.y);
    float se = rt_powf(elevation / (kPi / 2.0f), (1.0f / 3.0f));
    for (int ch = 0; ch < 10; ++ch) {
        for (int i = 0; i < 9; ++i) st.configs[ch * 9 + i] = fitting(t.skyDataSets + ch * 54, se, i);
        st.radiances[ch] = fitting2(t.skyDataSetsRad + ch * 6, se);
    }
    st.solar = t.solarDatasets;
    st.limb = t.limbDarkeningDatasets;
    st.cieX = t.cieX; st.cieY = t.cieY; st.cieZ = t.cieZ;
}

// XyzToRgbSrgb (color.h:19-30): column-major Mat3 built from row-major literals
static F3 xyz_to_srgb(F3 c) {
    const float m00 = (float)3.2404542, m01 = (float)-1.5371385, m02 = (float)-0.4985314;
    const float m10 = (float)-0.9692660, m11 = (float)1.8760108, m12 = (float)0.0415560;
    const float m20 = (float)0.0556434, m21 = (float)-0.2040259, m22 = (float)1.0572252;
    return f3(inner3(m00, c.x, m01, c.y, m02, c.z), inner3(m10, c.x, m11, c.y, m12, c.z),
              inner3(m20, c.x, m21, c.y, m22, c.z));
}

static float clampf(float a, float lo, float hi) { return a < lo ? lo : a > hi ? hi : a; }

static F3 sky_radiance(F3 raydir, F3 sunDir, const SkyState& st) {
    float theta = rt_acosf(raydir.y);
    float gamma = rt_acosf(clampf(dot(raydir, sunDir), -1, 1));
    F3 xyz = f3(0.0f);
    for (int ch = 0; ch < 10; ++ch) {
        const float* c = st.configs + ch * 9;
        const float expM = rt_expf(c[4] * gamma);
        const float rayM = rt_cosf(gamma) * rt_cosf(gamma);
        const float mieM = (1.0f + rt_cosf(gamma) * rt_cosf(gamma)) /
                           rt_powf((1.0f + c[8] * c[8] - 2.0f * c[8] * rt_cosf(gamma)), 1.5f);
        const float zenith = sqrtf(rt_cosf(theta));
        // (cos(theta) + 0.01) promotes to double; so does the left factor and the product
        double left = 1.0 + (double)c[0] * ORC_EXPD((double)c[1] / ((double)rt_cosf(theta) + 0.01));
        float right = c[2] + c[3] * expM + c[5] * rayM + c[6] * mieM + c[7] * zenith;
        float radianceInternal = (float)(left * (double)right);
        float radiance = radianceInternal * st.radiances[ch];
        xyz = xyz + radiance * f3(st.cieX[ch], st.cieY[ch], st.cieZ[ch]);
    }
    return xyz_to_srgb(xyz);
}

static F3 sun_radiance(F3 raydir, F3 sunDir, float sunAngle, const SkyState& st) {
    float gamma = rt_acosf(clampf(dot(raydir, sunDir), -1, 1));
    float elevation = (kPi / 2.0f) - rt_acosf(sunDir.y);
    const float solarRadius = sunAngle * kPi / 180.0f / 2.0f;
    const float sbs = 1.0f / ((sunAngle / 0.51f) * (sunAngle / 0.51f));
    F3 xyz = f3(0.0f);
    float srs = rt_sinf(solarRadius);
    float ar2 = 1.0f / (srs * srs);
    float sg = rt_sinf(gamma);
    float sc2 = 1.0f - ar2 * sg * sg;
    if (sc2 < 0.0f) sc2 = 0.0f;
    float sampleCosine = sqrtf(sc2);
    if (sampleCosine == 0.0f) return f3(0.0f);
    for (int ch = 0; ch < 10; ++ch) {
        const int pieces = 45, order = 4;
        int pos = (int)(rt_powf((float)(2.0 * (double)elevation / (double)kPi), (float)(1.0 / 3.0)) * pieces);
        if (pos > 44) pos = 44;
        const float break_x = (float)((double)rt_powf(((float)pos / (float)pieces), 3.0f) * ((double)kPi * 0.5));
        const float* coefs = st.solar + ch * 180 + (order * (pos + 1) - 1);
        float res = 0.0f;
        const float x = elevation - break_x;
        float x_exp = 1.0f;
        for (int i = 0; i < order; ++i) {
            res += x_exp * *coefs--;
            x_exp *= x;
        }
        float direct = res;
        const float* ld = st.limb + ch * 6;
        float dark = ld[0] + ld[1] * sampleCosine + ld[2] * rt_powf(sampleCosine, 2.0f) +
                     ld[3] * rt_powf(sampleCosine, 3.0f) + ld[4] * rt_powf(sampleCosine, 4.0f) +
                     ld[5] * rt_powf(sampleCosine, 5.0f);
        direct *= dark * sbs;
        xyz = xyz + direct * f3(st.cieX[ch], st.cieY[ch], st.cieZ[ch]);
    }
    return xyz_to_srgb(xyz);
}

F3 equal_area_map(float u, float v) {
    float z = v;
    float r = sqrtf(1.0f - v * v);
    float phi = kTwoPi * u;
    return f3(r * rt_cosf(phi), z, r * rt_sinf(phi));
}

void localize_sample(F3 n, F3& u, F3& v) {
    F3 w = f3(1.0f, 0.0f, 0.0f);
    if (fabsf(n.x) > 0.707f) w = f3(0.0f, 1.0f, 0.0f);
    u = cross(n, w);
    v = cross(n, u);
}

F3 equal_area_map_cone(F3 sunDir, float u, float v, float cosThetaMax) {
    float cosTheta = (1.0f - u) + u * cosThetaMax;
    float sinTheta = sqrtf(1.0f - cosTheta * cosTheta);
    float phi = v * kTwoPi;
    F3 t, b;
    localize_sample(sunDir, t, b);
    F3 c = f3(rt_cosf(phi) * sinTheta, cosTheta, rt_sinf(phi) * sinTheta);
    // Mat3(t, sunDir, b) * c, columns t, sunDir, b
    return f3(inner3(t.x, c.x, sunDir.x, c.y, b.x, c.z), inner3(t.y, c.x, sunDir.y, c.y, b.y, c.z),
              inner3(t.z, c.x, sunDir.z, c.y, b.z, c.z));
}

// Blelloch exclusive scan of n values in tree order (scan.cuh:31-137)
static void blelloch_exclusive(float* a, int n) {
    int offset = 1;
    for (int d = n >> 1; d > 0; d >>= 1) {
        for (int i = 0; i < d; ++i) {
            int ai = offset * (2 * i + 1) - 1, bi = offset * (2 * i + 2) - 1;
            a[bi] = a[bi] + a[ai];
        }
        offset *= 2;
    }
    a[n - 1] = 0.0f;
    for (int d = 1; d < n; d *= 2) {
        offset >>= 1;
        for (int i = 0; i < d; ++i) {
            int ai = offset * (2 * i + 1) - 1, bi = offset * (2 * i + 2) - 1;
            float t = a[ai];
            a[ai] = a[bi];
            a[bi] = a[bi] + t;
        }
    }
}

// Scan(in, out, tmp, size, blockSize, postfix) (scan.cuh:258-298); postfix 0: exclusive blocks
void scan_blocks(const float* in, float* out, int size, int blockSize, int postfix) {
    int blocks = size / blockSize;
    std::vector<float> sums(blocks), tmp(blockSize);
    for (int b = 0; b < blocks; ++b) {
        memcpy(tmp.data(), in + (size_t)b * blockSize, blockSize * 4);
        // block total = root of the up-sweep (same tree) — recomputed by scanning a copy
        std::vector<float> up(tmp);
        {
            int offset = 1;
            for (int d = blockSize >> 1; d > 0; d >>= 1) {
                for (int i = 0; i < d; ++i) {
                    int ai = offset * (2 * i + 1) - 1, bi = offset * (2 * i + 2) - 1;
                    up[bi] = up[bi] + up[ai];
                }
                offset *= 2;
            }
        }
        sums[b] = up[blockSize - 1];
        blelloch_exclusive(tmp.data(), blockSize);
        for (int i = 0; i < blockSize; ++i)
            out[(size_t)b * blockSize + i] = postfix ? tmp[i] + in[(size_t)b * blockSize + i] : tmp[i];
    }
    if (blocks > 1) {
        blelloch_exclusive(sums.data(), blocks);
        for (int b = 0; b < blocks; ++b)
            for (int i = 0; i < blockSize; ++i) out[(size_t)b * blockSize + i] = out[(size_t)b * blockSize + i] + sums[b];
    }
}

void scan_inclusive(const float* in, float* out, int size, int blockSize) { scan_blocks(in, out, size, blockSize, 1); }

}  // namespace orc

using namespace orc;

extern "C" void orc_scan(const float* in, float* out, int size, int blockSize) { scan_inclusive(in, out, size, blockSize); }
extern "C" void orc_scan_ex(const float* in, float* out, int size, int blockSize, int postfix) {
    scan_blocks(in, out, size, blockSize, postfix);
}
// CpuScan (scan.cuh:235-251): the reference's sequential float scan, its test's CPU side
extern "C" void orc_cpu_scan(const float* in, float* out, int size, int postfix) {
    float accu = 0.0f;
    for (int i = 0; i < size; ++i) {
        if (postfix) {
            accu += in[i];
            out[i] = accu;
        } else {
            out[i] = accu;
            accu += in[i];
        }
    }
}

extern "C" void orc_sun_dir(float timeOfDay, float sunAxisAngle, float* out) {
    F3 d = sun_direction(timeOfDay, sunAxisAngle);
    out[0] = d.x; out[1] = d.y; out[2] = d.z;
}

extern "C" void orc_sky(const OrcSkyTables* tables, const OrcSkyParams* params, OrcSkyOut* out) {
    OrcSkyParams p = *params;
    // kernel.cu:291-293
    p.sunScalar = fmx(p.sunScalar, 0.00001f);
    p.skyScalar = fmx(p.skyScalar, 0.00001f);
    p.sunAngle = fmx(p.sunAngle, 0.51f);
    F3 sunDir = sun_direction(p.timeOfDay, p.sunAxisAngle);
    out->sunDir[0] = sunDir.x; out->sunDir[1] = sunDir.y; out->sunDir[2] = sunDir.z;
    SkyState st;
    sky_state(sunDir, *tables, st);
    const int SW = 512, SH = 256, UW = 32, UH = 32;
    for (int y = 0; y < SH; ++y)
        for (int x = 0; x < SW; ++x) {
            float u = ((float)x + 0.5f) / SW, v = ((float)y + 0.5f) / SH;
            F3 c = sky_radiance(equal_area_map(u, v), sunDir, st) * p.skyScalar;
            c = max3(c, f3(0.0f));
            float* o = out->skyBuffer + ((size_t)y * SW + x) * 4;
            o[0] = c.x; o[1] = c.y; o[2] = c.z; o[3] = 0.0f;
            out->skyPdf[y * SW + x] = dot(c, f3(0.3f, 0.6f, 0.1f));
        }
    scan_inclusive(out->skyPdf, out->skyCdf, SW * SH, 256);
    const float cosMax = rt_cosf(p.sunAngle * kPi / 180.0f / 2.0f);  // M_PI is a float literal (linearMath.h:14-16)
    for (int y = 0; y < UH; ++y)
        for (int x = 0; x < UW; ++x) {
            float u = ((float)x + 0.5f) / UW, v = ((float)y + 0.5f) / UH;
            F3 rd = equal_area_map_cone(sunDir, u, v, cosMax);
            F3 c = sun_radiance(rd, sunDir, p.sunAngle, st) * p.sunScalar;
            c = max3(c, f3(0.0f));
            float* o = out->sunBuffer + ((size_t)y * UW + x) * 4;
            o[0] = c.x; o[1] = c.y; o[2] = c.z; o[3] = 0.0f;
            out->sunPdf[y * UW + x] = dot(c, f3(0.3f, 0.6f, 0.1f));
        }
    scan_inclusive(out->sunPdf, out->sunCdf, UW * UH, 32);
    float sunRadiusRadian = p.sunAngle * kPi / 180.0f / 2.0f;
    out->sunArea = rt_powf(rt_tanf(sunRadiusRadian), 2.0f) * kPi;
    out->sunAngleCosThetaMax = rt_cosf(sunRadiusRadian);
}

// Probe: GetSkyRadiance (unscaled) for one direction at the sun position of (timeOfDay,
// sunAxisAngle) — pins the sky model against SURVEY.md §8c's reference run (zenith).
extern "C" void orc_sky_radiance(const OrcSkyTables* tables, float timeOfDay, float sunAxisAngle, const float* dir,
                                 float* out) {
    F3 sunDir = sun_direction(timeOfDay, sunAxisAngle);
    SkyState st;
    sky_state(sunDir, *tables, st);
    F3 c = sky_radiance(f3(dir[0], dir[1], dir[2]), sunDir, st);
    out[0] = c.x; out[1] = c.y; out[2] = c.z;
}

extern "C" void orc_sky_radiance_sun(const OrcSkyTables* tables, const float* sun, const float* dir, float* out) {
    F3 sunDir = f3(sun[0], sun[1], sun[2]);
    SkyState st;
    sky_state(sunDir, *tables, st);
    F3 c = sky_radiance(f3(dir[0], dir[1], dir[2]), sunDir, st);
    out[0] = c.x; out[1] = c.y; out[2] = c.z;
}
