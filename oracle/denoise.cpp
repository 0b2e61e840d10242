// ORACLE (test infrastructure only; see ocommon.h) — SVGF-style denoiser and post-processing.
//
// Restates, in the reference's pass order (denoising.cu:5-189, postprocessing.cu:5-161,
// kernel.cu:376-381):
//   TemporalFilter              temporalDenoising.cuh:610-893
//   CalculateTileNoiseLevel     temporalDenoising.cuh:33-91 (32-lane shfl_down tree sums)
//   TileNoiseLevel8x8to16x16    temporalDenoising.cuh:93-102
//   TileNoiseLevelVisualize     temporalDenoising.cuh:104-140
//   SpatialFilter7x7            temporalDenoising.cuh:317-492 (24 taps, stride 2, phase frameNum%2)
//   CopyToHistoryColorBuffer    temporalDenoising.cuh:159-170
//   SpatialFilterGlobal5x5<S>   temporalDenoising.cuh:495-608 (S = 3, 6, 12)
//   ApplyAlbedo                 temporalDenoising.cuh:1127-1139
//   TemporalFilter2             temporalDenoising.cuh:896-1111
//   CopyToHistoryColorDepth     temporalDenoising.cuh:142-157
//   DownScale4                  postprocessing.cuh:142-170
//   Histogram2 / AutoExposure   postprocessing.cuh:24-136
//   BicubicScale                postprocessing.cuh:785-802 (SampleBicubicCatmullRom sampler.cuh:446-496)
//   SharpeningFilter            postprocessing.cuh:726-783
//   ToneMappingReinhardExtended postprocessing.cuh:542-564 (+ :488-516, luminance linearMath.h:746-749)
//   ToneMappingACES / ACES2 / Uncharted postprocessing.cuh:566-708 (ACESFitted, ACESFilm, Mat3 *)
//   BloomGuassian / Bloom       postprocessing.cuh:348-408
//   LensFlare(Pred)             postprocessing.cuh:414-487, sunPos/sunUv kernel.cu:126-127,
//                               predicate postprocessing.cu:88-94
//   CopyToOutput                kernel.cu:26-59
// Gaussian kernels gaussian.cuh:12-47; RgbToYcocg/YcocgToRgb temporalDenoising.cuh:10-21.
//
// Buffer semantics: CUDA surface reads clamp to the buffer edge, as here.
// The reference filters in place while neighbouring blocks read the same buffer (a race);
// this restatement reads every filter's input from the previous pass's buffer (ping-pong),
// which is the race-free meaning.  Threads outside the image write nothing (the reference's
// `x >= W && y >= H` test lets them write a clamped edge texel).  A pixel whose own colour is
// NaN is left unchanged by the LDS-staged filters (the reference returns before its barrier).
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <thread>
#include <vector>

#include "../include/rtx_amd.h"
#include "oracle.h"
#include "ocommon.h"
#include "opath.h"

namespace orc {
namespace {

// rows of a per-pixel pass over host threads: every pass below writes only its own pixel from
// read-only inputs, so the split changes nothing in the results (ORC_THREADS caps the count)
template <typename F>
void par_rows(int H, F f) {
    int T = (int)std::thread::hardware_concurrency();
    if (const char* e = getenv("ORC_THREADS")) T = atoi(e);
    T = T < 1 ? 1 : (T > 32 ? 32 : T);
    if (T == 1 || H < 64) {
        for (int y = 0; y < H; ++y) f(y);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            for (int y = t; y < H; y += T) f(y);
        });
    for (auto& x : th) x.join();
}

const double kG3[9] = {0.0578968, 0.0921378, 0.0584323, 0.0921378, 0.146629, 0.09299, 0.0584322, 0.0929898, 0.0589727};
const double kG5[25] = {0.00360466, 0.0144464, 0.0229902, 0.01458,   0.0036719,  0.0144464, 0.0578968,
                        0.0921378,  0.0584323, 0.0147159, 0.0229902, 0.0921378, 0.146629,  0.09299,
                        0.023419,   0.01458,   0.0584322, 0.0929898, 0.0589727, 0.014852,  0.00367191,
                        0.0147158,  0.0234191, 0.0148519, 0.0037404};
const double kG7[49] = {
    3.47404e-05, 0.000353875, 0.00141822, 0.00225698, 0.00143134,  0.000360475, 3.57221e-05,
    0.000353875, 0.00360466,  0.0144464,  0.0229902,  0.01458,     0.0036719,   0.000363875,
    0.00141822,  0.0144464,   0.0578968,  0.0921378,  0.0584323,   0.0147159,   0.0014583,
    0.00225698,  0.0229902,   0.0921378,  0.146629,   0.09299,     0.023419,    0.00232076,
    0.00143134,  0.01458,     0.0584322,  0.0929898,  0.0589727,   0.014852,    0.00147179,
    0.000360475, 0.00367191,  0.0147158,  0.0234191,  0.0148519,   0.0037404,   0.000370662,
    3.57221e-05, 0.000363875, 0.0014583,  0.00232075, 0.00147179,  0.000370662, 3.67315e-05};

// the tables as the filters use them (each double literal rounded to float), row-major
extern "C" int orc_filter_kernel(int size, float* out) {
    const double* g = size == 3 ? kG3 : size == 5 ? kG5 : size == 7 ? kG7 : nullptr;
    if (!g || !out) return -1;
    for (int i = 0; i < size * size; ++i) out[i] = (float)g[i];
    return 0;
}

const float kRayMaxF = 10e10f;

inline float h2f(uint16_t h) { return rt_h2f(h); }
inline uint16_t f2h(float f) { return rt_f2h(f); }
inline bool isnan3(F3 v) { return v.x != v.x || v.y != v.y || v.z != v.z; }
inline float clampf(float a, float lo = 0.0f, float hi = 1.0f) { return a < lo ? lo : a > hi ? hi : a; }
inline F3 clamp3(F3 a, F3 lo, F3 hi) { return f3(clampf(a.x, lo.x, hi.x), clampf(a.y, lo.y, hi.y), clampf(a.z, lo.z, hi.z)); }
inline F3 fmax3(F3 a, F3 b) { return f3(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z)); }
inline F3 fmin3(F3 a, F3 b) { return f3(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z)); }
inline F3 ycocg(F3 c) {
    const float t1 = c.x + c.z, t2 = c.y * 2.0f;
    return f3(t1 + t2, (c.x - c.z) * 2.0f, t2 - t1);
}
inline F3 ycocg_inv(F3 c) {
    const float t = c.x - c.z;
    return f3(t + c.y, c.x + c.z, t - c.y) * 0.25f;
}
inline int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

struct Img {  // a half4 / half buffer view with clamped reads
    int W, H;
    const uint16_t* p;
    int ch;
    size_t at(int x, int y) const { return ((size_t)clampi(y, 0, H - 1) * W + clampi(x, 0, W - 1)) * ch; }
    F3 rgb(int x, int y) const { const uint16_t* q = p + at(x, y); return f3(h2f(q[0]), h2f(q[1]), h2f(q[2])); }
    uint16_t u16(int x, int y, int c) const { return p[at(x, y) + c]; }
    float h(int x, int y, int c = 0) const { return h2f(p[at(x, y) + c]); }
};

// SampleBicubicSmoothStep<Load2DFuncHalf3Ushort1<Float3>> with the default (clamped) boundary
F3 bicubic_smooth_half(const Img& im, F2 uv) {
    const F2 UV = {uv.x * (float)im.W, uv.y * (float)im.H};
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
    for (int i = 0; i < 4; ++i) {
        sw += wt[i];
        o = o + im.rgb(sx[i], sy[i]) * wt[i];
    }
    return o / sw;
}

// 32-lane __shfl_down_sync tree sum as seen by lane 0 (offsets 16, 8, 4, 2, 1)
template <typename T>
T warp_tree_sum(const T* v) {
    T a[32];
    for (int i = 0; i < 32; ++i) a[i] = v[i];
    for (int off = 16; off > 0; off /= 2)
        for (int i = 0; i < off; ++i) a[i] = a[i] + a[i + off];
    return a[0];
}

struct Ctx {
    int W, H, frameNum;
    int hW, hH;  // historyDim (kernel.cu:266): size the accumulation / history colour were written at
    const rt_params* prm;
    const uint16_t *normal, *albedo, *depth, *motion;
    Img nrm() const { return Img{W, H, normal, 4}; }
    Img dep() const { return Img{W, H, depth, 1}; }
};

void store_color(uint16_t* dst, size_t p, F3 c, uint16_t mask) {
    dst[4 * p + 0] = f2h(c.x);
    dst[4 * p + 1] = f2h(c.y);
    dst[4 * p + 2] = f2h(c.z);
    dst[4 * p + 3] = mask;
}

void temporal_filter(const Ctx& c, const uint16_t* in, uint16_t* out, const uint16_t* accum) {
    const rt_denoising_params& dp = c.prm->denoise;
    const Img col{c.W, c.H, in, 4}, nrm = c.nrm(), dep = c.dep(), acc{c.hW, c.hH, accum, 4};
    memcpy(out, in, (size_t)c.W * c.H * 8);
    par_rows(c.H, [&](int y) {
        for (int x = 0; x < c.W; ++x) {
            const size_t p = (size_t)y * c.W + x;
            F3 cV = col.rgb(x, y);
            if (isnan3(cV)) continue;
            float dV = dep.h(x, y);
            F3 nV = nrm.rgb(x, y);
            const uint16_t mV = col.u16(x, y, 3);
            if (dV != dV) dV = 0.0f;
            if (isnan3(nV)) nV = f3(0.0f);
            if (dV >= kRayMaxF) continue;
            F3 nMax = ycocg(cV), nMin = ycocg(cV);
            F3 filt = f3(0.0f);
            float wsum = 0.0f;
            for (int j = 0; j < 9; ++j) {
                const int xo = j % 3, yo = j / 3;
                const int sx = x + xo - 1, sy = y + yo - 1;
                const F3 cc = col.rgb(sx, sy);
                const float d = dep.h(sx, sy);
                const F3 n = nrm.rgb(sx, sy);
                const uint16_t m = col.u16(sx, sy, 3);
                float w = 1.0f;
                w *= rt_powf(fmaxf(dot(nV, n), 0.0f), dp.temporal_denoise_sigma_normal);
                const float dd = (dV - d) / dp.temporal_denoise_sigma_depth;
                w *= rt_expf(-0.5f * dd * dd);
                w *= (mV != m) ? 1.0f / dp.temporal_denoise_sigma_material : 1.0f;
                w *= (float)kG3[xo + yo * 3];
                filt = filt + cc * w;
                wsum += w;
                const F3 nc = ycocg(cc);
                nMax = fmax3(nMax, nc);
                nMin = fmin3(nMin, nc);
            }
            if (wsum > 0) filt = filt / wsum;
            else filt = f3(0.0f);
            if (isnan3(filt)) filt = f3(0.0f);
            const F2 mv = {h2f(c.motion[2 * p]) - 0.5f, h2f(c.motion[2 * p + 1]) - 0.5f};
            const F2 inv = {1.0f / (float)c.W, 1.0f / (float)c.H};
            const F2 uv = {((float)x + 0.5f) * inv.x, ((float)y + 0.5f) * inv.y};
            const F2 huv = {uv.x + mv.x, uv.y + mv.y};
            if (huv.x < 0 || huv.y < 0 || huv.x > 1.0f || huv.y > 1.0f) {
                store_color(out, p, filt, mV);
                continue;
            }
            F3 cH = bicubic_smooth_half(acc, huv);
            F3 cHy = clamp3(ycocg(cH), nMin, nMax);
            cH = ycocg_inv(cHy);
            float lumaH = cHy.x;
            const float lumaMin = nMin.x, lumaMax = nMax.x, lumaC = ycocg(cV).x;
            float discard = 0.0f;
            const int hx = (int)floorf(huv.x * (float)c.hW), hy = (int)floorf(huv.y * (float)c.hH);
            for (int i = 0; i < 4; ++i) discard += (mV != acc.u16(hx + i % 2, hy + i / 2, 3)) ? 1.0f : 0.0f;
            discard /= 4.0f;
            cH = cH * (1.0f - discard) + filt * discard;
            lumaH = ycocg(cH).x;
            if (isnan3(cV)) cV = f3(0.0f);
            if (isnan3(cH)) cH = f3(0.0f);
            float blend = 1.0f / 8.0f;
            blend *= 0.2f + 0.8f * clampf(0.5f * fminf(fabsf(lumaH - lumaMin), fabsf(lumaH - lumaMax)) /
                                         fmaxf(fmaxf(lumaH, lumaC), 1e-4f));
            float wA = blend * fmaxf(0.0001f, 1.0f / (lumaC + 4.0f));
            float wB = (1.0f - blend) * fmaxf(0.0001f, 1.0f / (lumaH + 4.0f));
            const float ws = safe_divide(1.0f, wA + wB);
            wA *= ws;
            wB *= ws;
            F3 o = cV * wA + cH * wB;
            if (isnan3(o)) o = f3(0.0f);
            store_color(out, p, o, mV);
        }
    });
}

void tile_noise(const Ctx& c, const uint16_t* color, uint16_t* noise8, uint16_t* noise16) {
    const Img col{c.W, c.H, color, 4}, dep = c.dep();
    const int W8 = (c.W + 7) / 8, H8 = (c.H + 7) / 8, W16 = (c.W + 15) / 16, H16 = (c.H + 15) / 16;
    for (int by = 0; by < H8; ++by)
        for (int bx = 0; bx < W8; ++bx) {
            uint32_t bg1[32], bg2[32];
            float l1[32], l12[32], l2[32], l22[32];
            for (int lane = 0; lane < 32; ++lane) {
                const int tx = lane % 8, ty = lane / 8;
                const int x = bx * 8 + tx, ya = (by * 4 + ty) * 2, yb = ya + 1;
                const F3 ca = col.rgb(x, ya), cb = col.rgb(x, yb);
                bg1[lane] = dep.h(x, ya) >= kRayMaxF ? 1u : 0u;
                bg2[lane] = dep.h(x, yb) >= kRayMaxF ? 1u : 0u;
                l1[lane] = fmaxf(fmaxf(ca.x, ca.y), ca.z);
                l12[lane] = l1[lane] * l1[lane];
                l2[lane] = fmaxf(fmaxf(cb.x, cb.y), cb.z);
                l22[lane] = l2[lane] * l2[lane];
            }
            const uint32_t b1 = warp_tree_sum(bg1), b2 = warp_tree_sum(bg2);
            const float s1 = warp_tree_sum(l1), s12 = warp_tree_sum(l12), s2 = warp_tree_sum(l2), s22 = warp_tree_sum(l22);
            const float notSky = 1.0f - (float)(b1 + b2) / 64.0f;
            const float lumAve = (s1 + s2) / 64.0f;
            const float lumAveSq = lumAve * lumAve;
            const float lumSqAve = (s12 + s22) / 64.0f;
            const float var = fmaxf(1e-20f, lumSqAve - lumAveSq);
            float noise = var / fmaxf(lumAveSq, 1e-20f);
            noise *= notSky;
            noise8[(size_t)by * W8 + bx] = f2h(noise);
        }
    const Img n8{W8, H8, noise8, 1};
    for (int y = 0; y < H16; ++y)
        for (int x = 0; x < W16; ++x) {
            const float v1 = n8.h(2 * x, 2 * y), v2 = n8.h(2 * x + 1, 2 * y), v3 = n8.h(2 * x, 2 * y + 1),
                        v4 = n8.h(2 * x + 1, 2 * y + 1);
            noise16[(size_t)y * W16 + x] = f2h((v1 + v2 + v3 + v4) / 4);
        }
}

// TileNoiseLevelVisualize: outline noisy 16x16 tiles (debug pass, off by default)
void noise_visualize(const Ctx& c, uint16_t* color, uint16_t* normal, uint16_t* depth, const uint16_t* noise16, int level) {
    const int W16 = (c.W + 15) / 16;
    const float thr = level == 1 ? c.prm->denoise.noise_threshold_local : c.prm->denoise.noise_threshold_large;
    for (int y = 0; y < c.H; ++y)
        for (int x = 0; x < c.W; ++x) {
            const int tx = x % 16, ty = y % 16;
            if (!(tx == 0 || tx == 15 || ty == 0 || ty == 15)) continue;
            if (!(h2f(noise16[(size_t)(y / 16) * W16 + x / 16]) > thr)) continue;
            const size_t p = (size_t)y * c.W + x;
            store_color(color, p, level == 1 ? f3(1.0f, 0.5f, 0.0f) : f3(1.0f, 0.0f, 0.0f), 0xFFFF);
            for (int k = 0; k < 4; ++k) normal[4 * p + k] = f2h(0.0f);
            depth[p] = f2h(kRayMaxF);
        }
}

void spatial7x7(const Ctx& c, const uint16_t* in, uint16_t* out, const uint16_t* noise16) {
    const rt_denoising_params& dp = c.prm->denoise;
    const Img col{c.W, c.H, in, 4}, nrm = c.nrm(), dep = c.dep();
    const int W16 = (c.W + 15) / 16;
    memcpy(out, in, (size_t)c.W * c.H * 8);
    par_rows(c.H, [&](int y) {
        for (int x = 0; x < c.W; ++x) {
            if (h2f(noise16[(size_t)(y / 16) * W16 + x / 16]) < dp.noise_threshold_local) continue;
            F3 cV = col.rgb(x, y);
            if (isnan3(cV)) continue;
            float dV = dep.h(x, y);
            F3 nV = nrm.rgb(x, y);
            const uint16_t mV = col.u16(x, y, 3);
            if (dV != dV) dV = 0.0f;
            if (isnan3(nV)) nV = f3(0.0f);
            if (dV >= kRayMaxF) continue;
            F3 sum = f3(0.0f);
            float sw = 0.0f;
            int j = c.frameNum % 2;
            for (int i = 0; i < 24; ++i) {
                const int xo = j % 7, yo = j / 7;
                j += 2;
                const int sx = x + xo - 3, sy = y + yo - 3;
                F3 cc = col.rgb(sx, sy);
                float d = dep.h(sx, sy);
                F3 n = nrm.rgb(sx, sy);
                const uint16_t m = col.u16(sx, sy, 3);
                if (isnan3(cc)) cc = f3(0.0f);
                if (d != d) d = 0.0f;
                if (isnan3(n)) n = f3(0.0f);
                float w = 1.0f;
                w *= rt_powf(fmaxf(dot(nV, n), 0.0001f), dp.local_denoise_sigma_normal);
                const float dd = (dV - d) / dp.local_denoise_sigma_depth;
                w *= rt_expf(-0.5f * dd * dd);
                w *= (mV != m) ? 1.0f / dp.local_denoise_sigma_material : 1.0f;
                w *= (float)kG7[xo + yo * 7];
                sum = sum + cc * w;
                sw += w;
            }
            if (isnan3(sum)) sum = f3(0.0f);
            if (sw != sw) sw = 0.0f;
            F3 fin = sw == 0 ? f3(0.0f) : sum / sw;
            if (isnan3(fin)) fin = f3(0.0f);
            store_color(out, (size_t)y * c.W + x, fin, mV);
        }
    });
}

void spatial5x5(const Ctx& c, const uint16_t* in, uint16_t* out, const uint16_t* noise16, int S) {
    const rt_denoising_params& dp = c.prm->denoise;
    const Img col{c.W, c.H, in, 4}, nrm = c.nrm(), dep = c.dep();
    const int W16 = (c.W + 15) / 16;
    memcpy(out, in, (size_t)c.W * c.H * 8);
    par_rows(c.H, [&](int y) {
        for (int x = 0; x < c.W; ++x) {
            if (h2f(noise16[(size_t)(y / 16) * W16 + x / 16]) < dp.noise_threshold_large) continue;
            F3 nV = nrm.rgb(x, y);
            F3 cV = col.rgb(x, y);
            const uint16_t mV = col.u16(x, y, 3);
            float dV = dep.h(x, y);
            if (isnan3(cV)) cV = f3(0.0f);
            if (dV != dV) dV = 0.0f;
            if (isnan3(nV)) nV = f3(0.0f);
            if (dV >= 10e9f) continue;
            F3 sum = f3(0.0f);
            float sw = 0.0f;
            for (int k = 0; k < 25; ++k) {
                const int i = k % 5, j = k / 5;
                const int sx = x + (i - 2) * S, sy = y + (j - 2) * S;
                F3 cc = col.rgb(sx, sy);
                const float d = dep.h(sx, sy);
                const F3 n = nrm.rgb(sx, sy);
                const uint16_t m = col.u16(sx, sy, 3);
                float w = 1.0f;
                w *= rt_powf(fmaxf(dot(nV, n), 0.0f), dp.large_denoise_sigma_normal);
                const float dd = (dV - d) / dp.large_denoise_sigma_depth;
                w *= rt_expf(-0.5f * dd * dd);
                w *= (mV != m) ? 1.0f / dp.large_denoise_sigma_material : 1.0f;
                w *= (float)kG5[i + j * 5];
                if (isnan3(cc)) { cc = f3(0.0f); w = 0.0f; }
                sum = sum + cc * w;
                sw += w;
            }
            if (isnan3(sum)) sum = f3(0.0f);
            if (sw != sw) sw = 0.0f;
            F3 fin = sw == 0 ? f3(0.0f) : sum / sw;
            if (isnan3(fin)) fin = f3(0.0f);
            store_color(out, (size_t)y * c.W + x, fin, mV);
        }
    });
}

void apply_albedo(const Ctx& c, uint16_t* color) {
    const uint16_t one = f2h(1.0f);
    for (size_t p = 0; p < (size_t)c.W * c.H; ++p) {
        const F3 cc = f3(h2f(color[4 * p]), h2f(color[4 * p + 1]), h2f(color[4 * p + 2]));
        const F3 a = f3(h2f(c.albedo[4 * p]), h2f(c.albedo[4 * p + 1]), h2f(c.albedo[4 * p + 2]));
        store_color(color, p, cc * a, one);
    }
}

void temporal_filter2(const Ctx& c, const uint16_t* in, uint16_t* out, const uint16_t* hist) {
    const Img col{c.W, c.H, in, 4}, hc{c.hW, c.hH, hist, 4};
    memcpy(out, in, (size_t)c.W * c.H * 8);
    const float FLTMIN = 1.17549435e-38f, FLTMAX = 3.402823466e+38f;
    par_rows(c.H, [&](int y) {
        for (int x = 0; x < c.W; ++x) {
            const size_t p = (size_t)y * c.W + x;
            const F3 cV = ycocg_inv(ycocg(col.rgb(x, y)));
            const int mV = col.u16(x, y, 3);
            F3 nMax = f3(FLTMIN), nMin = f3(FLTMAX), nMax2 = f3(FLTMIN), nMin2 = f3(FLTMAX);
            for (int j = 0; j < 9; ++j) {
                const int xo = j % 3, yo = j / 3;
                const F3 cc = ycocg(col.rgb(x + xo - 1, y + yo - 1));
                const int m = col.u16(x + xo - 1, y + yo - 1, 3);
                if (m == mV) {
                    nMax = fmax3(nMax, cc);
                    nMin = fmin3(nMin, cc);
                    if (abs(xo - 1) + abs(yo - 1) <= 1) {
                        nMax2 = fmax3(nMax2, cc);
                        nMin2 = fmin3(nMin2, cc);
                    }
                }
            }
            nMax = (nMax + nMax2) / 2.0f;
            nMin = (nMin + nMin2) / 2.0f;
            const F2 mv = {h2f(c.motion[2 * p]) - 0.5f, h2f(c.motion[2 * p + 1]) - 0.5f};
            const F2 inv = {1.0f / (float)c.W, 1.0f / (float)c.H};
            const F2 uv = {((float)x + 0.5f) * inv.x, ((float)y + 0.5f) * inv.y};
            const F2 huv = {uv.x + mv.x, uv.y + mv.y};
            if (huv.x < 0 || huv.y < 0 || huv.x > 1.0f || huv.y > 1.0f) continue;
            F3 cH = bicubic_smooth_half(hc, huv);
            const F3 cHy = clamp3(ycocg(cH), nMin, nMax);
            cH = ycocg_inv(cHy);
            float lumaH = cHy.x;
            const float lumaMin = nMin.x, lumaMax = nMax.x, lumaC = ycocg(cV).x;
            float discard = 0.0f;
            const int hx = (int)floorf(huv.x * (float)c.hW), hy = (int)floorf(huv.y * (float)c.hH);
            for (int i = 0; i < 4; ++i) discard += (mV != (int)hc.u16(hx + i % 2, hy + i / 2, 3)) ? 1.0f : 0.0f;
            discard /= 4.0f;
            if (discard == 1.0f) continue;
            cH = cH * (1.0f - discard) + cV * discard;
            lumaH = ycocg(cH).x;
            float blend = 3.0f / 4.0f;
            blend *= 0.2f + 0.8f * clampf(0.5f * fminf(fabsf(lumaH - lumaMin), fabsf(lumaH - lumaMax)) /
                                         fmaxf(fmaxf(lumaH, lumaC), 1e-4f));
            float wA = blend * fmaxf(0.0001f, 1.0f / (lumaC + 4.0f));
            float wB = (1.0f - blend) * fmaxf(0.0001f, 1.0f / (lumaH + 4.0f));
            const float ws = safe_divide(1.0f, wA + wB);
            wA *= ws;
            wB *= ws;
            F3 o = cV * wA + cH * wB;
            if (isnan3(o)) o = f3(0.0f);
            store_color(out, p, o, (uint16_t)mV);
        }
    });
}

// ------------------------------------------------------------------ post
struct H4 { float x, y, z, w; };
H4 load_h4(const uint16_t* b, int W, int H, int x, int y) {
    const uint16_t* q = b + ((size_t)clampi(y, 0, H - 1) * W + clampi(x, 0, W - 1)) * 4;
    return H4{h2f(q[0]), h2f(q[1]), h2f(q[2]), h2f(q[3])};
}
H4 add4(H4 a, H4 b) { return H4{a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }

void downscale4(const uint16_t* in, int W, int H, uint16_t* out, int Wo, int Ho) {
    for (int oy = 0; oy < Ho; ++oy)
        for (int ox = 0; ox < Wo; ++ox) {
            H4 s[4][4];
            for (int a = 0; a < 4; ++a)
                for (int b = 0; b < 4; ++b) {
                    const H4 v = load_h4(in, W, H, 4 * ox + a, 4 * oy + b);
                    s[a][b] = H4{v.x / 16, v.y / 16, v.z / 16, v.z / 16};  // Float4::operator/ (linearMath.h:423)
                }
            H4 q[2][2];
            for (int a = 0; a < 2; ++a)
                for (int b = 0; b < 2; ++b)
                    q[a][b] = add4(add4(add4(s[2 * a][2 * b], s[2 * a + 1][2 * b]), s[2 * a][2 * b + 1]), s[2 * a + 1][2 * b + 1]);
            const H4 r = add4(add4(add4(q[0][0], q[1][0]), q[0][1]), q[1][1]);
            uint16_t* o = out + ((size_t)oy * Wo + ox) * 4;
            o[0] = f2h(r.x); o[1] = f2h(r.y); o[2] = f2h(r.z); o[3] = f2h(r.w);
        }
}

void histogram(const uint16_t* c64, int W64, int H64, uint32_t* hist) {
    memset(hist, 0, 64 * 4);
    const int tx = W64 < 32 ? W64 : 32, ty = H64 < 32 ? H64 : 32;
    const F3 wl = f3((float)0.3, (float)0.6, (float)0.1);
    for (int y = 0; y < ty; ++y)
        for (int x = 0; x < tx; ++x) {
            const H4 v = load_h4(c64, W64, H64, x, y);
            const float lum = dot(f3(v.x, v.y, v.z), wl);
            const float logL = (float)((double)rt_log2f(lum) * 0.1 + 0.75);
            const float sc = (float)((double)(clampf(logL, 0.0f, 1.0f) * 63) * 0.99999);
            const uint32_t b = (uint32_t)rintf(sc);
            hist[b] += 1;
        }
}

float bin_to_lum(int i) { return rt_exp2f((float)(((double)(float)i / (63 * 0.99999) - 0.75) / 0.1)); }

void auto_exposure(float* e, const uint32_t* hist, float area, float deltaTime, float gain) {
    const float darkT = (float)0.4, brightT = (float)0.9;
    float lumiSum = 0, lumiSumArea = 0, accu = 0, brightLum = 0;
    int i = 0;
    for (; i < 64; ++i) {
        const float fHist = (float)hist[i] / area;
        const float lum = bin_to_lum(i);
        accu += fHist;
        const float dark = accu - darkT;
        if (dark > 0) {
            lumiSumArea += dark;
            lumiSum += dark * lum;
            break;
        }
    }
    for (; i < 64; ++i) {
        const float fHist = (float)hist[i] / area;
        const float lum = bin_to_lum(i);
        accu += fHist;
        const float bright = accu - brightT;
        if (bright > 0) {
            const float partial = brightT - (accu - fHist);
            lumiSumArea += partial;
            lumiSum += partial * lum;
            brightLum = lum;
            break;
        } else {
            lumiSumArea += fHist;
            lumiSum += fHist * lum;
        }
    }
    float aveLum = lumiSum / lumiSumArea;
    aveLum = clampf(aveLum, 0.1f, 100.0f);
    float lumTemp = e[1], lumBright = e[2];
    const float k = 1.0f - rt_expf(-deltaTime * 0.001f);
    lumTemp = lumTemp + (aveLum - lumTemp) * k;
    lumBright = lumBright + (brightLum - lumBright) * k;
    const float EC = 1.03f - 2.0f / (rt_log10f(lumTemp + 1.0f) + 2.0f);
    const float EV = gain * EC / lumTemp;
    e[0] = EV;
    e[1] = lumTemp;
    e[2] = lumBright;
    e[3] = brightLum;
}

void bicubic_scale(const uint16_t* in, int W, int H, uint16_t* out, int Ws, int Hs) {
    par_rows(Hs, [&](int y) {
        for (int x = 0; x < Ws; ++x) {
            const F2 uv = {(float)x / Ws, (float)y / Hs};
            const F2 UV = {uv.x * (float)W, uv.y * (float)H};
            const float fx0 = floorf(UV.x - 0.5f), fy0 = floorf(UV.y - 0.5f);
            const F2 f = {UV.x - (fx0 + 0.5f), UV.y - (fy0 + 0.5f)};
            const F2 f2 = {f.x * f.x, f.y * f.y};
            const F2 f3v = {f2.x * f.x, f2.y * f.y};
            const F2 w0 = {f2.x - 0.5f * (f3v.x + f.x), f2.y - 0.5f * (f3v.y + f.y)};
            const F2 w1 = {1.5f * f3v.x - 2.5f * f2.x + 1.0f, 1.5f * f3v.y - 2.5f * f2.y + 1.0f};
            const F2 w3 = {0.5f * (f3v.x - f2.x), 0.5f * (f3v.y - f2.y)};
            const F2 w2 = {1.0f - w0.x - w1.x - w3.x, 1.0f - w0.y - w1.y - w3.y};
            const int t1x = (int)fx0, t1y = (int)fy0;
            const float wx[4] = {w0.x, w1.x, w2.x, w3.x}, wy[4] = {w0.y, w1.y, w2.y, w3.y};
            F3 o = f3(0.0f);
            float sw = 0.0f;
            for (int j = 0; j < 4; ++j)
                for (int i = 0; i < 4; ++i) {
                    const float w = wx[i] * wy[j];
                    sw += w;
                    const H4 v = load_h4(in, W, H, t1x - 1 + i, t1y - 1 + j);
                    o = o + f3(v.x, v.y, v.z) * w;
                }
            o = o / sw;
            uint16_t* q = out + ((size_t)y * Ws + x) * 4;
            q[0] = f2h(o.x); q[1] = f2h(o.y); q[2] = f2h(o.z); q[3] = f2h(1.0f);
        }
    });
}

void sharpen(const uint16_t* in, uint16_t* out, int W, int H) {
    par_rows(H, [&](int y) {
        for (int x = 0; x < W; ++x) {
            F3 c[3][3];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    const H4 v = load_h4(in, W, H, x + i - 1, y + j - 1);
                    c[i][j] = f3(v.x, v.y, v.z);
                }
            auto mx3 = [](F3 a, F3 b, F3 d) { return fmax3(fmax3(a, b), d); };
            auto mn3 = [](F3 a, F3 b, F3 d) { return fmin3(fmin3(a, b), d); };
            F3 t1 = mx3(c[1][1], c[0][1], c[2][1]);
            F3 t2 = mx3(t1, c[1][0], c[1][2]);
            F3 t3 = mx3(t2, c[0][0], c[0][2]);
            F3 t4 = mx3(t3, c[2][0], c[2][2]);
            const F3 smax = t2 + t4;
            t1 = mn3(c[1][1], c[0][1], c[2][1]);
            t2 = mn3(t1, c[1][0], c[1][2]);
            t3 = mn3(t2, c[0][0], c[0][2]);
            t4 = mn3(t3, c[2][0], c[2][2]);
            const F3 smin = t2 + t4;
            const F3 two_minus = f3(2.0f - smax.x, 2.0f - smax.y, 2.0f - smax.z);
            F3 amp = clamp3(fmin3(smin, two_minus) / smax, f3(0.0f), f3(1.0f));
            amp = f3(1.0f / sqrtf(amp.x), 1.0f / sqrtf(amp.y), 1.0f / sqrtf(amp.z));
            const float peak = 8.0f - 3.0f * 1.0f;
            const F3 w = f3(-1.0f) / (amp * peak);
            F3 o = (((c[0][1] + c[2][1]) + c[1][0]) + c[1][2]) * w + c[1][1];
            o = o / (f3(1.0f) + f3(4.0f) * w);
            uint16_t* q = out + ((size_t)y * W + x) * 4;
            q[0] = f2h(o.x); q[1] = f2h(o.y); q[2] = f2h(o.z); q[3] = f2h(1.0f);
        }
    });
}

float luminance(F3 v) { return dot(v, f3(0.2126f, 0.7152f, 0.0722f)); }

// ToneMappingReinhardExtended / ACES (ACESFitted) / ACES2 (ACESFilm) / Uncharted, each
// followed by the clamp3f(pow3f(color, 1 / gamma)) gamma step (postprocessing.cuh:488-708)
F3 mat3_mul(const float m[9], F3 v) {  // Mat3 * Float3: rows (m00 m01 m02) ... via InnerProduct
    return f3(inner3(m[0], v.x, m[1], v.y, m[2], v.z), inner3(m[3], v.x, m[4], v.y, m[5], v.z),
              inner3(m[6], v.x, m[7], v.y, m[8], v.z));
}

F3 tonemap_color(F3 c, int type, const rt_post_process_params& pp) {
    if (type == 3) {  // ReinhardExtendedLuminance
        const float lo = luminance(c);
        const float num = lo * (1.0f + (lo / (pp.maxWhite * pp.maxWhite)));
        const float ln = num / (1.0f + lo);
        c = c * (ln / luminance(c));
    } else if (type == 1) {  // ACESFitted
        const float in[9] = {(float)0.59719, (float)0.35458, (float)0.04823, (float)0.07600, (float)0.90834,
                             (float)0.01566, (float)0.02840, (float)0.13383, (float)0.83777};
        const float out[9] = {(float)1.60475, (float)-0.53108, (float)-0.07367, (float)-0.10208, (float)1.10813,
                              (float)-0.00605, (float)-0.00327, (float)-0.07276, (float)1.07602};
        c = mat3_mul(in, c);
        const float lum = luminance(c);  // RRTAndODTFitLuminance
        const float a = lum * (lum + 0.0245786f) - 0.000090537f;
        const float b = lum * (0.983729f * lum + 0.4329510f) + 0.238081f;
        c = c * ((a / b) / luminance(c));
        c = mat3_mul(out, c);
        c = clamp3(c, f3(0.0f), f3(1.0f));
    } else if (type == 2) {  // ACESFilm
        const float a = 2.51f, b = 0.03f, cc = 2.43f, d = 0.59f, e = 0.14f;
        const F3 num = c * (c * a + b);
        const F3 den = c * (c * cc + d) + e;
        c = clamp3(num / den, f3(0.0f), f3(1.0f));
    } else {  // Uncharted: Uncharted2Tonemap returns 0, so the white scale is 1/0
        const F3 curr = f3(0.0f);
        const F3 whiteScale = f3(1.0f / 0.0f);
        c = curr * whiteScale;
    }
    const float g = 1.0f / pp.gamma;
    return clamp3(f3(rt_powf(c.x, g), rt_powf(c.y, g), rt_powf(c.z, g)), f3(0.0f), f3(1.0f));
}

void tonemap(uint16_t* buf, int W, int H, float exposure, int type, const rt_post_process_params& pp) {
    for (size_t p = 0; p < (size_t)W * H; ++p) {
        F3 c = f3(h2f(buf[4 * p]), h2f(buf[4 * p + 1]), h2f(buf[4 * p + 2]));
        c = tonemap_color(c * exposure, type, pp);
        buf[4 * p] = f2h(c.x); buf[4 * p + 1] = f2h(c.y); buf[4 * p + 2] = f2h(c.z); buf[4 * p + 3] = f2h(1.0f);
    }
}

// BloomGuassian: brightness key max(sqrt(lum^2 - brightLum), 0) (a NaN square root keys to 0),
// then the 5x5 gaussian over the keyed texels, clamped reads
void bloom_gauss(const uint16_t* in, int W, int H, uint16_t* out, float brightLum) {
    std::vector<F3> keyed((size_t)W * H);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const H4 v = load_h4(in, W, H, x, y);
            F3 c = f3(v.x, v.y, v.z);
            const float lum = fmx(fmx(c.x, c.y), c.z);
            const float s = sqrtf(lum * lum - brightLum);
            c = c * (s > 0.0f ? s : 0.0f);
            keyed[(size_t)y * W + x] = c;
        }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            F3 o = f3(0.0f);
            float wsum = 0.0f;
            for (int i = 0; i < 25; ++i) {
                const int sx = clampi(x + i % 5 - 2, 0, W - 1), sy = clampi(y + i / 5 - 2, 0, H - 1);
                const float g = (float)kG5[i];
                o = o + keyed[(size_t)sy * W + sx] * g;
                wsum += g;
            }
            o = o / wsum;
            if (isnan3(o)) o = f3(0.0f);
            uint16_t* q = out + ((size_t)y * W + x) * 4;
            q[0] = f2h(o.x); q[1] = f2h(o.y); q[2] = f2h(o.z); q[3] = f2h(1.0f);
        }
}

// SampleBicubicCatmullRom<Load2DFuncHalf4<Float3>> (sampler.cuh:446-496), clamped reads
F3 catmull_rom(const uint16_t* in, int W, int H, F2 uv) {
    const F2 UV = {uv.x * (float)W, uv.y * (float)H};
    const float fx0 = floorf(UV.x - 0.5f), fy0 = floorf(UV.y - 0.5f);
    const F2 f = {UV.x - (fx0 + 0.5f), UV.y - (fy0 + 0.5f)};
    const F2 f2 = {f.x * f.x, f.y * f.y};
    const F2 f3v = {f2.x * f.x, f2.y * f.y};
    const F2 w0 = {f2.x - 0.5f * (f3v.x + f.x), f2.y - 0.5f * (f3v.y + f.y)};
    const F2 w1 = {1.5f * f3v.x - 2.5f * f2.x + 1.0f, 1.5f * f3v.y - 2.5f * f2.y + 1.0f};
    const F2 w3 = {0.5f * (f3v.x - f2.x), 0.5f * (f3v.y - f2.y)};
    const F2 w2 = {1.0f - w0.x - w1.x - w3.x, 1.0f - w0.y - w1.y - w3.y};
    const int t1x = (int)fx0, t1y = (int)fy0;
    const float wx[4] = {w0.x, w1.x, w2.x, w3.x}, wy[4] = {w0.y, w1.y, w2.y, w3.y};
    F3 o = f3(0.0f);
    float sw = 0.0f;
    for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 4; ++i) {
            const float w = wx[i] * wy[j];
            sw += w;
            const H4 v = load_h4(in, W, H, t1x - 1 + i, t1y - 1 + j);
            o = o + f3(v.x, v.y, v.z) * w;
        }
    return o / sw;
}

// Bloom: colour += (bloom4 + bloom16 sampled bicubically) * 0.05, alpha 1
void bloom_apply(uint16_t* color, int W, int H, const uint16_t* b4, int W4, int H4, const uint16_t* b16, int W16,
                 int H16) {
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const F2 uv = {(float)x / W, (float)y / H};
            const F3 s4 = catmull_rom(b4, W4, H4, uv), s16 = catmull_rom(b16, W16, H16, uv);
            uint16_t* q = color + ((size_t)y * W + x) * 4;
            F3 c = f3(h2f(q[0]), h2f(q[1]), h2f(q[2]));
            c = c + (s4 + s16) * 0.05f;
            if (isnan3(c)) c = f3(0.0f);
            q[0] = f2h(c.x); q[1] = f2h(c.y); q[2] = f2h(c.z); q[3] = f2h(1.0f);
        }
}

// ---- LensFlare (postprocessing.cuh:414-480)
float lf_fract(float x) { return x - truncf(x); }  // modff: the signed fractional part
float lf_rand(float w) { return lf_fract(rt_sinf(w) * 1000.0f); }
float lf_len(F2 p) { return sqrtf(p.x * p.x + p.y * p.y); }
float smoothstep1f(float a, float b, float w) { return a + (w * w * (3.0f - 2.0f * w)) * (b - a); }

float lf_reg_shape(F2 p, int N) {
    const float a = rt_atan2f(p.x, p.y) + 0.2f;
    const float b = kTwoPi / float(N);
    return smoothstep1f(0.5f, 0.51f, rt_cosf(floorf(0.5f + a / b) * b - a) * lf_len(p));
}

F3 lf_circle(F2 p, float size, float dist, F2 m) {
    const float d4 = (float)((double)dist * 4.0);
    const float l = lf_len(F2{p.x + m.x * d4, p.y + m.y * d4}) + size / 2.0f;
    const float c = fmx(0.01f - rt_powf(lf_len(F2{p.x + m.x * dist, p.y + m.y * dist}), size * 1.4f), 0.0f) * 30.0f;
    const float c1 = fmx(0.001f - rt_powf(l - 0.3f, 1.0f / 40.0f) + rt_sinf(l * 30.0f), 0.0f) * 3.0f;
    const F2 md = {m.x * dist / 2.0f, m.y * dist / 2.0f};
    const F2 q = {(p.x - md.x) + 0.09f, (p.y - md.y) + 0.09f};
    const float c2 = fmx(0.04f / rt_powf(lf_len(q) * 1.0f, 1.0f), 0.0f) / 20.0f;
    const F2 rp = {(p.x * 5.0f + (m.x * dist) * 5.0f) + 0.9f, (p.y * 5.0f + (m.y * dist) * 5.0f) + 0.9f};
    const float sh = fmx(0.01f - rt_powf(lf_reg_shape(rp, 6), 1.0f), 0.0f) * 6.0f;
    const F3 a = f3(0.44f * 8.0f + dist * 4.0f, 0.24f * 8.0f + dist * 4.0f, 0.2f * 8.0f + dist * 4.0f);
    const F3 color = f3(rt_cosf(a.x) * 0.5f + 0.5f, rt_cosf(a.y) * 0.5f + 0.5f, rt_cosf(a.z) * 0.5f + 0.5f);
    F3 f = color * c;
    f = f + color * c1;
    f = f + color * c2;
    f = f + color * sh;
    return f - 0.01f;
}

void lens_flare(uint16_t* color, int W, int H, F2 sunPos) {
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            F2 uv = {(float)x / (float)W, (float)y / (float)H};
            uv = F2{uv.x - 0.5f, uv.y - 0.5f};
            uv.x *= (float)W / (float)H;
            const F2 vec = {uv.x - sunPos.x, uv.y - sunPos.y};
            const float len = lf_len(vec);
            uint16_t* q = color + ((size_t)y * W + x) * 4;
            F3 c = f3(h2f(q[0]), h2f(q[1]), h2f(q[2]));
            for (int i = 0; i < 2; ++i)
                c = c + lf_circle(uv, rt_powf(lf_rand(i * 2000.0f) * 1.8f, 2.0f) + 1.41f,
                                  lf_rand(i * 20.0f) * 3.0f + 0.2f - 0.5f, sunPos);
            const float angle = rt_atan2f(vec.y, vec.x);
            c = c + fmx(0.1f / fmx(rt_powf(len * 10.0f, 5.0f), 0.0001f), 0.0f) *
                        fabsf(rt_sinf(angle * 5.0f + rt_cosf(angle * 9.0f))) / 20.0f;
            c = c + (fmx(0.1f / rt_powf(len * 10.0f, 1.0f / 20.0f), 0.0f) +
                     fabsf(rt_sinf(angle * 3.0f + rt_cosf(angle * 9.0f))) / 16.0f * fabsf(rt_sinf(angle * 9.0f)));
            q[0] = f2h(c.x); q[1] = f2h(c.y); q[2] = f2h(c.z); q[3] = f2h(1.0f);
        }
}

void copy_to_output(const uint16_t* scaled, int W, int H, int frameNum, const uint8_t* bn, uint8_t* rgba) {
    const float one_m_eps = 1.0f - 1.1920928955078125e-07f;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const size_t p = (size_t)y * W + x;
            F3 c = f3(h2f(scaled[4 * p]), h2f(scaled[4 * p + 1]), h2f(scaled[4 * p + 2]));
            const int s = frameNum * 1 + 0;
            const F3 jit = f3(bluenoise(bn, x, y, s, 0) / 256, bluenoise(bn, x, y, s, 1) / 256, bluenoise(bn, x, y, s, 2) / 256);
            c = clamp3(c + jit, f3(0.0f), f3(one_m_eps));
            rgba[4 * p] = (uint8_t)(c.x * 256);
            rgba[4 * p + 1] = (uint8_t)(c.y * 256);
            rgba[4 * p + 2] = (uint8_t)(c.z * 256);
            rgba[4 * p + 3] = 1;
        }
}

}  // namespace
}  // namespace orc

using namespace orc;

extern "C" int orc_denoise_post(const OrcDrawIO* io) {
    const int W = (int)io->W, H = (int)io->H, Ws = (int)io->Ws, Hs = (int)io->Hs;
    const size_t P = (size_t)W * H;
    const rt_params& prm = *io->params;
    const rt_render_pass_settings& ps = prm.pass;
    if (ps.enableToneMapping && (prm.post.toneMappingType < 0 || prm.post.toneMappingType > 3)) return -1;
    Ctx c{W, H, io->frameNum, io->histW ? (int)io->histW : W, io->histH ? (int)io->histH : H, io->params,
          io->normal, io->albedo, io->depth, io->motion};
    OrcPostState& st = *io->state;
    std::vector<uint16_t> tmp(P * 4);
    uint16_t* cur = io->color;
    uint16_t* alt = tmp.data();
    auto flip = [&]() {  // keep the result in io->color after every pass
        memcpy(io->color, alt, P * 8);
    };
    // local copies of normal/depth for the (debug) visualize pass, which writes them
    std::vector<uint16_t> nrmv, depv;
    if (ps.enableNoiseLevelVisualize) {
        nrmv.assign(io->normal, io->normal + P * 4);
        depv.assign(io->depth, io->depth + P);
        c.normal = nrmv.data();
        c.depth = depv.data();
    }
    if (ps.enableTemporalDenoising && io->frameNum != 1) {
        temporal_filter(c, cur, alt, st.accum);
        flip();
    }
    if (ps.enableLocalSpatialFilter) {
        tile_noise(c, cur, io->noise8, io->noise16);
        if (ps.enableNoiseLevelVisualize) noise_visualize(c, cur, nrmv.data(), depv.data(), io->noise16, 1);
        spatial7x7(c, cur, alt, io->noise16);
        flip();
    }
    if (ps.enableTemporalDenoising) memcpy(st.accum, cur, P * 8);
    if (ps.enableWideSpatialFilter) {
        tile_noise(c, cur, io->noise8, io->noise16);
        if (ps.enableNoiseLevelVisualize) noise_visualize(c, cur, nrmv.data(), depv.data(), io->noise16, 2);
        const int strides[3] = {3, 6, 12};
        for (int s : strides) {
            spatial5x5(c, cur, alt, io->noise16, s);
            flip();
        }
    }
    apply_albedo(c, cur);
    if (ps.enableTemporalDenoising2) {
        if (io->frameNum != 1) {
            temporal_filter2(c, cur, alt, st.histColor);
            flip();
        }
        memcpy(st.histColor, cur, P * 8);
        memcpy(st.histDepth, c.depth, P * 2);
    }
    // ---- post (postprocessing.cu:5-161)
    const int W4 = (W + 3) / 4, H4 = (H + 3) / 4, W16 = (W4 + 3) / 4, H16 = (H4 + 3) / 4, W64 = (W16 + 3) / 4,
              H64 = (H16 + 3) / 4;
    if (ps.enablePostProcess) {
        if (ps.enableDownScalePasses) {
            downscale4(cur, W, H, io->c4, W4, H4);
            downscale4(io->c4, W4, H4, io->c16, W16, H16);
            downscale4(io->c16, W16, H16, io->c64, W64, H64);
        }
        memset(io->histogram, 0, 64 * 4);  // kernel.cu:278
        if (ps.enableHistogram) histogram(io->c64, W64, H64, io->histogram);
        if (ps.enableAutoExposure) {
            auto_exposure(st.exposure, io->histogram, (float)(W64 * H64), io->deltaTime, prm.post.gain);
        } else {
            st.exposure[0] = prm.post.exposure;
            st.exposure[1] = st.exposure[2] = st.exposure[3] = 1.0f;
        }
        if (ps.enableBloomEffect) {
            std::vector<uint16_t> b4s((size_t)W4 * H4 * 4), b16s((size_t)W16 * H16 * 4);
            uint16_t* b4 = io->bloom4 ? io->bloom4 : b4s.data();
            uint16_t* b16 = io->bloom16 ? io->bloom16 : b16s.data();
            bloom_gauss(io->c4, W4, H4, b4, st.exposure[2]);
            bloom_gauss(io->c16, W16, H16, b16, st.exposure[2]);
            bloom_apply(cur, W, H, b4, W4, H4, b16, W16, H16);
        }
        if (ps.enableLensFlare && io->lensFlare) {
            const float d = h2f(io->depth[(size_t)io->sunUv[1] * W + io->sunUv[0]]);  // LensFlarePred
            if (!(d < kRayMaxF)) lens_flare(cur, W, H, F2{io->sunPos[0], io->sunPos[1]});
        }
    }
    bicubic_scale(cur, W, H, io->scaled, Ws, Hs);
    if (ps.enablePostProcess) {
        if (ps.enableSharpening) {
            std::vector<uint16_t> s2((size_t)Ws * Hs * 4);
            sharpen(io->scaled, s2.data(), Ws, Hs);
            memcpy(io->scaled, s2.data(), s2.size() * 2);
        }
        if (ps.enableToneMapping) tonemap(io->scaled, Ws, Hs, st.exposure[0], prm.post.toneMappingType, prm.post);
    }
    if (io->rgba) copy_to_output(io->scaled, Ws, Hs, io->frameNum, io->bluenoise, io->rgba);
    return 0;
}

extern "C" int orc_lens_flare_setup(const OrcCamera* cam, const float* sunDir, uint32_t W, uint32_t H, float* sunPos,
                                    int* sunUv) {
    Camera c;
    camera_update(*cam, c);
    const F3 sd = f3(sunDir[0], sunDir[1], sunDir[2]);
    // Camera::WorldToScreenSpace(pos + sunDir) (kernel.cuh:123-131): rows of the transposed view
    // matrix are left, up, dir
    const F3 d = (c.pos + sd) - c.pos;
    const F3 v = f3(dot(c.left, d), dot(c.up, d), dot(c.dir, d));
    const F2 s = {v.x / v.z, v.y / v.z};
    const F2 ndc = {s.x / c.tanHalfFov.x, s.y / c.tanHalfFov.y};
    F2 sp = {0.5f - ndc.x * 0.5f, 0.5f - ndc.y * 0.5f};
    sunUv[0] = (int)floorf(sp.x * (float)W);
    sunUv[1] = (int)floorf(sp.y * (float)H);
    const int on = sp.x > 0 && sp.x < 1 && sp.y > 0 && sp.y < 1 && sd.y > -0.0f && dot(sd, c.dir) > 0;
    sp = F2{sp.x - 0.5f, sp.y - 0.5f};
    sp.x *= (float)W / (float)H;
    sunPos[0] = sp.x;
    sunPos[1] = sp.y;
    return on;
}
