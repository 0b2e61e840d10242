// denoise.hip — SVGF-style temporal + à-trous denoiser, histogram auto-exposure and the
// post chain (scale, sharpen, tone map, dither to RGBA8) for gfx950.
//
// Pass order and arithmetic follow the reference (denoising.cu:5-189, temporalDenoising.cuh,
// postprocessing.cu:5-161, postprocessing.cuh, kernel.cu:26-59, 376-381).  Differences that
// are deliberate: every filter reads its input from the previous pass's buffer
// and writes a second buffer (the reference filters in place while neighbouring workgroups
// read the same surface), and only in-image pixels are written (the reference's edge threads
// write clamped texels).  Buffer reads clamp to the image edge like CUDA surfaces.
//
// Data layout (render size W x H, screen Ws x Hs), all row-major:
//   colour      uint2  = half r | half g << 16, half b | ushort mask << 16
//   normal      uint2  = half4, albedo uint2 = half4, depth ushort = half, motion uint = half2
//   noise8/16   ushort = half per 8x8 / 16x16 tile
//   c4/c16/c64  uint2  = half4 (DownScale4 chain), histogram uint32[64], exposure float[4]
//   scaled      uint2  = half4 at screen size, rgba uint32 = RGBA8
#include "gaussian_tables.h"
#include "frame_kernels.h"
#include "pt_common.h"
#include "rt_device.h"
#include "rtmath.h"
#include "rtmath_pk.h"

using namespace rtd;

// Wave priority of the denoise/post kernels (s_setprio, 0..3): in a pipelined frame these run
// beside the next frame's path-trace waves on the same SIMDs, and their chain is the frame's
// critical stream: raising it measured 0.887 -> 0.866 ms per 1080p frame (2 and 3 alike).
#ifndef RTX_DN_PRIO
#define RTX_DN_PRIO 3
#endif
#define DN_PRIO() do { if (RTX_DN_PRIO > 0) __builtin_amdgcn_s_setprio(RTX_DN_PRIO); } while (0)

namespace {

constexpr float kRayMaxF = 10e10f;

#define DN_POW(a, b) rt_powf(a, b)
#define DN_EXP(a) rt_expf(a)
// compile-time switches of A/B builds (tools/abl_build.sh "-DRTX_DN_PK=0" ...); the defaults are the product
#ifndef RTX_DN_PK
#define RTX_DN_PK 1
#endif
constexpr bool kDnPk = RTX_DN_PK != 0;  // paired tap weights (rtmath_pk.h)
#ifndef RTX_DN_PKB
#define RTX_DN_PKB 4  // taps per load batch with paired weights (even)
#endif
constexpr int kDnBatch = 5;  // SpatialFilterGlobal5x5 taps per load batch (unpaired)
#define DN5_BOUNDS __launch_bounds__(256)
#ifndef RTX_DN_SPLIT  // ablation builds only: 0 = the list passes at one thread per pixel
#define RTX_DN_SPLIT 1
#endif
constexpr bool kDnSplit = RTX_DN_SPLIT != 0;

// gaussian.cuh:12-43 (double literals converted to float, as the reference's float arrays)
__constant__ float cG3[9] = RT_GAUSS3_INIT;
__constant__ float cG5[25] = RT_GAUSS5_INIT;
__constant__ float cG7[49] = RT_GAUSS7_INIT;

RT_DEV float h2f(uint32_t h) { return rt_h2f((uint16_t)h); }
RT_DEV uint32_t f2h(float f) { return rt_f2h(f); }
RT_DEV int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }
RT_DEV bool isnan3(F3 v) { return v.x != v.x || v.y != v.y || v.z != v.z; }
RT_DEV float clampf(float a, float lo = 0.0f, float hi = 1.0f) { return a < lo ? lo : a > hi ? hi : a; }
RT_DEV F3 clamp3(F3 a, F3 lo, F3 hi) { return f3(clampf(a.x, lo.x, hi.x), clampf(a.y, lo.y, hi.y), clampf(a.z, lo.z, hi.z)); }
RT_DEV F3 fmax3(F3 a, F3 b) { return f3(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z)); }
RT_DEV F3 fmin3(F3 a, F3 b) { return f3(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z)); }
RT_DEV F3 ycocg(F3 c) {
    const float t1 = c.x + c.z, t2 = c.y * 2.0f;
    return f3(t1 + t2, (c.x - c.z) * 2.0f, t2 - t1);
}
RT_DEV F3 ycocg_inv(F3 c) {
    const float t = c.x - c.z;
    return f3(t + c.y, c.x + c.z, t - c.y) * 0.25f;
}

RT_DEV F3 rgb_of(uint2 q) { return f3(h2f(q.x & 0xFFFFu), h2f(q.x >> 16), h2f(q.y & 0xFFFFu)); }
RT_DEV uint32_t mask_of(uint2 q) { return q.y >> 16; }
// rgb_of(q) * w, each product one mixed-precision fma (v_fma_mix_f32, no conversion instruction):
// fmaf(c, w, +0) rounds the exact product once, as the multiply does, and differs from it only
// for a -0 product (+0 then).  Only for sums that start at +0, which are never -0, so that adding
// either zero gives the same sum.
RT_DEV F3 rgb_mul(uint2 q, float w) {
    return f3(__builtin_fmaf(h2f(q.x & 0xFFFFu), w, 0.0f), __builtin_fmaf(h2f(q.x >> 16), w, 0.0f),
              __builtin_fmaf(h2f(q.y & 0xFFFFu), w, 0.0f));
}
RT_DEV uint2 pack_color(F3 c, uint32_t mask) {
    return make_uint2(f2h(c.x) | (f2h(c.y) << 16), f2h(c.z) | (mask << 16));
}

struct View2 {  // clamped reads of a W x H uint2 image
    const uint2* p;
    int W, H;
    RT_DEV uint2 at(int x, int y) const { return p[(size_t)clampi(y, 0, H - 1) * W + clampi(x, 0, W - 1)]; }
};
struct View1 {
    const uint16_t* p;
    int W, H;
    RT_DEV float at(int x, int y) const { return h2f(p[(size_t)clampi(y, 0, H - 1) * W + clampi(x, 0, W - 1)]); }
};

// SampleBicubicSmoothStep: the footprint (first texel, weights) of uv, and the weighted sum of the
// four texels q[i] = im.at(t0x + (i & 1), t0y + (i >> 1)); split so callers can issue the loads early
struct SmoothTaps {
    int t0x, t0y;
    float wt[4];
};
RT_DEV SmoothTaps smooth_taps(const View2& im, F2 uv) {
    const F2 UV = {uv.x * (float)im.W, uv.y * (float)im.H};
    const float fx0 = floorf(UV.x - 0.5f), fy0 = floorf(UV.y - 0.5f);
    const F2 f = {UV.x - (fx0 + 0.5f), UV.y - (fy0 + 0.5f)};
    const F2 f2 = {f.x * f.x, f.y * f.y};
    const F2 f3v = {f2.x * f.x, f2.y * f.y};
    const F2 w1 = {f3v.x * -2.0f + f2.x * 3.0f, f3v.y * -2.0f + f2.y * 3.0f};
    const F2 w0 = {1.0f - w1.x, 1.0f - w1.y};
    return SmoothTaps{(int)fx0, (int)fy0, {w0.x * w0.y, w1.x * w0.y, w0.x * w1.y, w1.x * w1.y}};
}
RT_DEV F3 smooth_sum(const SmoothTaps& t, const uint2* q) {
    F3 o = f3(0.0f);
    float sw = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        sw += t.wt[i];
        o = o + rgb_mul(q[i], t.wt[i]);
    }
    return o / sw;
}
RT_DEV F3 bicubic_smooth(const View2& im, F2 uv) {
    const SmoothTaps t = smooth_taps(im, uv);
    uint2 q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = im.at(t.t0x + (i & 1), t.t0y + (i >> 1));
    return smooth_sum(t, q);
}

// (dV - d) / sigma_depth of pass k (0 TemporalFilter, 1 SpatialFilter7x7, 2 the a-trous passes):
// rt_div_rcp with the launch's reciprocal, the IEEE quotient for every depth difference (0 or
// |a| >= 2^-24, half depths) when the host found sigma in its range; the division otherwise
template <bool kRcp>
RT_DEV float depth_ratio(const DenoisePostParams& P, int k, float a, float sigma) {
    if (kRcp) return rt_div_rcp(a, sigma, P.rcpDepth[k]);
    return a / sigma;
}

// 16-row tile row of this workgroup: launches may cover tile rows [P.ty0, P.ty1) only
// The tile passes' grids are (tiles across, tile rows), in row-major order.  Dealing each XCD a
// contiguous eighth of the tiles instead (so a tile's neighbours share its L2) took TemporalFilter
// 26 -> 54 us and the full-frame a-trous passes 32 -> 105 us (profiles/r05_ab/xcd_tiles/).
RT_DEV int tile_x(const DenoisePostParams&) { return (int)blockIdx.x; }
RT_DEV int tile_y(const DenoisePostParams& P) { return (int)blockIdx.y + P.ty0; }

template <typename T>
RT_DEV T tree_sum32(T v) {
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) v = v + __shfl_down(v, off, 32);
    return v;
}

// TileNoiseLevel8x8 + TileNoiseLevel8x8to16x16 (denoising.cu:73-99) over the 16x16 output tile
// the calling workgroup just produced (sOut, in LDS): threads 0..127 are four 32-lane groups,
// one per 8x8 tile, with k_tile_noise's lane layout and shuffle-tree order; thread 0 then
// averages the four half-rounded tile values into the 16x16 noise level.  Reads outside the
// image clamp to its edge, which always lands inside this workgroup's tile.
RT_DEV float noise_epilogue(const DenoisePostParams& P, const uint2* sOut, uint16_t* sN8, int BX, int TY) {
    const int W = (int)P.W, H = (int)P.H;
    const int W8 = (W + 7) / 8, H8 = (H + 7) / 8, W16 = (W + 15) / 16, H16 = (H + 15) / 16;
    const int tid = threadIdx.x;
    const int x0 = BX * 16, y0 = TY * 16;
    if (tid < 128) {
        const int t = tid >> 5, lane = tid & 31;
        const int tx8 = 2 * BX + (t & 1), ty8 = 2 * TY + (t >> 1);
        const bool valid = tx8 < W8 && ty8 < H8;
        const int x = clampi((valid ? tx8 : 2 * BX) * 8 + (lane & 7), 0, W - 1);
        const int ya = clampi((valid ? ty8 : 2 * TY) * 8 + 2 * (lane >> 3), 0, H - 1);
        const int yb = clampi((valid ? ty8 : 2 * TY) * 8 + 2 * (lane >> 3) + 1, 0, H - 1);
        const F3 ca = rgb_of(sOut[(ya - y0) * 16 + (x - x0)]), cb = rgb_of(sOut[(yb - y0) * 16 + (x - x0)]);
        const uint32_t bg = (h2f(P.depth[(size_t)ya * W + x]) >= kRayMaxF ? 1u : 0u);
        const uint32_t bg2 = (h2f(P.depth[(size_t)yb * W + x]) >= kRayMaxF ? 1u : 0u);
        const float l1 = fmaxf(fmaxf(ca.x, ca.y), ca.z), l2 = fmaxf(fmaxf(cb.x, cb.y), cb.z);
        const uint32_t b1s = tree_sum32(bg), b2s = tree_sum32(bg2);
        const float s1 = tree_sum32(l1), s12 = tree_sum32(l1 * l1), s2 = tree_sum32(l2), s22 = tree_sum32(l2 * l2);
        if (lane == 0) {
            uint16_t h = 0;
            if (valid) {
                const float notSky = 1.0f - (float)(b1s + b2s) / 64.0f;
                const float lumAve = (s1 + s2) / 64.0f;
                const float lumAveSq = lumAve * lumAve;
                const float lumSqAve = (s12 + s22) / 64.0f;
                const float var = fmaxf(1e-20f, lumSqAve - lumAveSq);
                float noise = var / fmaxf(lumAveSq, 1e-20f);
                noise *= notSky;
                h = (uint16_t)f2h(noise);
                P.noise8[ty8 * W8 + tx8] = h;
            }
            sN8[t] = h;
        }
    }
    __syncthreads();
    float n16 = 0.0f;
    if (tid == 0 && BX < W16 && TY < H16) {
        // n8.at(2x + i, 2y + j) clamped to the tile grid: tile i/j falls back to 0 past its edge
        const int i1 = 2 * BX + 1 < W8 ? 1 : 0, j1 = 2 * TY + 1 < H8 ? 2 : 0;
        const float v1 = h2f(sN8[0]), v2 = h2f(sN8[i1]), v3 = h2f(sN8[j1]), v4 = h2f(sN8[i1 + j1]);
        const uint16_t h = (uint16_t)f2h((v1 + v2 + v3 + v4) / 4);
        P.noise16[TY * W16 + BX] = h;
        n16 = h2f(h);
    }
    return n16;  // thread 0: the tile's 16x16 noise level as the passes after it read it
}

// ---- Active-tile lists (the whole-frame chain).  The noise-gated passes
// (SpatialFilter7x7 against noise_threshold_local, the a-trous passes against _large) leave a tile
// below its threshold unchanged, so instead of every pass copying those tiles through its ping-pong
// buffer: TemporalFilter's epilogue sorts each tile by the noise level it just computed — a tile
// above the local threshold goes to list 0 (SpatialFilter7x7 runs only on those), the others write
// their TemporalFilter output straight into this frame's accumulation buffer (SpatialFilter7x7's copy
// of them; the chain alternates two accumulation buffers, since TemporalFilter reads the previous
// frame's) and go to list 1 if they are above the large threshold; SpatialFilter7x7's epilogue puts its tiles
// above the large threshold on list 1.  The first two a-trous passes run only on list 1; the taps of
// the second and third pass that land in a tile off the list read the accumulation buffer (the
// value every copy would have carried), and the third pass, which also applies the albedo, covers
// every tile.
//
// Layout of P.tileList: counters [parity][list][16 partitions] 32 words (128 B) apart (a tile goes
// to partition tile % 16: one device-scope counter per workgroup would serialise), then the entries
// [list][partition][tileCap / 16 + 1].  Each frame appends under its parity and TemporalFilter
// zeroes the other parity's counters, which the previous frame was the last to read.
constexpr int kListParts = 16;
RT_DEV uint32_t* list_counter(const DenoisePostParams& P, int parity, int list, int part) {
    return P.tileList + ((parity * 2 + list) * kListParts + part) * 32;
}
RT_DEV uint32_t list_cap(const DenoisePostParams& P) { return P.tileCap / kListParts + 1; }
RT_DEV uint32_t* list_entries(const DenoisePostParams& P, int list, int part) {
    return P.tileList + 2 * 2 * kListParts * 32 + (list * kListParts + part) * list_cap(P);
}
RT_DEV void list_append(const DenoisePostParams& P, int list, uint32_t tile) {
    const int part = (int)(tile % kListParts);
    const uint32_t i = atomicAdd(list_counter(P, P.tileParity, list, part), 1u);
    list_entries(P, list, part)[i] = tile;
}
// The list kernels launch one workgroup per list slot (16 partitions x (tileCap / 16 + 1), the list's
// capacity): workgroup b takes entry b / 16 of partition b % 16 and leaves at once past that
// partition's count.  A persistent grid walking the list instead held the tap arithmetic's uniform
// values across its loop: 106 SGPRs with spills into VGPR lanes, 145-149 VGPRs against the one-tile
// kernels' 126-129.
RT_DEV bool list_tile(const DenoisePostParams& P, int list, uint32_t& tile) {
    const uint32_t part = blockIdx.x % kListParts, j = blockIdx.x / kListParts;
    if (j >= *list_counter(P, P.tileParity, list, (int)part)) return false;
    tile = list_entries(P, list, (int)part)[j];
    return true;
}

// ------------------------------------------------------------------ TemporalFilter
template <bool kRcp, bool kPk>
RT_DEV uint2 temporal_pixel(const DenoisePostParams& P, const uint2* in, int x, int y);

// kNoise: also the tile noise levels of the output (noise_epilogue); kList: and the tile's place on
// the active-tile lists (above), with the output of a tile SpatialFilter7x7 leaves unchanged also
// written to this frame's accumulation buffer (P.accumAlt: P.accum, the previous frame's, is read
// at reprojected positions by every workgroup); kRcp: the depth weight's division by reciprocal
template <bool kNoise, bool kList, bool kRcp, bool kPk = false>
__global__ __launch_bounds__(256) void k_temporal(DenoisePostParams P, const uint2* in, uint2* out) {
    DN_PRIO();
    __shared__ uint2 sOut[kNoise ? 256 : 1];
    __shared__ uint16_t sN8[4];
    __shared__ int sCopy;
    const int x = tile_x(P) * 16 + (threadIdx.x & 15), y = tile_y(P) * 16 + (threadIdx.x >> 4);
    const int W = (int)P.W, H = (int)P.H;
    if (kList && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 2 * kListParts)  // the other parity's
        *list_counter(P, P.tileParity ^ 1, (int)threadIdx.x / kListParts, (int)threadIdx.x % kListParts) = 0u;
    if (x < W && y < H) {
        const uint2 res = temporal_pixel<kRcp, kPk>(P, in, x, y);
        out[(size_t)y * W + x] = res;
        if (kNoise) sOut[threadIdx.x] = res;
        if (P.histDepthInTemporal) P.histDepth[(size_t)y * W + x] = P.depth[(size_t)y * W + x];
    }
    if (kNoise) {
        __syncthreads();
        const float n16 = noise_epilogue(P, sOut, sN8, tile_x(P), tile_y(P));
        if (kList) {
            if (threadIdx.x == 0) {
                const uint32_t tile = (uint32_t)(tile_y(P) * (int)((P.W + 15) / 16) + tile_x(P));
                const bool act7 = !(n16 < P.dn.noise_threshold_local), act5 = !(n16 < P.dn.noise_threshold_large);
                if (act7) list_append(P, 0, tile);
                else if (act5) list_append(P, 1, tile);
                sCopy = act7 ? 0 : 1;
            }
            __syncthreads();
            if (sCopy && x < W && y < H) P.accumAlt[(size_t)y * W + x] = sOut[threadIdx.x];
        }
    }
}

// TemporalFilter after its spatial taps: the normalised sum, then the reprojected history clamped to
// the neighbourhood's YCoCg box and blended with the pixel
RT_DEV uint2 temporal_tail(const DenoisePostParams& P, const View2& acc, int x, int y, size_t p, F3 filt, float wsum,
                           F3 nMin, F3 nMax, F3 cV, uint32_t mV) {
    const int W = (int)P.W, H = (int)P.H;
    uint2 res;
    if (wsum > 0) filt = filt / wsum;
    else filt = f3(0.0f);
    if (isnan3(filt)) filt = f3(0.0f);
    const uint32_t mvq = P.motion[p];
    const F2 mv = {h2f(mvq & 0xFFFFu) - 0.5f, h2f(mvq >> 16) - 0.5f};
    const F2 inv = {1.0f / (float)W, 1.0f / (float)H};
    const F2 uv = {((float)x + 0.5f) * inv.x, ((float)y + 0.5f) * inv.y};
    const F2 huv = {uv.x + mv.x, uv.y + mv.y};
    if (huv.x < 0 || huv.y < 0 || huv.x > 1.0f || huv.y > 1.0f) {
        res = pack_color(filt, mV);
    } else {
        F3 cH = bicubic_smooth(acc, huv);
        const F3 cHy = clamp3(ycocg(cH), nMin, nMax);
        cH = ycocg_inv(cHy);
        const float lumaMin = nMin.x, lumaMax = nMax.x, lumaC = ycocg(cV).x;
        float discard = 0.0f;
        const int hx = (int)floorf(huv.x * (float)acc.W), hy = (int)floorf(huv.y * (float)acc.H);
#pragma unroll
        for (int i = 0; i < 4; ++i) discard += (mV != mask_of(acc.at(hx + i % 2, hy + i / 2))) ? 1.0f : 0.0f;
        discard /= 4.0f;
        cH = cH * (1.0f - discard) + filt * discard;
        const float lumaH = ycocg(cH).x;
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
        res = pack_color(o, mV);
    }
    return res;
}

// TemporalFilter's weights of taps [kBeg, kEnd) (kBeg even: the pairs are those of the whole set)
template <bool kRcp, bool kPk, int kBeg, int kEnd>
RT_DEV void temporal_weights(const DenoisePostParams& P, F3 nV, float dV, uint32_t mV, bool yOdd, const uint2* qv,
                             const float* dv, const uint2* nq, float* wv) {
#pragma unroll
    for (int j = kBeg; j < kEnd; j += (kPk ? 2 : 1)) {
        if (kPk && j + 1 < kEnd) {  // taps j, j + 1 as one register pair (rtmath_pk.h)
            using rtpk::F2;
            const F3 n0 = rgb_of(nq[j]), n1 = rgb_of(nq[j + 1]);
            const F2 dt = rtpk::inner3_2(nV.x, F2{n0.x, n1.x}, nV.y, F2{n0.y, n1.y}, nV.z, F2{n0.z, n1.z});
            const F2 pw = rtpk::pow_pos2(F2{fmaxf(dt.x, 0.0f), fmaxf(dt.y, 0.0f)},
                                         P.dn.temporal_denoise_sigma_normal, yOdd);
            const F2 dz = F2{dV - dv[j], dV - dv[j + 1]};
            const float sd = P.dn.temporal_denoise_sigma_depth;
            const F2 dd = kRcp ? rtpk::div_rcp2(dz, sd, P.rcpDepth[0]) : F2{dz.x / sd, dz.y / sd};
            const F2 ew = rtpk::expf2((rtpk::splat(-0.5f) * dd) * dd);
            const float mw = 1.0f / P.dn.temporal_denoise_sigma_material;
            F2 w = pw * ew;
            w = w * F2{mV != mask_of(qv[j]) ? mw : 1.0f, mV != mask_of(qv[j + 1]) ? mw : 1.0f};
            w = w * F2{cG3[j], cG3[j + 1]};
            wv[j] = w.x;
            wv[j + 1] = w.y;
        } else {
            const F3 n = rgb_of(nq[j]);
            float w = 1.0f;
            w *= DN_POW(fmaxf(dot(nV, n), 0.0f), P.dn.temporal_denoise_sigma_normal);
            const float dd = depth_ratio<kRcp>(P, 0, dV - dv[j], P.dn.temporal_denoise_sigma_depth);
            w *= DN_EXP(-0.5f * dd * dd);
            w *= (mV != mask_of(qv[j])) ? 1.0f / P.dn.temporal_denoise_sigma_material : 1.0f;
            w *= cG3[j];  // (j % 3) + (j / 3) * 3
            wv[j] = w;
        }
    }
}

template <bool kRcp, bool kPk>
RT_DEV uint2 temporal_pixel(const DenoisePostParams& P, const uint2* in, int x, int y) {
    const int W = (int)P.W, H = (int)P.H;
    const View2 col{in, W, H}, nrm{P.normal, W, H}, acc{P.accum, (int)P.histW, (int)P.histH};
    const View1 dep{P.depth, W, H};
    const size_t p = (size_t)y * W + x;
    const uint2 c0 = in[p];
    uint2 res = c0;
    F3 cV = rgb_of(c0);
    float dV = dep.at(x, y);
    F3 nV = rgb_of(nrm.at(x, y));
    const uint32_t mV = mask_of(c0);
    if (dV != dV) dV = 0.0f;
    if (isnan3(nV)) nV = f3(0.0f);
    const bool yOdd = kPk && rtpk::pow_y_odd(P.dn.temporal_denoise_sigma_normal);
    if (!isnan3(cV) && dV < kRayMaxF) {
        F3 nMax = ycocg(cV), nMin = ycocg(cV);
        F3 filt = f3(0.0f);
        float wsum = 0.0f;
        // the nine taps' loads issued together (see k_spatial5's batches)
        uint2 qv[9], nq[9];
        float dv[9];
#pragma unroll
        for (int j = 0; j < 9; ++j) {
            const int sx = x + j % 3 - 1, sy = y + j / 3 - 1;
            qv[j] = col.at(sx, sy);
            dv[j] = dep.at(sx, sy);
            nq[j] = nrm.at(sx, sy);
        }
        float wv[9];
        temporal_weights<kRcp, kPk, 0, 9>(P, nV, dV, mV, yOdd, qv, dv, nq, wv);
#pragma unroll
        for (int j = 0; j < 9; ++j) {  // the sums in tap order
            const F3 cc = rgb_of(qv[j]);
            const float w = wv[j];
            filt = filt + cc * w;
            wsum += w;
            const F3 nc = ycocg(cc);
            nMax = fmax3(nMax, nc);
            nMin = fmin3(nMin, nc);
        }
        res = temporal_tail(P, acc, x, y, p, filt, wsum, nMin, nMax, cV, mV);
    }
    return res;
}

// ------------------------------------------------------------------ tile noise level
// One 32-lane group per 8x8 tile (two per wave64): lane L = tx + 8*ty covers rows 2ty, 2ty+1.
// Sums use the reference's __shfl_down tree (offsets 16..1) so lane 0 gets its exact order.

__global__ __launch_bounds__(256) void k_tile_noise(DenoisePostParams P, const uint2* color) {
    const int W = (int)P.W, H = (int)P.H;
    const int W8 = (W + 7) / 8, H8 = (H + 7) / 8;
    const int tile = blockIdx.x * 8 + (threadIdx.x >> 5), lane = threadIdx.x & 31;
    const bool valid = tile < W8 * H8;
    const int bx = valid ? tile % W8 : 0, by = valid ? tile / W8 : 0;
    const View2 col{color, W, H};
    const View1 dep{P.depth, W, H};
    const int x = bx * 8 + (lane & 7), ya = by * 8 + 2 * (lane >> 3), yb = ya + 1;
    const F3 ca = rgb_of(col.at(x, ya)), cb = rgb_of(col.at(x, yb));
    const uint32_t bg = (dep.at(x, ya) >= kRayMaxF ? 1u : 0u), bg2 = (dep.at(x, yb) >= kRayMaxF ? 1u : 0u);
    const float l1 = fmaxf(fmaxf(ca.x, ca.y), ca.z), l2 = fmaxf(fmaxf(cb.x, cb.y), cb.z);
    const uint32_t b1s = tree_sum32(bg), b2s = tree_sum32(bg2);
    const float s1 = tree_sum32(l1), s12 = tree_sum32(l1 * l1), s2 = tree_sum32(l2), s22 = tree_sum32(l2 * l2);
    if (lane == 0 && valid) {
        const float notSky = 1.0f - (float)(b1s + b2s) / 64.0f;
        const float lumAve = (s1 + s2) / 64.0f;
        const float lumAveSq = lumAve * lumAve;
        const float lumSqAve = (s12 + s22) / 64.0f;
        const float var = fmaxf(1e-20f, lumSqAve - lumAveSq);
        float noise = var / fmaxf(lumAveSq, 1e-20f);
        noise *= notSky;
        P.noise8[tile] = (uint16_t)f2h(noise);
    }
}

__global__ __launch_bounds__(256) void k_noise16(DenoisePostParams P) {
    const int W8 = ((int)P.W + 7) / 8, H8 = ((int)P.H + 7) / 8, W16 = ((int)P.W + 15) / 16, H16 = ((int)P.H + 15) / 16;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= W16 * H16) return;
    const int x = i % W16, y = i / W16;
    const View1 n8{P.noise8, W8, H8};
    const float v1 = n8.at(2 * x, 2 * y), v2 = n8.at(2 * x + 1, 2 * y), v3 = n8.at(2 * x, 2 * y + 1),
                v4 = n8.at(2 * x + 1, 2 * y + 1);
    P.noise16[i] = (uint16_t)f2h((v1 + v2 + v3 + v4) / 4);
}

// TileNoiseLevelVisualize (debug pass): outline 16x16 tiles above the noise threshold
__global__ __launch_bounds__(256) void k_noise_visualize(DenoisePostParams P, uint2* color, int level) {
    const int x = tile_x(P) * 16 + (threadIdx.x & 15), y = tile_y(P) * 16 + (threadIdx.x >> 4);
    if (x >= (int)P.W || y >= (int)P.H) return;
    const int tx = x & 15, ty = y & 15;
    if (!(tx == 0 || tx == 15 || ty == 0 || ty == 15)) return;
    const int W16 = ((int)P.W + 15) / 16;
    const float thr = level == 1 ? P.dn.noise_threshold_local : P.dn.noise_threshold_large;
    if (!(h2f(P.noise16[(y >> 4) * W16 + (x >> 4)]) > thr)) return;
    const size_t p = (size_t)y * P.W + x;
    color[p] = pack_color(level == 1 ? f3(1.0f, 0.5f, 0.0f) : f3(1.0f, 0.0f, 0.0f), 0xFFFFu);
    P.normal[p] = make_uint2(0u, 0u);
    P.depth[p] = (uint16_t)f2h(kRayMaxF);
}

// ------------------------------------------------------------------ SpatialFilter7x7
// 16x16 tile + 3-pixel apron staged in LDS (22 x 22 entries of colour, normal, depth).
template <int kParity, bool kRcp, bool kPk = false>
RT_DEV uint2 spatial7_pixel(const DenoisePostParams& P, const uint2* sC, const uint2* sN, const float* sD, int tx,
                            int ty);
constexpr int kS7Split = 12;  // SpatialFilter7x7 with two threads per pixel: half 0 takes taps [0, 12)
template <int kParity, bool kRcp, bool kPk>
RT_DEV uint2 spatial7_pixel_split(const DenoisePostParams& P, const uint2* sC, const uint2* sN, const float* sD,
                                  int tx, int ty, int half, bool inside, float* sX);

struct S7Lds {
    uint2 C[22 * 22];
    uint2 N[22 * 22];
    float D[22 * 22];
    uint2 Out[256];
    uint16_t N8[4];
};

// one 16x16 tile (BX, TY) of SpatialFilter7x7 into `out`: the apron staged (when filtered), the
// pixel filtered or copied (gated), the result also kept in L.Out for a noise epilogue
template <bool kRcp, bool kPk = false>
RT_DEV void spatial7_tile(const DenoisePostParams& P, const uint2* in, uint2* out, S7Lds& L, int BX, int TY,
                          bool gated, int lid) {
    const int W = (int)P.W, H = (int)P.H;
    const int tx = lid & 15, ty = lid >> 4;
    const int x = BX * 16 + tx, y = TY * 16 + ty;
    const View2 col{in, W, H}, nrm{P.normal, W, H};
    const View1 dep{P.depth, W, H};
    if (!gated) {
        for (int i = lid; i < 22 * 22; i += 256) {
            const int lx = BX * 16 - 3 + i % 22, ly = TY * 16 - 3 + i / 22;
            L.C[i] = col.at(lx, ly);
            L.N[i] = nrm.at(lx, ly);
            L.D[i] = dep.at(lx, ly);
        }
    }
    __syncthreads();
    if (x < W && y < H) {
        const size_t p = (size_t)y * W + x;
        // the tap set alternates with the frame parity: both sets compiled with constant offsets
        const uint2 res = gated ? in[p]
                          : (P.frameNum % 2 == 0 ? spatial7_pixel<0, kRcp, kPk>(P, L.C, L.N, L.D, tx, ty)
                                                 : spatial7_pixel<1, kRcp, kPk>(P, L.C, L.N, L.D, tx, ty));
        out[p] = res;
        L.Out[lid] = res;
    }
}

template <bool kNoise, bool kRcp>
__global__ __launch_bounds__(256) void k_spatial7(DenoisePostParams P, const uint2* in, uint2* out) {
    DN_PRIO();
    __shared__ S7Lds L;
    const int TY = tile_y(P), W16 = ((int)P.W + 15) / 16;
    const bool gated = h2f(P.noise16[TY * W16 + tile_x(P)]) < P.dn.noise_threshold_local;
    spatial7_tile<kRcp>(P, in, out, L, tile_x(P), TY, gated, (int)threadIdx.x);
    if (kNoise) {
        __syncthreads();
        noise_epilogue(P, L.Out, L.N8, tile_x(P), TY);
    }
}

// SpatialFilter7x7 over active-tile list 0 only (tile rows outside [ty0, ty1) are skipped), with the
// noise epilogue, which puts tiles above the large threshold on list 1
template <bool kRcp, bool kPk = false>
__global__ __launch_bounds__(256) void k_spatial7_list(DenoisePostParams P, const uint2* in, uint2* out) {
    DN_PRIO();
    __shared__ S7Lds L;
    const int W16 = ((int)P.W + 15) / 16;
    uint32_t tile;
    if (!list_tile(P, 0, tile)) return;
    const int BX = (int)(tile % (uint32_t)W16), TY = (int)(tile / (uint32_t)W16);
    if (TY < P.ty0 || TY >= P.ty1) return;
    spatial7_tile<kRcp, kPk>(P, in, out, L, BX, TY, false, (int)threadIdx.x);
    __syncthreads();
    const float n16 = noise_epilogue(P, L.Out, L.N8, BX, TY);
    if (threadIdx.x == 0 && !(n16 < P.dn.noise_threshold_large)) list_append(P, 1, tile);
}

// k_spatial7_list with two threads per pixel (spatial7_pixel_split)
template <bool kRcp, bool kPk>
__global__ __launch_bounds__(512) void k_spatial7_list2(DenoisePostParams P, const uint2* in, uint2* out) {
    DN_PRIO();
    __shared__ S7Lds L;
    __shared__ float sX[(24 - kS7Split) * 256];
    const int W = (int)P.W, H = (int)P.H, W16 = (W + 15) / 16;
    uint32_t tile;
    if (!list_tile(P, 0, tile)) return;
    const int BX = (int)(tile % (uint32_t)W16), TY = (int)(tile / (uint32_t)W16);
    if (TY < P.ty0 || TY >= P.ty1) return;
    const int lid = (int)(threadIdx.x & 255u), half = (int)(threadIdx.x >> 8);
    const int tx = lid & 15, ty = lid >> 4;
    const int x = BX * 16 + tx, y = TY * 16 + ty;
    const View2 col{in, W, H}, nrm{P.normal, W, H};
    const View1 dep{P.depth, W, H};
    for (int i = (int)threadIdx.x; i < 22 * 22; i += 512) {
        const int lx = BX * 16 - 3 + i % 22, ly = TY * 16 - 3 + i / 22;
        L.C[i] = col.at(lx, ly);
        L.N[i] = nrm.at(lx, ly);
        L.D[i] = dep.at(lx, ly);
    }
    __syncthreads();
    const bool inside = x < W && y < H;
    // the tap set alternates with the frame parity: both sets compiled with constant offsets
    const uint2 res = P.frameNum % 2 == 0 ? spatial7_pixel_split<0, kRcp, kPk>(P, L.C, L.N, L.D, tx, ty, half, inside, sX)
                                          : spatial7_pixel_split<1, kRcp, kPk>(P, L.C, L.N, L.D, tx, ty, half, inside, sX);
    if (half == 0 && inside) {
        out[(size_t)y * W + x] = res;
        L.Out[lid] = res;
    }
    __syncthreads();
    const float n16 = noise_epilogue(P, L.Out, L.N8, BX, TY);
    if (threadIdx.x == 0 && !(n16 < P.dn.noise_threshold_large)) list_append(P, 1, tile);
}

// the weight of one SpatialFilter7x7 tap (tap d, n already sanitised)
template <bool kRcp>
RT_DEV float spatial7_weight(const DenoisePostParams& P, F3 nV, float dV, uint32_t mV, uint32_t mq, float d, F3 n,
                             int g) {
    float w = 1.0f;
    w *= DN_POW(fmaxf(dot(nV, n), 0.0001f), P.dn.local_denoise_sigma_normal);
    const float dd = depth_ratio<kRcp>(P, 1, dV - d, P.dn.local_denoise_sigma_depth);
    w *= DN_EXP(-0.5f * dd * dd);
    w *= (mV != mq) ? 1.0f / P.dn.local_denoise_sigma_material : 1.0f;
    w *= cG7[g];
    return w;
}

// two taps' weights as one register pair (spatial5_weight2; the clamped dot is >= 0.0001, so the
// pair pow's zero case never applies)
template <bool kRcp>
RT_DEV rtpk::F2 spatial7_weight2(const DenoisePostParams& P, F3 nV, float dV, uint32_t mV, uint32_t mq0, uint32_t mq1,
                                 float d0, float d1, F3 n0, F3 n1, int g0, int g1) {
    using rtpk::F2;
    const F2 dt = rtpk::inner3_2(nV.x, F2{n0.x, n1.x}, nV.y, F2{n0.y, n1.y}, nV.z, F2{n0.z, n1.z});
    const F2 pw = rtpk::pow_pos2(F2{fmaxf(dt.x, 0.0001f), fmaxf(dt.y, 0.0001f)}, P.dn.local_denoise_sigma_normal, false);
    const F2 dz = F2{dV - d0, dV - d1};
    const float sd = P.dn.local_denoise_sigma_depth;
    const F2 dd = kRcp ? rtpk::div_rcp2(dz, sd, P.rcpDepth[1]) : F2{dz.x / sd, dz.y / sd};
    const F2 ew = rtpk::expf2((rtpk::splat(-0.5f) * dd) * dd);
    const float mw = 1.0f / P.dn.local_denoise_sigma_material;
    F2 w = pw * ew;
    w = w * F2{mV != mq0 ? mw : 1.0f, mV != mq1 ? mw : 1.0f};
    return w * F2{cG7[g0], cG7[g1]};
}

// The centre pixel of SpatialFilter7x7 (NaNs sanitised) and whether it is filtered
struct S7Centre {
    uint2 c0;
    F3 nV;
    float dV;
    uint32_t mV;
    bool filt;
};
RT_DEV S7Centre spatial7_centre(const uint2* sC, const uint2* sN, const float* sD, int tx, int ty) {
    const int ci = (tx + 3) + (ty + 3) * 22;
    S7Centre c;
    c.c0 = sC[ci];
    const F3 cV = rgb_of(c.c0);
    c.dV = sD[ci];
    c.nV = rgb_of(sN[ci]);
    c.mV = mask_of(c.c0);
    if (c.dV != c.dV) c.dV = 0.0f;
    if (isnan3(c.nV)) c.nV = f3(0.0f);
    c.filt = !isnan3(cV) && c.dV < kRayMaxF;
    return c;
}

// Taps i in [kBeg, kEnd) of SpatialFilter7x7 (tap j = kParity + 2i of the 7x7 window), in tap order:
// each tap's sanitised colour and its weight go to sink(i, cc, w).  kBeg is a multiple of 6.
template <int kParity, bool kRcp, bool kPk, int kBeg, int kEnd, class Sink>
RT_DEV void spatial7_taps(const DenoisePostParams& P, const uint2* sC, const uint2* sN, const float* sD, int tx, int ty,
                          const S7Centre& c, Sink&& sink) {
    static_assert(kBeg % 6 == 0 && kEnd % 6 == 0 && kBeg < kEnd && kEnd <= 24, "tap range");
    // LDS reads in batches of six taps (as k_spatial5's loads)
#pragma unroll
    for (int i0 = kBeg; i0 < kEnd; i0 += 6) {
        uint2 qv[6], nq[6];
        float dv[6];
#pragma unroll
        for (int m = 0; m < 6; ++m) {
            const int j = kParity + 2 * (i0 + m);  // P.frameNum % 2 + 2i
            const int li = (tx + j % 7) + (ty + j / 7) * 22;
            qv[m] = sC[li];
            dv[m] = sD[li];
            nq[m] = sN[li];
        }
        F3 cc[6], n[6];
        float d[6], w[6];
#pragma unroll
        for (int m = 0; m < 6; ++m) {
            cc[m] = rgb_of(qv[m]);
            d[m] = dv[m];
            n[m] = rgb_of(nq[m]);
            if (isnan3(cc[m])) cc[m] = f3(0.0f);
            if (d[m] != d[m]) d[m] = 0.0f;
            if (isnan3(n[m])) n[m] = f3(0.0f);
        }
#pragma unroll
        for (int m = 0; m < 6; m += (kPk ? 2 : 1)) {
            const int j = kParity + 2 * (i0 + m), g = j % 7 + (j / 7) * 7;
            if (kPk) {
                const int j1 = j + 2, g1 = j1 % 7 + (j1 / 7) * 7;
                const rtpk::F2 w2 = spatial7_weight2<kRcp>(P, c.nV, c.dV, c.mV, mask_of(qv[m]), mask_of(qv[m + 1]), d[m],
                                                           d[m + 1], n[m], n[m + 1], g, g1);
                w[m] = w2.x;
                w[m + 1] = w2.y;
            } else {
                w[m] = spatial7_weight<kRcp>(P, c.nV, c.dV, c.mV, mask_of(qv[m]), d[m], n[m], g);
            }
        }
#pragma unroll
        for (int m = 0; m < 6; ++m) sink(i0 + m, cc[m], w[m]);
    }
}

RT_DEV uint2 spatial7_finish(F3 sum, float sw, uint32_t mV) {
    if (isnan3(sum)) sum = f3(0.0f);
    if (sw != sw) sw = 0.0f;
    F3 fin = sw == 0 ? f3(0.0f) : sum / sw;
    if (isnan3(fin)) fin = f3(0.0f);
    return pack_color(fin, mV);
}

template <int kParity, bool kRcp, bool kPk>
RT_DEV uint2 spatial7_pixel(const DenoisePostParams& P, const uint2* sC, const uint2* sN, const float* sD, int tx,
                            int ty) {
    const S7Centre c = spatial7_centre(sC, sN, sD, tx, ty);
    if (!c.filt) return c.c0;
    F3 sum = f3(0.0f);
    float sw = 0.0f;
    spatial7_taps<kParity, kRcp, kPk, 0, 24>(P, sC, sN, sD, tx, ty, c, [&](int, F3 cc, float w) {  // the sums in tap order
        sum = sum + cc * w;
        sw += w;
    });
    return spatial7_finish(sum, sw, c.mV);
}

// Two threads per pixel (spatial5_tile_split's scheme): half 0 sums taps 0..11, half 1 leaves taps
// 12..23's weights in LDS (sX), and half 0 adds those taps in order after the barrier, their colours
// read again from the staged apron (the same texels, sanitised the same way)
template <int kParity, bool kRcp, bool kPk>
RT_DEV uint2 spatial7_pixel_split(const DenoisePostParams& P, const uint2* sC, const uint2* sN, const float* sD,
                                  int tx, int ty, int half, bool inside, float* sX) {
    const int lid = ty * 16 + tx;
    const S7Centre c = spatial7_centre(sC, sN, sD, tx, ty);  // in the staged apron for every lane
    const bool filt = inside && c.filt;
    F3 sum = f3(0.0f);
    float sw = 0.0f;
    if (half == 1) {
        if (filt)
            spatial7_taps<kParity, kRcp, kPk, kS7Split, 24>(P, sC, sN, sD, tx, ty, c,
                                                            [&](int i, F3, float w) { sX[(i - kS7Split) * 256 + lid] = w; });
    } else if (filt) {
        spatial7_taps<kParity, kRcp, kPk, 0, kS7Split>(P, sC, sN, sD, tx, ty, c, [&](int, F3 cc, float w) {
            sum = sum + cc * w;
            sw += w;
        });
    }
    __syncthreads();
    if (!filt || half != 0) return c.c0;
#pragma unroll
    for (int i = kS7Split; i < 24; ++i) {
        const int j = kParity + 2 * i;
        F3 cc = rgb_of(sC[(tx + j % 7) + (ty + j / 7) * 22]);
        if (isnan3(cc)) cc = f3(0.0f);
        const float w = sX[(i - kS7Split) * 256 + lid];
        sum = sum + cc * w;
        sw += w;
    }
    return spatial7_finish(sum, sw, c.mV);
}

// ------------------------------------------------------------------ SpatialFilterGlobal5x5<S>
// Tiles of list 1 (above noise_threshold_large) around tile (TX, TY): bit (dy + 2) * 5 + (dx + 2)
// for tile (TX + dx, TY + dy), |dx|, |dy| <= 2 (the reach of a stride-12 tap).  Every wave builds it
// from its own lanes 0..24, so the value is wave-uniform without LDS or a barrier.
RT_DEV uint32_t active_neighbourhood(const DenoisePostParams& P, int TX, int TY) {
    const int lane = (int)(threadIdx.x & 63u);
    const int W16 = ((int)P.W + 15) / 16, H16 = ((int)P.H + 15) / 16;
    const int tx = TX + lane % 5 - 2, ty = TY + lane / 5 - 2;
    bool a = false;
    if (lane < 25 && tx >= 0 && ty >= 0 && tx < W16 && ty < H16)
        a = !(h2f(P.noise16[ty * W16 + tx]) < P.dn.noise_threshold_large);
    return (uint32_t)__ballot(a);
}

// One tap's weight and weighted colour of SpatialFilterGlobal5x5 (the scalar form)
// The a-trous passes' sigmas and depth reciprocal, read from the launch parameters once per pixel
// and passed by value (reading them in each tap's weight, the split kernels had copied them through
// a private array)
struct S5Sig {
    float sn, sd, sm, rcp;
};
RT_DEV S5Sig s5_sig(const DenoisePostParams& P) {
    // uniform values: through readfirstlane, so that no vectorised copy of the triple is formed
    auto u = [](float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
    return S5Sig{u(P.dn.large_denoise_sigma_normal), u(P.dn.large_denoise_sigma_depth),
                 u(P.dn.large_denoise_sigma_material), u(P.rcpDepth[2])};
}

template <bool kRcp>
RT_DEV float spatial5_weight(const S5Sig g, F3 nV, float dV, uint32_t mV, uint2 q, float d, uint2 nq, int k) {
    const F3 n = rgb_of(nq);
    float w = 1.0f;
    w *= DN_POW(fmaxf(dot(nV, n), 0.0f), g.sn);
    const float dd = kRcp ? rt_div_rcp(dV - d, g.sd, g.rcp) : (dV - d) / g.sd;  // depth_ratio of pass 2
    w *= DN_EXP(-0.5f * dd * dd);
    w *= (mV != mask_of(q)) ? 1.0f / g.sm : 1.0f;
    w *= cG5[k];
    return w;
}

// The weights of taps k and k + 1 as one register pair (rtmath_pk.h: the same operations per
// element, the polynomial and compensated-dot chains issued once for both); pow's special cases
// need large_denoise_sigma_normal finite and > 0 (rtpk::pow_pos_ok, checked by the launcher)
template <bool kRcp>
RT_DEV rtpk::F2 spatial5_weight2(const S5Sig g, F3 nV, float dV, uint32_t mV, uint2 q0, uint2 q1, float d0, float d1,
                                 uint2 nq0, uint2 nq1, int k, bool yOdd) {
    using rtpk::F2;
    const F3 n0 = rgb_of(nq0), n1 = rgb_of(nq1);
    const F2 dt = rtpk::inner3_2(nV.x, F2{n0.x, n1.x}, nV.y, F2{n0.y, n1.y}, nV.z, F2{n0.z, n1.z});
    const F2 pw = rtpk::pow_pos2(F2{fmaxf(dt.x, 0.0f), fmaxf(dt.y, 0.0f)}, g.sn, yOdd);
    const F2 dz = F2{dV - d0, dV - d1};
    const float sd = g.sd;
    const F2 dd = kRcp ? rtpk::div_rcp2(dz, sd, g.rcp) : F2{dz.x / sd, dz.y / sd};
    const F2 ew = rtpk::expf2((rtpk::splat(-0.5f) * dd) * dd);
    const float mw = 1.0f / g.sm;
    F2 w = pw * ew;
    w = w * F2{mV != mask_of(q0) ? mw : 1.0f, mV != mask_of(q1) ? mw : 1.0f};
    return w * F2{cG5[k], cG5[k + 1]};
}

// the texel of tap k (clamped; kRedirect: `alt` outside the list-1 tiles of `act`)
template <int S, bool kRedirect>
RT_DEV const uint2* spatial5_tap_src(const DenoisePostParams& P, const uint2* in, const uint2* alt, uint32_t act, int x,
                                     int y, int TX, int TY, int k, size_t& q) {
    const int W = (int)P.W, H = (int)P.H;
    const int cx = clampi(x + (k % 5 - 2) * S, 0, W - 1), cy = clampi(y + (k / 5 - 2) * S, 0, H - 1);
    q = (size_t)cy * W + cx;
    if (!kRedirect) return in;
    const int bit = ((cy >> 4) - TY + 2) * 5 + ((cx >> 4) - TX + 2);
    return ((act >> bit) & 1u) ? in : alt;
}

// Taps [kBeg, kEnd) of SpatialFilterGlobal5x5<S> around pixel (x, y) of a filtered tile (TX, TY), in
// tap order: each tap's colour and weight, after the NaN rule, go to sink(k, cc, w).  kRedirect: `in`
// holds only the list-1 tiles, so a tap whose (clamped) texel lies in a tile off the list (its bit
// clear in `act`) reads `alt`, the accumulation buffer those tiles would have been copied from.  kPk:
// tap weights two at a time (spatial5_weight2), batches of RTX_DN_PKB taps; kBeg is even.
template <int S, bool kRcp, bool kRedirect, bool kPk, int kBeg, int kEnd, class Sink>
RT_DEV void spatial5_taps(const DenoisePostParams& P, const uint2* in, const uint2* alt, uint32_t act, int x, int y,
                          int TX, int TY, F3 nV, float dV, uint32_t mV, bool yOdd, const S5Sig g, Sink&& sink) {
    static_assert(kBeg % 2 == 0 && kBeg < kEnd && kEnd <= 25, "tap range");
    constexpr int kB = kPk ? RTX_DN_PKB : kDnBatch;
    // taps in batches of kB: a batch's loads are issued together, then its weights computed
    // (the branches of rt_powf otherwise keep the compiler from hoisting the next tap's loads,
    // one memory round trip per tap)
#pragma unroll
    for (int k0 = kBeg; k0 < kEnd; k0 += kB) {
        uint2 qv[kB], nq[kB];
        float dv[kB];
#pragma unroll
        for (int m = 0; m < kB; ++m) {
            const int k = k0 + m < kEnd ? k0 + m : kEnd - 1;
            size_t q;
            const uint2* src = spatial5_tap_src<S, kRedirect>(P, in, alt, act, x, y, TX, TY, k, q);
            qv[m] = src[q];
            dv[m] = h2f(P.depth[q]);
            nq[m] = P.normal[q];
        }
        float wv[kB];
#pragma unroll
        for (int m = 0; m < kB; ++m) {
            const int k = k0 + m;
            if (k >= kEnd) break;
            if (kPk && m % 2 == 0 && k + 1 < kEnd && m + 1 < kB) {
                const rtpk::F2 w2 = spatial5_weight2<kRcp>(g, nV, dV, mV, qv[m], qv[m + 1], dv[m], dv[m + 1],
                                                           nq[m], nq[m + 1], k, yOdd);
                wv[m] = w2.x;
                wv[m + 1] = w2.y;
            } else if (!kPk || m % 2 == 0) {
                wv[m] = spatial5_weight<kRcp>(g, nV, dV, mV, qv[m], dv[m], nq[m], k);
            }
        }
#pragma unroll
        for (int m = 0; m < kB; ++m) {
            if (k0 + m >= kEnd) break;
            F3 cc = rgb_of(qv[m]);
            float w = wv[m];
            if (isnan3(cc)) { cc = f3(0.0f); w = 0.0f; }
            sink(k0 + m, cc, w);
        }
    }
}

// The centre pixel's values SpatialFilterGlobal5x5 weighs its taps against (NaNs sanitised)
struct S5Centre {
    uint2 c0;
    F3 nV;
    float dV;
    uint32_t mV;
};
RT_DEV S5Centre spatial5_centre(const DenoisePostParams& P, const uint2* in, size_t p) {
    S5Centre c;
    c.c0 = in[p];
    c.nV = rgb_of(P.normal[p]);
    c.mV = mask_of(c.c0);
    c.dV = h2f(P.depth[p]);
    if (c.dV != c.dV) c.dV = 0.0f;
    if (isnan3(c.nV)) c.nV = f3(0.0f);
    return c;
}
// the filtered pixel from the tap sums
RT_DEV uint2 spatial5_finish(F3 sum, float sw, uint32_t mV) {
    if (isnan3(sum)) sum = f3(0.0f);
    if (sw != sw) sw = 0.0f;
    F3 fin = sw == 0 ? f3(0.0f) : sum / sw;
    if (isnan3(fin)) fin = f3(0.0f);
    return pack_color(fin, mV);
}

// One pixel of SpatialFilterGlobal5x5<S> in a filtered tile (TX, TY): the 25 taps summed in tap order
template <int S, bool kRcp, bool kRedirect, bool kPk = false>
RT_DEV uint2 spatial5_pixel(const DenoisePostParams& P, const uint2* in, const uint2* alt, uint32_t act, int x, int y,
                            int TX, int TY) {
    const S5Centre c = spatial5_centre(P, in, (size_t)y * P.W + x);
    if (!(c.dV < 10e9f)) return c.c0;
    const bool yOdd = kPk && rtpk::pow_y_odd(P.dn.large_denoise_sigma_normal);
    F3 sum = f3(0.0f);
    float sw = 0.0f;
    spatial5_taps<S, kRcp, kRedirect, kPk, 0, 25>(P, in, alt, act, x, y, TX, TY, c.nV, c.dV, c.mV, yOdd, s5_sig(P),
                                                   [&](int, F3 cc, float w) {
                                                       sum = sum + cc * w;
                                                       sw += w;
                                                   });
    return spatial5_finish(sum, sw, c.mV);
}

// Two threads per pixel (a 512-thread workgroup per 16x16 tile), for the passes that filter only
// the tiles of a short list: half 0 sums taps 0..11 in order, half 1 computes the weights of taps
// 12..24 and leaves them in LDS, and half 0 — which loads those taps' texels again while it waits at
// the barrier — adds them in order after it: the same products and the same sums in the same order
// as spatial5_pixel, on twice the waves (a list pass's few tiles otherwise leave ~2 waves per SIMD
// to cover the taps' latency), with 4 bytes of LDS per tap.
constexpr int kS5Split = 12;  // half 0: taps [0, kS5Split)
template <int S, bool kRcp, bool kRedirect, bool kPk>
RT_DEV void spatial5_tile_split(const DenoisePostParams& P, const uint2* in, const uint2* alt, uint2* out, uint32_t act,
                                int TX, int TY, float* sX, bool albedo) {
    const int W = (int)P.W, H = (int)P.H;
    const int lid = (int)(threadIdx.x & 255u), half = (int)(threadIdx.x >> 8);
    const int x = TX * 16 + (lid & 15), y = TY * 16 + (lid >> 4);
    const bool inside = x < W && y < H;
    const size_t p = (size_t)y * W + x;
    // read at the clamped pixel outside the image (no lane keeps it), so the centre is never a
    // conditionally initialised aggregate (which the compiler had put in scratch)
    const S5Centre c = spatial5_centre(P, in, (size_t)(y < H ? y : H - 1) * W + (x < W ? x : W - 1));
    const bool filt = inside && c.dV < 10e9f;
    const bool yOdd = kPk && rtpk::pow_y_odd(P.dn.large_denoise_sigma_normal);
    F3 sum = f3(0.0f);
    float sw = 0.0f;
    if (half == 1) {
        if (filt)
            spatial5_taps<S, kRcp, kRedirect, kPk, kS5Split, 25>(
                P, in, alt, act, x, y, TX, TY, c.nV, c.dV, c.mV, yOdd, s5_sig(P),
                [&](int k, F3, float w) { sX[(k - kS5Split) * 256 + lid] = w; });
    }
    uint2 qv[25 - kS5Split];
    if (half == 0 && filt) {
        spatial5_taps<S, kRcp, kRedirect, kPk, 0, kS5Split>(P, in, alt, act, x, y, TX, TY, c.nV, c.dV, c.mV, yOdd, s5_sig(P),
                                                             [&](int, F3 cc, float w) {
                                                                 sum = sum + cc * w;
                                                                 sw += w;
                                                             });
#pragma unroll
        for (int k = kS5Split; k < 25; ++k) {
            size_t q;
            const uint2* src = spatial5_tap_src<S, kRedirect>(P, in, alt, act, x, y, TX, TY, k, q);
            qv[k - kS5Split] = src[q];
        }
    }
    __syncthreads();
    if (half != 0 || !inside) return;
    uint2 res = c.c0;
    if (filt) {
#pragma unroll
        for (int k = kS5Split; k < 25; ++k) {  // spatial5_taps' sink for these taps
            F3 cc = rgb_of(qv[k - kS5Split]);
            float w = sX[(k - kS5Split) * 256 + lid];
            if (isnan3(cc)) { cc = f3(0.0f); w = 0.0f; }
            sum = sum + cc * w;
            sw += w;
        }
        res = spatial5_finish(sum, sw, c.mV);
    }
    if (albedo) res = pack_color(rgb_of(res) * rgb_of(P.albedo[p]), 0x3C00u);  // w = half(1.0)
    out[p] = res;
}

// every tile of the launch's rows: tiles below the large threshold pass their input through (from
// `alt` when kRedirect: `in` holds only the list-1 tiles); kAlbedo: ApplyAlbedo (denoising.cu:160-171)
// fused into the store of the last wide pass
template <int S, bool kAlbedo, bool kRcp, bool kRedirect, bool kPk = false>
__global__ DN5_BOUNDS void k_spatial5(DenoisePostParams P, const uint2* in, uint2* out, const uint2* alt) {
    DN_PRIO();
    const int W = (int)P.W, H = (int)P.H;
    const int TX = tile_x(P), TY = tile_y(P);
    const int x = TX * 16 + (threadIdx.x & 15), y = TY * 16 + (threadIdx.x >> 4);
    const int W16 = (W + 15) / 16;
    const bool active = !(h2f(P.noise16[TY * W16 + TX]) < P.dn.noise_threshold_large);
    uint32_t act = 0u;
    if (kRedirect && active) act = active_neighbourhood(P, TX, TY);  // before any lane leaves
    if (x >= W || y >= H) return;
    const size_t p = (size_t)y * W + x;
    uint2 res = active ? spatial5_pixel<S, kRcp, kRedirect, kPk>(P, in, alt, act, x, y, TX, TY) : (kRedirect ? alt : in)[p];
    if (kAlbedo) res = pack_color(rgb_of(res) * rgb_of(P.albedo[p]), 0x3C00u);  // w = half(1.0)
    out[p] = res;
}

// ApplyAlbedo over `alt` into `out` for tile b of rows [P.cty0, P.cty1) when it is off list 1 (kCopy
// of the list kernels below: what the last a-trous pass would pass through for that tile)
RT_DEV void copy_off_list_tile(const DenoisePostParams& P, const uint2* alt, uint2* out, int W, int H, int W16) {
    const uint32_t t = (uint32_t)P.cty0 * (uint32_t)W16 + blockIdx.x;
    const int CX = (int)(t % (uint32_t)W16), CY = (int)(t / (uint32_t)W16);
    if (CY < P.cty1 && h2f(P.noise16[t]) < P.dn.noise_threshold_large) {
        const int x = CX * 16 + (int)(threadIdx.x & 15u), y = CY * 16 + (int)(threadIdx.x >> 4);
        if (x < W && y < H) {
            const size_t p = (size_t)y * W + x;
            out[p] = pack_color(rgb_of(alt[p]) * rgb_of(P.albedo[p]), 0x3C00u);  // w = half(1.0)
        }
    }
}

// SpatialFilterGlobal5x5<S> over active-tile list 1 only (tile rows outside [ty0, ty1) are skipped):
// `out` is written in those tiles only.  kAlbedo / kCopy: as k_spatial5_list2 below
template <int S, bool kRcp, bool kRedirect, bool kPk = false, bool kAlbedo = false, bool kCopy = false>
__global__ DN5_BOUNDS void k_spatial5_list(DenoisePostParams P, const uint2* in, uint2* out, const uint2* alt) {
    DN_PRIO();
    const int W = (int)P.W, H = (int)P.H, W16 = (W + 15) / 16;
    if (kCopy) copy_off_list_tile(P, alt, out, W, H, W16);
    uint32_t tile;
    if (!list_tile(P, 1, tile)) return;
    const int TX = (int)(tile % (uint32_t)W16), TY = (int)(tile / (uint32_t)W16);
    if (TY < P.ty0 || TY >= P.ty1) return;
    const uint32_t act = kRedirect ? active_neighbourhood(P, TX, TY) : 0u;
    const int x = TX * 16 + (threadIdx.x & 15), y = TY * 16 + (threadIdx.x >> 4);
    if (x < W && y < H) {
        uint2 res = spatial5_pixel<S, kRcp, kRedirect, kPk>(P, in, alt, act, x, y, TX, TY);
        const size_t p = (size_t)y * W + x;
        if (kAlbedo) res = pack_color(rgb_of(res) * rgb_of(P.albedo[p]), 0x3C00u);  // w = half(1.0)
        out[p] = res;
    }
}

// k_spatial5_list with two threads per pixel (spatial5_tile_split).  kAlbedo: the last a-trous pass
// (ApplyAlbedo fused into its store).  kCopy: the first one, which also writes the last pass's output
// for the tiles off list 1 — ApplyAlbedo over the accumulation buffer (`alt`), what the last pass
// would pass through for them — workgroup b for tile b of rows [P.cty0, P.cty1): list 1 is final
// once SpatialFilter7x7 has run, and no a-trous pass reads `out` outside list-1 tiles (their taps
// there read `alt`), so those tiles need no pass of their own after the list passes.
template <int S, bool kRcp, bool kRedirect, bool kPk, bool kAlbedo = false, bool kCopy = false>
__global__ __launch_bounds__(512) void k_spatial5_list2(DenoisePostParams P, const uint2* in, uint2* out, const uint2* alt) {
    DN_PRIO();
    __shared__ float sX[(25 - kS5Split) * 256];
    const int W = (int)P.W, H = (int)P.H, W16 = (W + 15) / 16;
    if (kCopy && threadIdx.x < 256) copy_off_list_tile(P, alt, out, W, H, W16);
    uint32_t tile;
    if (!list_tile(P, 1, tile)) return;
    const int TX = (int)(tile % (uint32_t)W16), TY = (int)(tile / (uint32_t)W16);
    if (TY < P.ty0 || TY >= P.ty1) return;
    const uint32_t act = kRedirect ? active_neighbourhood(P, TX, TY) : 0u;
    spatial5_tile_split<S, kRcp, kRedirect, kPk>(P, in, alt, out, act, TX, TY, sX, kAlbedo);
}

// ------------------------------------------------------------------ ApplyAlbedo (in place, pointwise)
__global__ __launch_bounds__(256) void k_apply_albedo(DenoisePostParams P, const uint2* in, uint2* out) {
    const size_t p = (size_t)P.ty0 * 16 * P.W + (size_t)blockIdx.x * 256 + threadIdx.x;  // rows of tiles ty0..
    if (p >= (size_t)P.W * P.H || p >= (size_t)P.ty1 * 16 * P.W) return;
    const F3 c = rgb_of(in[p]);
    const F3 a = rgb_of(P.albedo[p]);
    out[p] = pack_color(c * a, 0x3C00u);  // w = half(1.0)
}

// ------------------------------------------------------------------ post
struct H4 { float x, y, z, w; };
RT_DEV H4 h4_of(uint2 q) { return H4{h2f(q.x & 0xFFFFu), h2f(q.x >> 16), h2f(q.y & 0xFFFFu), h2f(q.y >> 16)}; }
RT_DEV H4 add4(H4 a, H4 b) { return H4{a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
RT_DEV uint2 pack_h4(H4 v) { return make_uint2(f2h(v.x) | (f2h(v.y) << 16), f2h(v.z) | (f2h(v.w) << 16)); }

// DownScale4: output texel = 4x4 box of inputs, summed as the reference's 2x2-of-2x2 tree
template <class Img>
RT_DEV uint2 down4(const Img& im, int ox, int oy) {
    H4 q[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            H4 s[2][2];
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int v = 0; v < 2; ++v) {
                    const H4 t = h4_of(im.at(4 * ox + 2 * a + u, 4 * oy + 2 * b + v));
                    s[u][v] = H4{t.x / 16, t.y / 16, t.z / 16, t.z / 16};  // Float4::operator/ (linearMath.h:423)
                }
            q[a][b] = add4(add4(add4(s[0][0], s[1][0]), s[0][1]), s[1][1]);
        }
    return pack_h4(add4(add4(add4(q[0][0], q[1][0]), q[0][1]), q[1][1]));
}

// output rows [oy0, oy1) only (a strip-local denoise computes its own rows)
__global__ __launch_bounds__(256) void k_downscale4(const uint2* in, int Wi, int Hi, uint2* out, int Wo, int Ho,
                                                    int oy0, int oy1) {
    int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= Wo * (oy1 - oy0)) return;
    const int ox = i % Wo, oy = oy0 + i / Wo;
    if (oy >= Ho) return;
    out[oy * Wo + ox] = down4(View2{in, Wi, Hi}, ox, oy);
}

// Histogram2's bin of one 1/64 texel
RT_DEV uint32_t histogram_bin(uint2 q) {
    const H4 v = h4_of(q);
    const float lum = dot(f3(v.x, v.y, v.z), f3((float)0.3, (float)0.6, (float)0.1));
    const float logL = (float)((double)rt_log2f(lum) * 0.1 + 0.75);
    const float sc = (float)((double)(clampf(logL, 0.0f, 1.0f) * 63) * 0.99999);
    return (uint32_t)rintf(sc);
}

// Histogram2: one 32x32 workgroup over the top-left min(W64,32) x min(H64,32) texels
// y0 / y1: the texel rows of this (strip-local) count; the ranks' counts are summed afterwards
__global__ __launch_bounds__(1024) void k_histogram(const uint2* c64, int W64, int H64, uint32_t* hist, int y0, int y1) {
    __shared__ uint32_t h[64];
    if (threadIdx.x < 64) h[threadIdx.x] = 0u;
    __syncthreads();
    const int x = threadIdx.x & 31, y = threadIdx.x >> 5;
    const int tw = W64 < 32 ? W64 : 32, th = H64 < 32 ? H64 : 32;
    if (x < tw && y < th && y >= y0 && y < y1) atomicAdd(&h[histogram_bin(c64[y * W64 + x])], 1u);
    __syncthreads();
    if (threadIdx.x < 64) hist[threadIdx.x] = h[threadIdx.x];
}

RT_DEV float bin_to_lum(int i) { return rt_exp2f((float)(((double)(float)i / (63 * 0.99999) - 0.75) / 0.1)); }

// AutoExposure (postprocessing.cu:5-44) by the first wave of the workgroup (the caller's threads
// 0..63 all call it): lane i evaluates bin i's share and luminance, then every lane walks the
// bins in order with the reference's running sums, reading bin i from lane i (v_readlane, no
// memory round trip per bin), and lane 0 stores the state.
RT_DEV void auto_exposure_wave(float* e, const uint32_t* hist, float area, float deltaTime, float gain, int enabled,
                               float fixedExposure) {
    const int lane = (int)threadIdx.x;
    if (!enabled) {
        if (lane == 0) {
            e[0] = fixedExposure;
            e[1] = e[2] = e[3] = 1.0f;
        }
        return;
    }
    const float myFh = (float)hist[lane] / area, myLum = bin_to_lum(lane);
    auto fh = [&](int i) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(myFh), i)); };
    auto lumOf = [&](int i) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(myLum), i)); };
    const float darkT = (float)0.4, brightT = (float)0.9;
    float lumiSum = 0, lumiSumArea = 0, accu = 0, brightLum = 0;
    int i = 0;
    for (; i < 64; ++i) {
        const float fHist = fh(i);
        accu += fHist;
        const float dark = accu - darkT;
        if (dark > 0) {
            lumiSumArea += dark;
            lumiSum += dark * lumOf(i);
            break;
        }
    }
    for (; i < 64; ++i) {
        const float fHist = fh(i);
        const float lum = lumOf(i);
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
    if (lane != 0) return;
    float aveLum = clampf(lumiSum / lumiSumArea, 0.1f, 100.0f);
    float lumTemp = e[1], lumBright = e[2];
    const float k = 1.0f - rt_expf(-deltaTime * 0.001f);
    lumTemp = lumTemp + (aveLum - lumTemp) * k;
    lumBright = lumBright + (brightLum - lumBright) * k;
    const float EC = 1.03f - 2.0f / (rt_log10f(lumTemp + 1.0f) + 2.0f);
    e[0] = gain * EC / lumTemp;
    e[1] = lumTemp;
    e[2] = lumBright;
    e[3] = brightLum;
}

__global__ __launch_bounds__(64) void k_auto_exposure(float* e, const uint32_t* hist, float area, float deltaTime,
                                                      float gain, int enabled, float fixedExposure) {
    auto_exposure_wave(e, hist, area, deltaTime, gain, enabled, fixedExposure);
}

// DownScale4 x 3 + Histogram2 + AutoExposure in one launch (full frame, every pass enabled).
// Workgroup (X, Y) of the W64 x H64 grid takes the 64x64 render block under 1/64 texel (X, Y): its
// 16x16 quarter texels (one per thread, from the colour), 4x4 sixteenth texels and the 1/64 texel
// from LDS, each level's clamped reads landing inside the block (the level's last texel is in the
// block that covers the edge).  The last workgroup to finish — a device-scope counter, the 1/64
// texels published with agent-coherent stores — counts the histogram over the 1/64 image and
// runs the exposure update, and re-arms the counter.
struct LdsLevel {  // clamped reads of an image level, of the block staged in LDS
    const uint2* s;
    int W, H, x0, y0, pitch;
    RT_DEV uint2 at(int x, int y) const {
        return s[(clampi(y, 0, H - 1) - y0) * pitch + (clampi(x, 0, W - 1) - x0)];
    }
};

// ------------------------------------------------------------------ TemporalFilter2
RT_DEV uint2 temporal2_pixel(const DenoisePostParams& P, const uint2* in, int x, int y) {
    const int W = (int)P.W, H = (int)P.H;
    const size_t p = (size_t)y * W + x;
    const View2 col{in, W, H}, hc{P.histColor, (int)P.histW, (int)P.histH};
    // Loads in two batches — the 3x3 neighbourhood with the motion vector, then the history texels
    // it points at — and the reference's early-outs (history off screen, every history texel of
    // another material) as one select of the output.  Written as branches, the compiler split each
    // neighbour load into a mask read and a dependent colour read and sank the history reads below
    // the discard test: ~13 dependent round trips per pixel instead of 2.
    uint2 qs[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) qs[j] = col.at(x + j % 3 - 1, y + j / 3 - 1);  // qs[4]: the pixel
    const uint32_t mvq = P.motion[p];
    const F2 mv = {h2f(mvq & 0xFFFFu) - 0.5f, h2f(mvq >> 16) - 0.5f};
    const F2 inv = {1.0f / (float)W, 1.0f / (float)H};
    const F2 uv = {((float)x + 0.5f) * inv.x, ((float)y + 0.5f) * inv.y};
    const F2 huv = {uv.x + mv.x, uv.y + mv.y};
    const bool onScreen = !(huv.x < 0 || huv.y < 0 || huv.x > 1.0f || huv.y > 1.0f);
    const SmoothTaps ht = smooth_taps(hc, huv);  // clamped reads: safe off screen too
    const int hx = (int)floorf(huv.x * (float)hc.W), hy = (int)floorf(huv.y * (float)hc.H);
    uint2 hq[4];
    uint32_t hm[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        hq[i] = hc.at(ht.t0x + (i & 1), ht.t0y + (i >> 1));
        hm[i] = mask_of(hc.at(hx + i % 2, hy + i / 2));
    }
    const uint2 c0 = qs[4];
    const F3 cV = ycocg_inv(ycocg(rgb_of(c0)));
    const int mV = (int)mask_of(c0);
    const float FLTMIN = 1.17549435e-38f, FLTMAX = 3.402823466e+38f;
    F3 nMax = f3(FLTMIN), nMin = f3(FLTMAX), nMax2 = f3(FLTMIN), nMin2 = f3(FLTMAX);
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        const int xo = j % 3, yo = j / 3;
        const bool same = (int)mask_of(qs[j]) == mV;
        // a tap of another material enters the bounds as NaN, which fmaxf / fminf (IEEE maxNum /
        // minNum, v_max_f32 / v_min_f32) pass over: the reference's `same ? fmax(b, c) : b` with one
        // select per channel instead of one per bound and channel (the bounds are never NaN)
        const F3 cc = ycocg(rgb_of(qs[j]));
        const float qn = __builtin_nanf("");
        const F3 cs = same ? cc : f3(qn);
        nMax = fmax3(nMax, cs);
        nMin = fmin3(nMin, cs);
        if (abs(xo - 1) + abs(yo - 1) <= 1) {
            nMax2 = fmax3(nMax2, cs);
            nMin2 = fmin3(nMin2, cs);
        }
    }
    nMax = (nMax + nMax2) / 2.0f;
    nMin = (nMin + nMin2) / 2.0f;
    F3 cH = smooth_sum(ht, hq);
    const F3 cHy = clamp3(ycocg(cH), nMin, nMax);
    cH = ycocg_inv(cHy);
    const float lumaMin = nMin.x, lumaMax = nMax.x, lumaC = ycocg(cV).x;
    float discard = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) discard += (mV != (int)hm[i]) ? 1.0f : 0.0f;
    discard /= 4.0f;
    cH = cH * (1.0f - discard) + cV * discard;
    const float lumaH = ycocg(cH).x;
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
    const uint2 blended = pack_color(o, (uint32_t)mV & 0xFFFFu);
    return onScreen && discard != 1.0f ? blended : c0;
}

// kDown: also DownScale4's first level of the tile (its 4 x 4 quarter texels, each a 4 x 4 box that
// lies inside the 16 x 16 tile, clamped reads included), so the downscale chain starts from c4
template <bool kDown>
__global__ __launch_bounds__(256) void k_temporal2(DenoisePostParams P, const uint2* in, uint2* out) {
    DN_PRIO();
    __shared__ uint2 sT[kDown ? 256 : 1];
    const int W = (int)P.W, H = (int)P.H;
    const int x = tile_x(P) * 16 + (threadIdx.x & 15), y = tile_y(P) * 16 + (threadIdx.x >> 4);
    if (x < W && y < H) {
        const uint2 r = temporal2_pixel(P, in, x, y);
        out[(size_t)y * W + x] = r;
        if (kDown) sT[threadIdx.x] = r;
    }
    if (kDown) {
        __syncthreads();
        const int t = (int)threadIdx.x, W4 = (W + 3) / 4, H4 = (H + 3) / 4;
        const int ox = tile_x(P) * 4 + (t & 3), oy = tile_y(P) * 4 + (t >> 2);
        if (t < 16 && ox < W4 && oy < H4)
            P.c4[oy * W4 + ox] = down4(LdsLevel{sT, W, H, tile_x(P) * 16, tile_y(P) * 16, 16}, ox, oy);
    }
}


// kFromC4: TemporalFilter2 already wrote the first level (k_temporal2<true>)
template <bool kFromC4>
__global__ __launch_bounds__(256) void k_downscale_chain(DenoisePostParams P, const uint2* in, uint32_t* counter) {
    DN_PRIO();
    __shared__ uint2 s4[16 * 16];
    __shared__ uint2 s16[4 * 4];
    __shared__ uint32_t sHist[64];
    __shared__ int sLast;
    const int W = (int)P.W, H = (int)P.H;
    const int W4 = (W + 3) / 4, H4 = (H + 3) / 4, W16 = (W4 + 3) / 4, H16 = (H4 + 3) / 4, W64 = (W16 + 3) / 4,
              H64 = (H16 + 3) / 4;
    const int X = (int)blockIdx.x, Y = (int)blockIdx.y, t = (int)threadIdx.x;
    {
        const int ox = X * 16 + (t & 15), oy = Y * 16 + (t >> 4);
        if (ox < W4 && oy < H4) {
            if (kFromC4) {
                s4[t] = P.c4[oy * W4 + ox];
            } else {
                const uint2 v = down4(View2{in, W, H}, ox, oy);
                s4[t] = v;
                P.c4[oy * W4 + ox] = v;
            }
        }
    }
    __syncthreads();
    if (t < 16) {
        const int ox = X * 4 + (t & 3), oy = Y * 4 + (t >> 2);
        if (ox < W16 && oy < H16) {
            const uint2 v = down4(LdsLevel{s4, W4, H4, X * 16, Y * 16, 16}, ox, oy);
            s16[t] = v;
            P.c16[oy * W16 + ox] = v;
        }
    }
    __syncthreads();
    if (t == 0) {
        // the 1/64 texel handed to the last workgroup through rt_device.h's xwg_* (agent-coherent
        // store, then the count; no release fence: on gfx950 that writes back and invalidates the
        // XCD's whole L2, once per workgroup); the last one takes one acquire
        const uint2 v = down4(LdsLevel{s16, W16, H16, X * 4, Y * 4, 4}, X, Y);
        xwg_store((unsigned long long*)&P.c64[Y * W64 + X], ((unsigned long long)v.y << 32) | v.x);
        const bool last = xwg_arrive(counter) == gridDim.x * gridDim.y - 1;
        if (last) xwg_acquire();
        sLast = last;
    }
    __syncthreads();
    if (!sLast) return;
    if (t < 64) sHist[t] = 0u;
    __syncthreads();
    const int tw = W64 < 32 ? W64 : 32, th = H64 < 32 ? H64 : 32;
    for (int i = t; i < 32 * 32; i += 256) {
        const int x = i & 31, y = i >> 5;
        if (x < tw && y < th) {
            const unsigned long long q = xwg_load((const unsigned long long*)&P.c64[y * W64 + x]);
            atomicAdd(&sHist[histogram_bin(make_uint2((uint32_t)q, (uint32_t)(q >> 32)))], 1u);
        }
    }
    __syncthreads();
    if (t < 64) {
        P.histogram[t] = sHist[t];
        if (t == 0) *counter = 0u;
        if (P.postProcess)
            auto_exposure_wave(P.exposure, sHist, (float)(W64 * H64), P.deltaTime, P.gain, P.autoExposure,
                               P.fixedExposure);
    }
}

// BicubicScale with SampleBicubicCatmullRom (16 taps, clamped)
// BicubicScale's source column / row of output pixel x (t1 of the 16-tap Catmull-Rom footprint)
RT_DEV int scale_t1(int x, int Ws, int W) { return (int)floorf((float)x / Ws * (float)W - 0.5f); }


// BicubicScale's per-axis part (postprocessing.cuh:785-802): the first tap t1 and the four
// Catmull-Rom weights of screen coordinate x (Ws screen texels over W render texels)
RT_DEV int bicubic_axis(int x, int Ws, int W, float w[4]) {
    const float uv = (float)x / Ws;
    const float UV = uv * (float)W;
    const float fx0 = floorf(UV - 0.5f);
    const float f = UV - (fx0 + 0.5f);
    const float f2 = f * f;
    const float f3v = f2 * f;
    w[0] = f2 - 0.5f * (f3v + f);
    w[1] = 1.5f * f3v - 2.5f * f2 + 1.0f;
    w[3] = 0.5f * (f3v - f2);
    w[2] = 1.0f - w[0] - w[1] - w[3];
    return (int)fx0;
}

// (k_scale_post's fallback beyond its LDS tile: one row of taps at a time, or the sixteen loads
// in flight set the kernel's VGPR peak for a path the usual scale factors never take)
template <class Img>
RT_DEV uint2 bicubic_scale_px(const Img& im, int W, int H, int x, int y, int Ws, int Hs) {
    float wx[4], wy[4];
    const int t1x = bicubic_axis(x, Ws, W, wx), t1y = bicubic_axis(y, Hs, H, wy);
    F3 o = f3(0.0f);
    float sw = 0.0f;
#pragma unroll 1
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float w = wx[i] * wy[j];
            sw += w;
            o = o + rgb_mul(im.at(t1x - 1 + i, t1y - 1 + j), w);
        }
    o = o / sw;
    return pack_color(o, 0x3C00u);
}

// ---- tone mappers (postprocessing.cuh:488-708), each followed by the gamma step
RT_DEV float luminance(F3 v) { return dot(v, f3(0.2126f, 0.7152f, 0.0722f)); }  // linearMath.h:746-749

RT_DEV F3 mat3_mul(const float* m, F3 v) {  // Mat3 * Float3 (linearMath.h:533-538), rows via InnerProduct
    if (kDnPk) {  // rows 0 and 1 as one register pair (rtmath_pk.h inner3_2g)
        using rtpk::F2;
        const F2 r01 = rtpk::inner3_2g(F2{m[0], m[3]}, rtpk::splat(v.x), F2{m[1], m[4]}, rtpk::splat(v.y),
                                       F2{m[2], m[5]}, rtpk::splat(v.z));
        return f3(r01.x, r01.y, inner3(m[6], v.x, m[7], v.y, m[8], v.z));
    }
    return f3(inner3(m[0], v.x, m[1], v.y, m[2], v.z), inner3(m[3], v.x, m[4], v.y, m[5], v.z),
              inner3(m[6], v.x, m[7], v.y, m[8], v.z));
}

__constant__ float cAcesIn[9] = {(float)0.59719, (float)0.35458, (float)0.04823, (float)0.07600, (float)0.90834,
                                 (float)0.01566, (float)0.02840, (float)0.13383, (float)0.83777};
__constant__ float cAcesOut[9] = {(float)1.60475, (float)-0.53108, (float)-0.07367, (float)-0.10208, (float)1.10813,
                                  (float)-0.00605, (float)-0.00327, (float)-0.07276, (float)1.07602};

RT_DEV F3 tonemap_color(F3 c, int type, float maxWhite, float gamma) {
    if (type == 3) {  // ToneMappingReinhardExtended: ReinhardExtendedLuminance
        const float lo = luminance(c);
        const float num = lo * (1.0f + (lo / (maxWhite * maxWhite)));
        const float ln = num / (1.0f + lo);
        c = c * (ln / luminance(c));
    } else if (type == 1) {  // ToneMappingACES: ACESFitted with RRTAndODTFitLuminance
        c = mat3_mul(cAcesIn, c);
        const float lum = luminance(c);
        const float a = lum * (lum + 0.0245786f) - 0.000090537f;
        const float b = lum * (0.983729f * lum + 0.4329510f) + 0.238081f;
        c = c * ((a / b) / luminance(c));
        c = mat3_mul(cAcesOut, c);
        c = clamp3(c, f3(0.0f), f3(1.0f));
    } else if (type == 2) {  // ToneMappingACES2: ACESFilm
        const F3 num = c * (c * 2.51f + 0.03f);
        const F3 den = c * (c * 2.43f + 0.59f) + 0.14f;
        c = clamp3(num / den, f3(0.0f), f3(1.0f));
    } else {  // ToneMappingUncharted: Uncharted2Tonemap returns 0, white scale 1/0
        c = f3(0.0f) * f3(__builtin_inff());
    }
    const float g = 1.0f / gamma;
    F3 o;
    if (kDnPk && rtpk::pow_pos_ok(g)) {  // red and green as a pair (rtmath_pk.h), x >= 0 finite
        const float inf = __builtin_inff();
        const bool ok0 = c.x >= 0.0f && c.x < inf, ok1 = c.y >= 0.0f && c.y < inf;
        rtpk::F2 r = rtpk::pow_pos2(rtpk::F2{ok0 ? c.x : 1.0f, ok1 ? c.y : 1.0f}, g, rtpk::pow_y_odd(g));
        if (!ok0) r.x = rt_powf(c.x, g);  // negative, infinite or NaN: rt_powf's special cases
        if (!ok1) r.y = rt_powf(c.y, g);
        o = f3(r.x, r.y, rt_powf(c.z, g));
    } else {
        o = f3(rt_powf(c.x, g), rt_powf(c.y, g), rt_powf(c.z, g));
    }
    return clamp3(o, f3(0.0f), f3(1.0f));
}

// ---- BloomGuassian (postprocessing.cuh:348-388): a 16x16 workgroup keys a 16x16 tile
// (2-texel apron, clamped reads) into LDS and its inner 12x12 threads take the 5x5 gaussian.
__global__ __launch_bounds__(256) void k_bloom_gauss(const uint2* in, int W, int H, uint2* out, const float* exposure) {
    __shared__ F3 sh[16][16];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int x = blockIdx.x * 12 + tx - 2, y = blockIdx.y * 12 + ty - 2;
    const View2 im{in, W, H};
    F3 c = rgb_of(im.at(x, y));
    const float lum = fmx(fmx(c.x, c.y), c.z);
    const float sq = __builtin_sqrtf(lum * lum - exposure[2]);
    c = c * (sq > 0.0f ? sq : 0.0f);  // max(sqrtf(.), 0.0): a NaN root keys to 0
    sh[tx][ty] = c;
    __syncthreads();
    if (tx < 2 || ty < 2 || tx > 13 || ty > 13 || x >= W || y >= H) return;
    F3 o = f3(0.0f);
    float wsum = 0.0f;
#pragma unroll
    for (int i = 0; i < 25; ++i) {
        o = o + sh[tx + i % 5 - 2][ty + i / 5 - 2] * cG5[i];
        wsum += cG5[i];
    }
    o = o / wsum;
    if (isnan3(o)) o = f3(0.0f);
    out[(size_t)y * W + x] = pack_color(o, 0x3C00u);
}

// SampleBicubicCatmullRom<Load2DFuncHalf4<Float3>> (sampler.cuh:446-496)
RT_DEV F3 catmull_rom(const View2& im, F2 uv) {
    const F2 UV = {uv.x * (float)im.W, uv.y * (float)im.H};
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
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float w = wx[i] * wy[j];
            sw += w;
            o = o + rgb_mul(im.at(t1x - 1 + i, t1y - 1 + j), w);
        }
    return o / sw;
}

// Bloom (postprocessing.cuh:390-408), out of place: `in` may be the next frame's history
__global__ __launch_bounds__(256) void k_bloom_apply(DenoisePostParams P, const uint2* in, uint2* out) {
    const int W = (int)P.W, H = (int)P.H;
    const int x = tile_x(P) * 16 + (threadIdx.x & 15), y = tile_y(P) * 16 + (threadIdx.x >> 4);
    if (x >= W || y >= H) return;
    const int W4 = (W + 3) / 4, H4 = (H + 3) / 4, W16 = (W4 + 3) / 4, H16 = (H4 + 3) / 4;
    const F2 uv = {(float)x / W, (float)y / H};
    const F3 s4 = catmull_rom(View2{P.bloom4, W4, H4}, uv), s16 = catmull_rom(View2{P.bloom16, W16, H16}, uv);
    const size_t p = (size_t)y * W + x;
    F3 c = rgb_of(in[p]);
    c = c + (s4 + s16) * 0.05f;
    if (isnan3(c)) c = f3(0.0f);
    out[p] = pack_color(c, 0x3C00u);
}

// ---- LensFlare (postprocessing.cuh:414-480); LensFlarePred's depth test runs per thread
RT_DEV float lf_len(F2 p) { return __builtin_sqrtf(p.x * p.x + p.y * p.y); }
RT_DEV float lf_rand(float w) {  // fract(sinf(w) * 1000) with modff: the signed fractional part
    const float v = rt_sinf(w) * 1000.0f;
    return v - truncf(v);
}
RT_DEV float lf_reg_shape(F2 p, int N) {
    const float a = rt_atan2f(p.x, p.y) + 0.2f;
    const float b = kTwoPi / float(N);
    const float w = rt_cosf(floorf(0.5f + a / b) * b - a) * lf_len(p);
    return 0.5f + (w * w * (3.0f - 2.0f * w)) * (0.51f - 0.5f);  // smoothstep1f (linearMath.h:494)
}
RT_DEV F3 lf_circle(F2 p, float size, float dist, F2 m) {
    const float d4 = (float)((double)dist * 4.0);
    const float l = lf_len(F2{p.x + m.x * d4, p.y + m.y * d4}) + size / 2.0f;
    const float c = fmx(0.01f - rt_powf(lf_len(F2{p.x + m.x * dist, p.y + m.y * dist}), size * 1.4f), 0.0f) * 30.0f;
    const float c1 = fmx(0.001f - rt_powf(l - 0.3f, 1.0f / 40.0f) + rt_sinf(l * 30.0f), 0.0f) * 3.0f;
    const F2 md = {m.x * dist / 2.0f, m.y * dist / 2.0f};
    const float c2 = fmx(0.04f / rt_powf(lf_len(F2{(p.x - md.x) + 0.09f, (p.y - md.y) + 0.09f}) * 1.0f, 1.0f), 0.0f) / 20.0f;
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

__global__ __launch_bounds__(256) void k_lens_flare(DenoisePostParams P, const uint2* in, uint2* out) {
    const int W = (int)P.W, H = (int)P.H;
    const int x = tile_x(P) * 16 + (threadIdx.x & 15), y = tile_y(P) * 16 + (threadIdx.x >> 4);
    if (x >= W || y >= H) return;
    const size_t p = (size_t)y * W + x;
    const float sunDepth = h2f(P.depth[(size_t)P.sunUv[1] * W + P.sunUv[0]]);
    if (sunDepth < kRayMaxF) {  // the sun is behind geometry: LensFlarePred launches nothing
        if (in != out) out[p] = in[p];
        return;
    }
    const F2 sunPos = {P.sunPos[0], P.sunPos[1]};
    F2 uv = {(float)x / (float)W, (float)y / (float)H};
    uv = F2{uv.x - 0.5f, uv.y - 0.5f};
    uv.x *= (float)W / (float)H;
    const F2 vec = {uv.x - sunPos.x, uv.y - sunPos.y};
    const float len = lf_len(vec);
    F3 c = rgb_of(in[p]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
        c = c + lf_circle(uv, rt_powf(lf_rand(i * 2000.0f) * 1.8f, 2.0f) + 1.41f, lf_rand(i * 20.0f) * 3.0f + 0.2f - 0.5f,
                          sunPos);
    const float angle = rt_atan2f(vec.y, vec.x);
    c = c + fmx(0.1f / fmx(rt_powf(len * 10.0f, 5.0f), 0.0001f), 0.0f) *
                fabsf(rt_sinf(angle * 5.0f + rt_cosf(angle * 9.0f))) / 20.0f;
    c = c + (fmx(0.1f / rt_powf(len * 10.0f, 1.0f / 20.0f), 0.0f) +
             fabsf(rt_sinf(angle * 3.0f + rt_cosf(angle * 9.0f))) / 16.0f * fabsf(rt_sinf(angle * 9.0f)));
    out[p] = pack_color(c, 0x3C00u);
}

// BicubicScale, SharpeningFilter (FidelityFX CAS), the selected tone mapper and CopyToOutput's
// dither in one pass.  Each workgroup evaluates the scaled image over its 16x16 screen tile and
// a 1-pixel apron into LDS, rounded to half exactly as the reference stores ScaledColorBuffer;
// the sharpened and tone-mapped values are rounded to half in between too, as the reference's
// separate passes store and reload them.
// kLds: render texels staged per workgroup: 24 x 24 covers the 16x16 tile's footprint up to a
// render / screen ratio of ~1.1 (the usual case, 22 x 22 at 1:1), 48 x 48 up to ~2.5; the host
// picks the small one when the ratio allows (scale_lds_small), the kernel checks the footprint
// either way (unstaged reads beyond it).  Occupancy is set by the VGPRs, not the LDS, with the
// small tile.
constexpr int kScaleLdsSmall = 24 * 24, kScaleLdsLarge = 48 * 48;

// 256 threads compute the 18x18 scaled apron in two passes (324 = 256 + 68); 384 threads in one pass
// (the two extra waves leaving after it) measured slower: serial denoise + post 0.274 -> 0.282 ms,
// pipelined frame 0.869 -> 0.880 (profiles/r04_ab/ablations/scale_post/)
constexpr int kScaleThreads = 256;

template <int kLds>
__global__ __launch_bounds__(kScaleThreads) void k_scale_post(DenoisePostParams P, const uint2* render) {
    DN_PRIO();
    __shared__ uint2 sIn[kLds];
    __shared__ uint2 sS[18 * 18];
    __shared__ uint32_t sSobol[256];  // sobol dims 0..3 (bn_value): CopyToOutput's dither
    const int W = (int)P.W, H = (int)P.H, Ws = (int)P.Ws, Hs = (int)P.Hs;
    const int X0 = tile_x(P) * 16 - 1, Y0 = tile_y(P) * 16 - 1;
    // the dither's per-pixel bytes and the sobol rows are loaded with the render texels, so the
    // lookup after the passes reads LDS and registers only
    const int x = tile_x(P) * 16 + (threadIdx.x & 15), y = tile_y(P) * 16 + (threadIdx.x >> 4);
    const BnPixel bnp = bn_pixel(P.bluenoise, x, y);
    bn_stage_sobol(P.bluenoise, sSobol, (int)threadIdx.x, kScaleThreads);
    // Wave 0 evaluates the apron's 18 columns and 18 rows (lanes 0-17 x, 18-35 y; bicubic_axis:
    // the x weights and tap columns depend on the apron column only, the y ones on the row only),
    // and from the first taps of its end columns / rows the render texels the 18x18 apron reads (t1
    // is monotone in x and y) — once per workgroup instead of in every wave
    __shared__ float sW[2][18][4];
    __shared__ int sT[2][18][4];  // tap column within the tile / tap row offset (row * TW)
    __shared__ int sB[4];         // ix0, iy0, TW, TH
    const int t = threadIdx.x;
    if (t < 64) {
        const int ax = t < 18 ? 0 : 1, k = t < 36 ? t - 18 * ax : 17;
        const int S = ax ? Hs : Ws, R = ax ? H : W, O = ax ? Y0 : X0;
        float w[4];
        const int t1 = bicubic_axis(clampi(O + k, 0, S - 1), S, R, w);
        const int ix0 = clampi(__builtin_amdgcn_readlane(t1, 0) - 1, 0, W - 1);
        const int ix1 = clampi(__builtin_amdgcn_readlane(t1, 17) + 2, 0, W - 1);
        const int iy0 = clampi(__builtin_amdgcn_readlane(t1, 18) - 1, 0, H - 1);
        const int iy1 = clampi(__builtin_amdgcn_readlane(t1, 35) + 2, 0, H - 1);
        const int TW = ix1 - ix0 + 1;
        if (t < 36) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                sT[ax][k][i] = ax ? (clampi(t1 - 1 + i, 0, H - 1) - iy0) * TW : clampi(t1 - 1 + i, 0, W - 1) - ix0;
                sW[ax][k][i] = w[i];
            }
        }
        if (t == 0) {
            sB[0] = ix0;
            sB[1] = iy0;
            sB[2] = TW;
            sB[3] = iy1 - iy0 + 1;
        }
    }
    __syncthreads();
    const int ix0 = __builtin_amdgcn_readfirstlane(sB[0]), iy0 = __builtin_amdgcn_readfirstlane(sB[1]);
    const int TW = __builtin_amdgcn_readfirstlane(sB[2]), TH = __builtin_amdgcn_readfirstlane(sB[3]);
    const bool staged = TW * TH <= kLds;
    if (staged) {  // rows of 32 lanes (no division by TW)
        for (int r = t >> 5; r < TH; r += kScaleThreads / 32)
            for (int c = t & 31; c < TW; c += 32) sIn[r * TW + c] = render[(size_t)(iy0 + r) * W + ix0 + c];
    }
    __syncthreads();
    if (staged) {
        for (int i = threadIdx.x; i < 18 * 18; i += kScaleThreads) {
            const int cx = i % 18, ry = i / 18;
            F3 o = f3(0.0f);
            float sw = 0.0f;
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int k = 0; k < 4; ++k) {  // the loop order of bicubic_scale_px
                    const float w = sW[0][cx][k] * sW[1][ry][j];
                    sw += w;
                    o = o + rgb_mul(sIn[sT[1][ry][j] + sT[0][cx][k]], w);
                }
            o = o / sw;
            sS[i] = pack_color(o, 0x3C00u);
        }
    } else {
        const View2 gi{render, W, H};
        for (int i = threadIdx.x; i < 18 * 18; i += kScaleThreads) {
            const int sx = clampi(X0 + i % 18, 0, Ws - 1), sy = clampi(Y0 + i / 18, 0, Hs - 1);
            sS[i] = bicubic_scale_px(gi, W, H, sx, sy, Ws, Hs);
        }
    }
    __syncthreads();
    if (x >= Ws || y >= Hs) return;
    const size_t p = (size_t)y * Ws + x;
    struct {  // clamped reads of the scaled image, from the LDS tile
        const uint2* s;
        int X0, Y0, Ws, Hs;
        RT_DEV uint2 at(int xx, int yy) const {
            return s[(clampi(yy, 0, Hs - 1) - Y0) * 18 + (clampi(xx, 0, Ws - 1) - X0)];
        }
    } im{sS, X0, Y0, Ws, Hs};
    uint2 cur = im.at(x, y);
    if (P.sharpen) {
        F3 c[3][3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) c[i][j] = rgb_of(im.at(x + i - 1, y + j - 1));
        F3 t1 = fmax3(fmax3(c[1][1], c[0][1]), c[2][1]);
        F3 t2 = fmax3(fmax3(t1, c[1][0]), c[1][2]);
        F3 t3 = fmax3(fmax3(t2, c[0][0]), c[0][2]);
        F3 t4 = fmax3(fmax3(t3, c[2][0]), c[2][2]);
        const F3 smax = t2 + t4;
        t1 = fmin3(fmin3(c[1][1], c[0][1]), c[2][1]);
        t2 = fmin3(fmin3(t1, c[1][0]), c[1][2]);
        t3 = fmin3(fmin3(t2, c[0][0]), c[0][2]);
        t4 = fmin3(fmin3(t3, c[2][0]), c[2][2]);
        const F3 smin = t2 + t4;
        F3 amp = clamp3(fmin3(smin, f3(2.0f - smax.x, 2.0f - smax.y, 2.0f - smax.z)) / smax, f3(0.0f), f3(1.0f));
        amp = f3(1.0f / __builtin_sqrtf(amp.x), 1.0f / __builtin_sqrtf(amp.y), 1.0f / __builtin_sqrtf(amp.z));
        const float peak = 8.0f - 3.0f * 1.0f;
        const F3 w = f3(-1.0f) / (amp * peak);
        F3 o = (((c[0][1] + c[2][1]) + c[1][0]) + c[1][2]) * w + c[1][1];
        o = o / (f3(1.0f) + f3(4.0f) * w);
        cur = pack_color(o, 0x3C00u);
    }
    if (P.tonemap) {
        const F3 c = tonemap_color(rgb_of(cur) * P.exposure[0], P.toneMappingType, P.maxWhite, P.gamma);
        cur = pack_color(c, 0x3C00u);
    }
    P.scaledB[p] = cur;
    // CopyToOutput (kernel.cu:26-59): blue-noise dither (bn/256; the -1/512 is integer 0)
    const int s = P.frameNum;
    F3 c = rgb_of(cur) + f3(bn_value(sSobol, bnp, s, 0) / 256, bn_value(sSobol, bnp, s, 1) / 256,
                            bn_value(sSobol, bnp, s, 2) / 256);
    const float hi = 1.0f - 1.1920928955078125e-07f;
    c = clamp3(c, f3(0.0f), f3(hi));
    P.rgba[(size_t)y * P.rgbaPitch + x] = (uint32_t)(uint8_t)(c.x * 256) | ((uint32_t)(uint8_t)(c.y * 256) << 8) |
                ((uint32_t)(uint8_t)(c.z * 256) << 16) | (1u << 24);
}

__global__ __launch_bounds__(256) void k_hdr_out(const uint2* color, float4* hdr, size_t n) {
    const size_t p = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    const F3 c = rgb_of(color[p]);
    hdr[p] = make_float4(c.x, c.y, c.z, 1.0f);
}

}  // namespace

// the list chain's first two a-trous passes: depth-weight reciprocal x paired tap weights
template <int S, bool kRedirect, bool kAlbedo = false, bool kCopy = false>
static void launch_s5_list(bool rcp, bool pk, dim3 g, hipStream_t s, const DenoisePostParams& Q, const uint2* in,
                           uint2* out, const uint2* alt) {
    if (kDnSplit && Q.listSplit) {  // two threads per pixel (spatial5_tile_split)
        const dim3 b2(512);
        if (rcp && pk) hipLaunchKernelGGL((k_spatial5_list2<S, true, kRedirect, true, kAlbedo, kCopy>), g, b2, 0, s, Q, in, out, alt);
        else if (rcp) hipLaunchKernelGGL((k_spatial5_list2<S, true, kRedirect, false, kAlbedo, kCopy>), g, b2, 0, s, Q, in, out, alt);
        else if (pk) hipLaunchKernelGGL((k_spatial5_list2<S, false, kRedirect, true, kAlbedo, kCopy>), g, b2, 0, s, Q, in, out, alt);
        else hipLaunchKernelGGL((k_spatial5_list2<S, false, kRedirect, false, kAlbedo, kCopy>), g, b2, 0, s, Q, in, out, alt);
        return;
    }
    const dim3 b(256);
    if (rcp && pk) hipLaunchKernelGGL((k_spatial5_list<S, true, kRedirect, true, kAlbedo, kCopy>), g, b, 0, s, Q, in, out, alt);
    else if (rcp) hipLaunchKernelGGL((k_spatial5_list<S, true, kRedirect, false, kAlbedo, kCopy>), g, b, 0, s, Q, in, out, alt);
    else if (pk) hipLaunchKernelGGL((k_spatial5_list<S, false, kRedirect, true, kAlbedo, kCopy>), g, b, 0, s, Q, in, out, alt);
    else hipLaunchKernelGGL((k_spatial5_list<S, false, kRedirect, false, kAlbedo, kCopy>), g, b, 0, s, Q, in, out, alt);
}

// k_scale_post's footprint of 18 screen texels along an axis spans at most 17 * r + 5 render
// texels (r = render / screen: the first tap one before t1, the last two after, one more for the
// floors' rounding); the small LDS tile holds 24 of them
static bool scale_lds_small(int render, int screen) { return 17 * render + 5 * screen <= 24 * screen - screen; }

#define LAUNCH_CHECK()                          \
    do {                                        \
        hipError_t e__ = hipGetLastError();     \
        if (e__ != hipSuccess) return e__;      \
    } while (0)

// HIP events around denoise kernel k (P->marks: bench.py's per-kernel split of whole frames)
static hipError_t dn_mark(const DenoisePostParams* P, int k, int end, hipStream_t s) {
    if (!P->marks || !P->marks[2 * k + end]) return hipSuccess;
    return hipEventRecord(P->marks[2 * k + end], s);
}
#define DN_MARK(k, end)                                                 \
    do {                                                                \
        hipError_t e__ = dn_mark(P, (k), (end), s);                     \
        if (e__ != hipSuccess) return e__;                              \
    } while (0)

// Tile rows of each pass.  The full frame computes every tile; a strip-local denoise (multi-GPU,
// rows [rowA, rowB) in 64-row blocks) computes each pass only on the rows the passes after it
// read for the strip: the stencil radii of the chain summed backwards from the strip — 3 rows for
// the bicubic scale + sharpen, 1 for TemporalFilter2, 24, 12 and 6 for the a-trous passes, 3 for
// SpatialFilter7x7 (which also reads the tile-noise levels of its own tiles), 1 for
// TemporalFilter — rounded out to 16-row tiles (A, B: the strip in tiles):
//   scale / sharpen / tone map  [A, B)         TemporalFilter2, S5<12>, albedo   [A-1, B+1)
//   S5<6>                       [A-2, B+2)     S5<3>, SpatialFilter7x7           [A-3, B+3)
//   TemporalFilter (+ noise)    [A-4, B+4)
// The accumulation / history rows of the strip itself and the histogram counts are exchanged
// between the ranks afterwards (rt_set_collective_hook).
namespace {
void tile_range(const DenoisePostParams* P, int halo, int& t0, int& t1) {
    const int H16 = ((int)P->H + 15) / 16;
    if (!P->stripLocal) { t0 = 0; t1 = H16; return; }
    t0 = (int)P->rowA / 16 - halo;
    t1 = ((int)P->rowB + 15) / 16 + halo;
    t0 = t0 < 0 ? 0 : t0;
    t1 = t1 > H16 ? H16 : t1;
}
}  // namespace

// phase 0: TemporalSpatialDenoising + DownScale4 + Histogram2 (the histogram is this strip's share
// when strip-local); phase 1: AutoExposure onwards.  A multi-GPU host sums the histograms between
// the phases.
static hipError_t denoise_phase3(DenoisePostParams* P, hipStream_t s);

extern "C" hipError_t rtk_denoise_phase(DenoisePostParams* P, hipStream_t s, int phase) {
    if (phase == 3) return denoise_phase3(P, s);
    const int W = (int)P->W, H = (int)P->H, Ws = (int)P->Ws, Hs = (int)P->Hs;
    const size_t Pn = (size_t)W * H;
    const dim3 b256(256);
    const int W4 = (W + 3) / 4, H4 = (H + 3) / 4, W16b = (W4 + 3) / 4, H16b = (H4 + 3) / 4, W64 = (W16b + 3) / 4,
              H64 = (H16b + 3) / 4;
    hipError_t e;
    // a copy of the parameters for the launch of tile rows [t0, t1) (halo tiles around the strip)
    auto tiles = [&](int halo, DenoisePostParams& Q, dim3& g) {
        int t0, t1;
        tile_range(P, halo, t0, t1);
        Q = *P;
        Q.ty0 = t0;
        Q.ty1 = t1;
        g = dim3((W + 15) / 16, (unsigned)(t1 > t0 ? t1 - t0 : 0));
        return t1 > t0;
    };
    DenoisePostParams Q;
    dim3 g;
    if (phase == 1) {
        uint2* cur = P->finalColor;
        if (P->postProcess) {
            if (!P->exposureDone) {
                hipLaunchKernelGGL(k_auto_exposure, dim3(1), dim3(64), 0, s, P->exposure, (const uint32_t*)P->histogram,
                                   (float)(W64 * H64), P->deltaTime, P->gain, P->autoExposure, P->fixedExposure);
                LAUNCH_CHECK();
            }
            // Bloom and LensFlare modify RenderColorBuffer, which here may be the next frame's
            // history (TemporalFilter2's output): both write a colour buffer instead (full frame only).
            uint2* post = cur == P->colorA ? P->colorB : P->colorA;
            const dim3 g16((W + 15) / 16, (H + 15) / 16);
            if (P->bloom) {
                hipLaunchKernelGGL(k_bloom_gauss, dim3((W4 + 11) / 12, (H4 + 11) / 12), b256, 0, s, (const uint2*)P->c4,
                                   W4, H4, P->bloom4, (const float*)P->exposure);
                LAUNCH_CHECK();
                hipLaunchKernelGGL(k_bloom_gauss, dim3((W16b + 11) / 12, (H16b + 11) / 12), b256, 0, s,
                                   (const uint2*)P->c16, W16b, H16b, P->bloom16, (const float*)P->exposure);
                LAUNCH_CHECK();
                hipLaunchKernelGGL(k_bloom_apply, g16, b256, 0, s, *P, (const uint2*)cur, post);
                LAUNCH_CHECK();
                cur = post;
            }
            if (P->lensFlare) {
                hipLaunchKernelGGL(k_lens_flare, g16, b256, 0, s, *P, (const uint2*)cur, post);
                LAUNCH_CHECK();
                cur = post;
            }
            P->finalColor = cur;
        }
        Q = *P;
        Q.sharpen = P->postProcess && P->sharpen;
        Q.tonemap = P->postProcess && P->tonemap;
        int t0 = 0, t1 = (Hs + 15) / 16;
        if (P->stripLocal) tile_range(P, 0, t0, t1);  // screen = render size for strips
        Q.ty0 = t0;
        Q.ty1 = t1;
        if (t1 > t0) {
            DN_MARK(7, 0);
            const dim3 gs((Ws + 15) / 16, (unsigned)(t1 - t0));
            if (scale_lds_small(W, Ws) && scale_lds_small(H, Hs))
                hipLaunchKernelGGL(k_scale_post<kScaleLdsSmall>, gs, dim3(kScaleThreads), 0, s, Q, (const uint2*)cur);
            else
                hipLaunchKernelGGL(k_scale_post<kScaleLdsLarge>, gs, dim3(kScaleThreads), 0, s, Q, (const uint2*)cur);
            LAUNCH_CHECK();
            DN_MARK(7, 1);
        }
        P->finalScaled = P->scaledB;
        return hipSuccess;
    }
    // Buffer plan: the path-trace colour (colorA) and colorB ping-pong; SpatialFilter7x7 writes
    // AccumulationColorBuffer directly and TemporalFilter2 the next history buffer, so neither
    // needs the reference's copy (denoising.cu:110-112, 178-183).  The tile noise levels are
    // computed in the epilogue of the pass that produces their input when the debug
    // visualisation is off.
    uint2* cur = P->colorA;
    uint2* spare = P->colorB;
    auto next_from = [&](uint2* dst) { if (cur == P->colorA || cur == P->colorB) spare = cur; cur = dst; };
    const int W8 = (W + 7) / 8, H8 = (H + 7) / 8, W16 = (W + 15) / 16, H16 = (H + 15) / 16;
    auto noise = [&](int level) -> hipError_t {
        hipLaunchKernelGGL(k_tile_noise, dim3((W8 * H8 + 7) / 8), b256, 0, s, *P, (const uint2*)cur);
        LAUNCH_CHECK();
        hipLaunchKernelGGL(k_noise16, dim3((W16 * H16 + 255) / 256), b256, 0, s, *P);
        LAUNCH_CHECK();
        if (P->visualize) {
            DenoisePostParams V = *P;
            V.ty0 = 0;
            V.ty1 = H16;
            hipLaunchKernelGGL(k_noise_visualize, dim3(W16, H16), b256, 0, s, V, cur, level);
            LAUNCH_CHECK();
        }
        return hipSuccess;
    };
    // ---- TemporalSpatialDenoising (denoising.cu:51-188)
    // The whole chain with the tile noise levels computed in the passes' epilogues runs the
    // noise-gated passes over active-tile lists (above); rcp: the depth weights' divisor of pass k
    // as a reciprocal (DenoisePostParams::rcpDepthOk)
    // TemporalFilter reads the previous frame's accumulation buffer at reprojected positions while
    // it also writes tiles of this frame's, so the list chain writes another buffer (accumAlt): the
    // host swaps the two, or, when the accumulation buffer is the caller's (a strip-local denoise
    // exchanges it), copies the rows this chain finished back into it (frame.cpp run_denoise)
    const bool useList = P->tileList && P->accumAlt && P->temporal && P->frameNum != 1 &&
                         P->localSpatial && P->wideSpatial && !P->visualize;
    uint2* const accOut = useList ? P->accumAlt : P->accum;
    P->listUsed = useList ? 1 : 0;
    const bool rcpT = (P->rcpDepthOk & 1) != 0, rcp7 = (P->rcpDepthOk & 2) != 0, rcp5 = (P->rcpDepthOk & 4) != 0;
    const float sn5 = P->dn.large_denoise_sigma_normal;
    const bool pk5 = kDnPk && sn5 > 0.0f && sn5 < __builtin_inff();  // rtpk::pow_pos_ok
    const float sn7 = P->dn.local_denoise_sigma_normal;
    const bool pk7 = kDnPk && sn7 > 0.0f && sn7 < __builtin_inff();
    const float snT = P->dn.temporal_denoise_sigma_normal;
    const bool pkT = kDnPk && snT > 0.0f && snT < __builtin_inff();
    // one workgroup per list slot the frame can fill: the lists hold tiles of TemporalFilter's tile
    // rows only (a strip-local rank's strip and halo), a contiguous run of tile indices, so a
    // partition (tile % 16) holds at most a sixteenth of them
    int lt0, lt1;
    tile_range(P, 4, lt0, lt1);
    const uint32_t listRows = (uint32_t)(lt1 > lt0 ? ((lt1 - lt0) * ((W + 15) / 16) + kListParts - 1) / kListParts : 0);
    const uint32_t capRows = P->tileCap / kListParts + 1;
    const dim3 gList((unsigned)(kListParts * (listRows < capRows ? listRows : capRows)));
    bool noise1 = false, histDepthDone = false;
    if (P->temporal && P->frameNum != 1) {
        noise1 = P->localSpatial && !P->visualize;
        uint2* dst = spare;
        if (tiles(4, Q, g)) {
            // the whole frame without the debug outlines (which rewrite depth): TemporalFilter2's
            // HistoryDepthBuffer copy rides on this pass's depth reads
            Q.histDepthInTemporal = histDepthDone = P->temporal2 && !P->stripLocal && !P->visualize;
            DN_MARK(0, 0);
            if (useList) {
                if (rcpT && pkT) hipLaunchKernelGGL((k_temporal<true, true, true, true>), g, b256, 0, s, Q, (const uint2*)cur, dst);
                else if (rcpT) hipLaunchKernelGGL((k_temporal<true, true, true>), g, b256, 0, s, Q, (const uint2*)cur, dst);
                else if (pkT) hipLaunchKernelGGL((k_temporal<true, true, false, true>), g, b256, 0, s, Q, (const uint2*)cur, dst);
                else hipLaunchKernelGGL((k_temporal<true, true, false>), g, b256, 0, s, Q, (const uint2*)cur, dst);
            } else if (noise1) {
                if (rcpT) hipLaunchKernelGGL((k_temporal<true, false, true>), g, b256, 0, s, Q, (const uint2*)cur, dst);
                else hipLaunchKernelGGL((k_temporal<true, false, false>), g, b256, 0, s, Q, (const uint2*)cur, dst);
            } else {
                if (rcpT) hipLaunchKernelGGL((k_temporal<false, false, true>), g, b256, 0, s, Q, (const uint2*)cur, dst);
                else hipLaunchKernelGGL((k_temporal<false, false, false>), g, b256, 0, s, Q, (const uint2*)cur, dst);
            }
            LAUNCH_CHECK();
            DN_MARK(0, 1);
        }
        next_from(dst);
    }
    bool noise2 = false;
    if (P->localSpatial) {
        if (!noise1 && (e = noise(1)) != hipSuccess) return e;
        noise2 = P->wideSpatial && !P->visualize;
        uint2* dst = P->temporal ? accOut : spare;
        if (tiles(3, Q, g)) {
            DN_MARK(1, 0);
            if (useList) {  // list 0 only; TemporalFilter wrote the other tiles into the accumulation buffer
                const dim3 b512(512);
                const bool split = kDnSplit && Q.listSplit;
                if (split && rcp7 && pk7) hipLaunchKernelGGL((k_spatial7_list2<true, true>), gList, b512, 0, s, Q, (const uint2*)cur, dst);
                else if (split && rcp7) hipLaunchKernelGGL((k_spatial7_list2<true, false>), gList, b512, 0, s, Q, (const uint2*)cur, dst);
                else if (split && pk7) hipLaunchKernelGGL((k_spatial7_list2<false, true>), gList, b512, 0, s, Q, (const uint2*)cur, dst);
                else if (split) hipLaunchKernelGGL((k_spatial7_list2<false, false>), gList, b512, 0, s, Q, (const uint2*)cur, dst);
                else if (rcp7 && pk7) hipLaunchKernelGGL((k_spatial7_list<true, true>), gList, b256, 0, s, Q, (const uint2*)cur, dst);
                else if (rcp7) hipLaunchKernelGGL((k_spatial7_list<true, false>), gList, b256, 0, s, Q, (const uint2*)cur, dst);
                else if (pk7) hipLaunchKernelGGL((k_spatial7_list<false, true>), gList, b256, 0, s, Q, (const uint2*)cur, dst);
                else hipLaunchKernelGGL((k_spatial7_list<false, false>), gList, b256, 0, s, Q, (const uint2*)cur, dst);
            } else if (noise2) {
                if (rcp7) hipLaunchKernelGGL((k_spatial7<true, true>), g, b256, 0, s, Q, (const uint2*)cur, dst);
                else hipLaunchKernelGGL((k_spatial7<true, false>), g, b256, 0, s, Q, (const uint2*)cur, dst);
            } else {
                if (rcp7) hipLaunchKernelGGL((k_spatial7<false, true>), g, b256, 0, s, Q, (const uint2*)cur, dst);
                else hipLaunchKernelGGL((k_spatial7<false, false>), g, b256, 0, s, Q, (const uint2*)cur, dst);
            }
            LAUNCH_CHECK();
            DN_MARK(1, 1);
        }
        next_from(dst);
    } else if (P->temporal) {
        if ((e = hipMemcpyAsync(P->accum, cur, Pn * 8, hipMemcpyDeviceToDevice, s)) != hipSuccess) return e;
    }
    if (P->wideSpatial) {
        if (P->visualize && cur == P->accum) {  // the debug outlines must not land in the history
            if ((e = hipMemcpyAsync(spare, cur, Pn * 8, hipMemcpyDeviceToDevice, s)) != hipSuccess) return e;
            next_from(spare);
        }
        if (!noise2 && (e = noise(2)) != hipSuccess) return e;
        // a: a colour buffer other than the one being read; b: the other colour buffer.  With the
        // lists the first pass reads the accumulation buffer (cur) and every pass's taps outside
        // list 1 read it too (alt)
        uint2* a = cur == P->colorA ? P->colorB : cur == P->colorB ? P->colorA : spare;
        uint2* b = a == P->colorA ? P->colorB : P->colorA;
        const uint2* alt = cur;
        // folded list chain ([tuning] dnFold): the first pass also finishes the tiles off list 1
        // for the last (kCopy), which then runs over list 1 only with ApplyAlbedo in its store
        const bool fold = useList && (P->listFold || (kDnSplit && P->listSplit));
        int c0 = 0, c1 = 0;
        tile_range(P, 1, c0, c1);
        if (tiles(3, Q, g)) {
            DN_MARK(2, 0);
            if (fold) {
                Q.cty0 = c0;
                Q.cty1 = c1;
                launch_s5_list<3, false, false, true>(rcp5, pk5, gList, s, Q, (const uint2*)cur, a, alt);
            } else if (useList) {
                launch_s5_list<3, false>(rcp5, pk5, gList, s, Q, (const uint2*)cur, a, alt);
            } else {
                if (rcp5) hipLaunchKernelGGL((k_spatial5<3, false, true, false>), g, b256, 0, s, Q, (const uint2*)cur, a, alt);
                else hipLaunchKernelGGL((k_spatial5<3, false, false, false>), g, b256, 0, s, Q, (const uint2*)cur, a, alt);
            }
            LAUNCH_CHECK();
            DN_MARK(2, 1);
        }
        if (tiles(2, Q, g)) {
            DN_MARK(3, 0);
            if (useList) {
                launch_s5_list<6, true>(rcp5, pk5, gList, s, Q, (const uint2*)a, b, alt);
            } else {
                if (rcp5) hipLaunchKernelGGL((k_spatial5<6, false, true, false>), g, b256, 0, s, Q, (const uint2*)a, b, alt);
                else hipLaunchKernelGGL((k_spatial5<6, false, false, false>), g, b256, 0, s, Q, (const uint2*)a, b, alt);
            }
            LAUNCH_CHECK();
            DN_MARK(3, 1);
        }
        if (tiles(1, Q, g)) {
            DN_MARK(4, 0);
            if (fold) {
                launch_s5_list<12, true, true>(rcp5, pk5, gList, s, Q, (const uint2*)b, a, alt);
            } else if (useList) {
                if (rcp5 && pk5) hipLaunchKernelGGL((k_spatial5<12, true, true, true, true>), g, b256, 0, s, Q, (const uint2*)b, a, alt);
                else if (rcp5) hipLaunchKernelGGL((k_spatial5<12, true, true, true>), g, b256, 0, s, Q, (const uint2*)b, a, alt);
                else if (pk5) hipLaunchKernelGGL((k_spatial5<12, true, false, true, true>), g, b256, 0, s, Q, (const uint2*)b, a, alt);
                else hipLaunchKernelGGL((k_spatial5<12, true, false, true>), g, b256, 0, s, Q, (const uint2*)b, a, alt);
            } else {
                if (rcp5) hipLaunchKernelGGL((k_spatial5<12, true, true, false>), g, b256, 0, s, Q, (const uint2*)b, a, alt);
                else hipLaunchKernelGGL((k_spatial5<12, true, false, false>), g, b256, 0, s, Q, (const uint2*)b, a, alt);
            }
            LAUNCH_CHECK();
            DN_MARK(4, 1);
        }
        cur = a;
        spare = b;
    } else {  // out of place when cur is the accumulation buffer (the next frame's history)
        uint2* dst = cur == P->accum ? spare : cur;
        if (tiles(1, Q, g)) {
            const size_t rows = (size_t)(Q.ty1 - Q.ty0) * 16 * W;
            hipLaunchKernelGGL(k_apply_albedo, dim3((unsigned)((rows + 255) / 256)), b256, 0, s, Q, (const uint2*)cur, dst);
            LAUNCH_CHECK();
        }
        cur = dst;
    }
    P->svgfOut = cur;
    P->histDepthDone = histDepthDone ? 1 : 0;
    if (phase == 2) return hipSuccess;
    return rtk_denoise_phase(P, s, 3);
}

// phase 3: TemporalFilter2 onwards, up to the histogram (the tail of phase 0)
static hipError_t denoise_phase3(DenoisePostParams* P, hipStream_t s) {
    const int W = (int)P->W, H = (int)P->H;
    const size_t Pn = (size_t)W * H;
    const dim3 b256(256);
    const int W4 = (W + 3) / 4, H4 = (H + 3) / 4, W16b = (W4 + 3) / 4, H16b = (H4 + 3) / 4, W64 = (W16b + 3) / 4,
              H64 = (H16b + 3) / 4;
    hipError_t e;
    auto tiles = [&](int halo, DenoisePostParams& Q, dim3& g) {
        int t0, t1;
        tile_range(P, halo, t0, t1);
        Q = *P;
        Q.ty0 = t0;
        Q.ty1 = t1;
        g = dim3((W + 15) / 16, (unsigned)(t1 > t0 ? t1 - t0 : 0));
        return t1 > t0;
    };
    DenoisePostParams Q;
    dim3 g;
    uint2* cur = P->svgfOut;
    const bool histDepthDone = P->histDepthDone != 0;
    // the whole frame with every post pass on runs DownScale4 x 3 + Histogram2 + AutoExposure as
    // k_downscale_chain; TemporalFilter2 then also writes the first DownScale4 level
    const bool chain = P->postProcess && P->downScale && P->histogramOn && !P->stripLocal;
    bool down = false;
    if (P->temporal2) {
        down = chain && P->frameNum != 1;
        if (P->frameNum != 1) {
            if (tiles(1, Q, g)) {
                DN_MARK(5, 0);
                if (down) hipLaunchKernelGGL(k_temporal2<true>, g, b256, 0, s, Q, (const uint2*)cur, P->histColorOut);
                else hipLaunchKernelGGL(k_temporal2<false>, g, b256, 0, s, Q, (const uint2*)cur, P->histColorOut);
                LAUNCH_CHECK();
                DN_MARK(5, 1);
            }
        } else if ((e = hipMemcpyAsync(P->histColorOut, cur, Pn * 8, hipMemcpyDeviceToDevice, s)) != hipSuccess) {
            return e;
        }
        cur = P->histColorOut;
        if (!histDepthDone &&
            (e = hipMemcpyAsync(P->histDepth, P->depth, Pn * 2, hipMemcpyDeviceToDevice, s)) != hipSuccess)
            return e;
    }
    P->finalColor = cur;
    if (P->hdrOut && !P->stripLocal) {  // strip-local: after the rows exchange (rtk_hdr_out, frame.cpp)
        hipLaunchKernelGGL(k_hdr_out, dim3((unsigned)((Pn + 255) / 256)), b256, 0, s, (const uint2*)cur, P->hdrOut, Pn);
        LAUNCH_CHECK();
    }
    // ---- PostProcessing (postprocessing.cu:5-161) up to the histogram: the DownScale4 chain and
    // the histogram over this context's rows (64-row aligned strips keep each level's texels local)
    if (chain) {
        // the whole frame with every pass on: the three DownScale4 levels, Histogram2 and
        // AutoExposure in one launch
        DN_MARK(6, 0);
        if (down) hipLaunchKernelGGL(k_downscale_chain<true>, dim3(W64, H64), b256, 0, s, *P, (const uint2*)cur, P->chainCounter);
        else hipLaunchKernelGGL(k_downscale_chain<false>, dim3(W64, H64), b256, 0, s, *P, (const uint2*)cur, P->chainCounter);
        LAUNCH_CHECK();
        DN_MARK(6, 1);
        P->exposureDone = 1;
    } else if (P->postProcess) {
        const int ra = P->stripLocal ? (int)P->rowA : 0, rb = P->stripLocal ? (int)P->rowB : H;
        auto span = [](int a, int b, int f, int n, int& o0, int& o1) {
            o0 = a / f;
            o1 = (b + f - 1) / f;
            o1 = o1 > n ? n : o1;
        };
        if (P->downScale) {
            int o0, o1;
            span(ra, rb, 4, H4, o0, o1);
            hipLaunchKernelGGL(k_downscale4, dim3((W4 * (o1 - o0) + 255) / 256), b256, 0, s, (const uint2*)cur, W, H,
                               P->c4, W4, H4, o0, o1);
            LAUNCH_CHECK();
            span(ra, rb, 16, H16b, o0, o1);
            hipLaunchKernelGGL(k_downscale4, dim3((W16b * (o1 - o0) + 255) / 256), b256, 0, s, (const uint2*)P->c4, W4,
                               H4, P->c16, W16b, H16b, o0, o1);
            LAUNCH_CHECK();
            span(ra, rb, 64, H64, o0, o1);
            hipLaunchKernelGGL(k_downscale4, dim3((W64 * (o1 - o0) + 255) / 256), b256, 0, s, (const uint2*)P->c16,
                               W16b, H16b, P->c64, W64, H64, o0, o1);
            LAUNCH_CHECK();
        }
        if (P->histogramOn) {
            int o0, o1;
            span(ra, rb, 64, H64, o0, o1);
            hipLaunchKernelGGL(k_histogram, dim3(1), dim3(1024), 0, s, (const uint2*)P->c64, W64, H64, P->histogram, o0, o1);
            LAUNCH_CHECK();
        } else if ((e = hipMemsetAsync(P->histogram, 0, 256, s)) != hipSuccess) {
            return e;
        }
    }
    return hipSuccess;
}

extern "C" hipError_t rtk_hdr_out(const uint2* color, float4* hdr, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hdr_out, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, color, hdr, n);
    return hipGetLastError();
}

extern "C" hipError_t rtk_denoise_post(DenoisePostParams* P, hipStream_t s) {
    hipError_t e = rtk_denoise_phase(P, s, 0);
    return e == hipSuccess ? rtk_denoise_phase(P, s, 1) : e;
}
