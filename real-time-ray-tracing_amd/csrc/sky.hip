// sky.hip — sky / sun radiance images and their luminance CDFs for gfx950.
//
//   k_sky    Sky kernel (sky.cuh:280-298): Hosek-Wilkie radiance per 512x256 equal-area texel,
//            including the reference's double-precision sub-expressions (sky.cuh:165-190)
//   k_sun    SkySun kernel (sky.cuh:300-320): limb-darkened solar disc on a 32x32 cone map
//   scan     Scan (scan.cuh:258-298): per-block Blelloch scan in LDS + block totals, an
//            exclusive Blelloch scan of the totals, and a uniform add — the inclusive scan the
//            reference intends (DESIGN.md §5 on its orig[] indexing).  Tree order is kept, so
//            the fp32 CDF is bit-identical to the oracle's.
// These run only when the sky parameters change (kernel.cu:286-307), not per frame.
#include "frame_kernels.h"
#include "rt_device.h"
#include "rtmath.h"
#include "shade.h"

using namespace rtd;

namespace {

RT_DEV F3 xyz_to_srgb(F3 c) {  // XyzToRgbSrgb (color.h:19-30)
    // Mat3(float...) built from double literals (each converted to float once)
    const float m00 = (float)3.2404542, m01 = (float)-1.5371385, m02 = (float)-0.4985314;
    const float m10 = (float)-0.9692660, m11 = (float)1.8760108, m12 = (float)0.0415560;
    const float m20 = (float)0.0556434, m21 = (float)-0.2040259, m22 = (float)1.0572252;
    return f3(inner3(m00, c.x, m01, c.y, m02, c.z), inner3(m10, c.x, m11, c.y, m12, c.z),
              inner3(m20, c.x, m21, c.y, m22, c.z));
}

RT_DEV F3 sky_radiance(F3 rd, F3 sunDir, const SkyGenParams& P) {
    const float theta = rt_acosf(rd.y);
    const float gamma = rt_acosf(clampf(dot(rd, sunDir), -1.0f, 1.0f));
    const float cg = rt_cosf(gamma), ct = rt_cosf(theta);
    const float zenith = __builtin_sqrtf(ct);
    F3 xyz = f3(0.0f);
    for (int ch = 0; ch < 10; ++ch) {
        const float* c = P.st.configs + ch * 9;
        const float expM = rt_expf(c[4] * gamma);
        const float rayM = cg * cg;
        const float mieM = (1.0f + cg * cg) / rt_powf((1.0f + c[8] * c[8] - 2.0f * c[8] * cg), 1.5f);
        const double left = 1.0 + (double)c[0] * rtm::expd((double)c[1] / ((double)ct + 0.01));
        const float right = c[2] + c[3] * expM + c[5] * rayM + c[6] * mieM + c[7] * zenith;
        const float radiance = (float)(left * (double)right) * P.st.radiances[ch];
        xyz = xyz + radiance * f3(P.cie[ch], P.cie[10 + ch], P.cie[20 + ch]);
    }
    return xyz_to_srgb(xyz);
}

RT_DEV F3 sun_radiance(F3 rd, F3 sunDir, const SkyGenParams& P) {
    const float gamma = rt_acosf(clampf(dot(rd, sunDir), -1.0f, 1.0f));
    const float elevation = (kPi / 2.0f) - rt_acosf(sunDir.y);
    const float solarRadius = P.sunAngle * kPi / 180.0f / 2.0f;
    const float sbs = 1.0f / ((P.sunAngle / 0.51f) * (P.sunAngle / 0.51f));
    const float srs = rt_sinf(solarRadius);
    const float ar2 = 1.0f / (srs * srs);
    const float sg = rt_sinf(gamma);
    float sc2 = 1.0f - ar2 * sg * sg;
    if (sc2 < 0.0f) sc2 = 0.0f;
    const float sampleCosine = __builtin_sqrtf(sc2);
    if (sampleCosine == 0.0f) return f3(0.0f);
    int pos = (int)(rt_powf((float)(2.0 * (double)elevation / (double)kPi), (float)(1.0 / 3.0)) * 45);
    if (pos > 44) pos = 44;
    const float break_x = (float)((double)rt_powf(((float)pos / 45.0f), 3.0f) * ((double)kPi * 0.5));
    const float x = elevation - break_x;
    const float sc2p = rt_powf(sampleCosine, 2.0f), sc3p = rt_powf(sampleCosine, 3.0f);
    const float sc4p = rt_powf(sampleCosine, 4.0f), sc5p = rt_powf(sampleCosine, 5.0f);
    F3 xyz = f3(0.0f);
    for (int ch = 0; ch < 10; ++ch) {
        const float* coefs = P.solar + ch * 180 + (4 * (pos + 1) - 1);
        float res = 0.0f, x_exp = 1.0f;
        for (int i = 0; i < 4; ++i) {
            res += x_exp * coefs[-i];
            x_exp *= x;
        }
        const float* ld = P.limb + ch * 6;
        const float dark = ld[0] + ld[1] * sampleCosine + ld[2] * sc2p + ld[3] * sc3p + ld[4] * sc4p + ld[5] * sc5p;
        const float direct = res * (dark * sbs);
        xyz = xyz + direct * f3(P.cie[ch], P.cie[10 + ch], P.cie[20 + ch]);
    }
    return xyz_to_srgb(xyz);
}

}  // namespace

__global__ __launch_bounds__(256) void k_sky(SkyGenParams P) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= kSkySize) return;
    const int x = i % kSkyW, y = i / kSkyW;
    const float u = ((float)x + 0.5f) / kSkyW, v = ((float)y + 0.5f) / kSkyH;
    const F3 sunDir = f3(P.sunDir[0], P.sunDir[1], P.sunDir[2]);
    const F3 c = max3(sky_radiance(equal_area_map(u, v), sunDir, P) * P.skyScalar, f3(0.0f));
    P.skyBuffer[i] = make_float4(c.x, c.y, c.z, 0.0f);
    P.skyPdf[i] = dot(c, f3(0.3f, 0.6f, 0.1f));
}

__global__ __launch_bounds__(256) void k_sun(SkyGenParams P) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= kSunSize) return;
    const int x = i % kSunW, y = i / kSunW;
    const float u = ((float)x + 0.5f) / kSunW, v = ((float)y + 0.5f) / kSunH;
    const F3 sunDir = f3(P.sunDir[0], P.sunDir[1], P.sunDir[2]);
    const F3 rd = equal_area_map_cone(sunDir, u, v, P.cosThetaMax);
    const F3 c = max3(sun_radiance(rd, sunDir, P) * P.sunScalar, f3(0.0f));
    P.sunBuffer[i] = make_float4(c.x, c.y, c.z, 0.0f);
    P.sunPdf[i] = dot(c, f3(0.3f, 0.6f, 0.1f));
}

// Blelloch scan of one block of n (power of two, 2..8192) values in dynamic LDS: blockDim.x
// threads (<= 256) take the d active pairs of each tree level in strides, so every level performs
// the reference's additions in its order (ScanSingleBlock<n, batch>, scan.cuh:31-137, splits the
// same levels over n/2/batch threads).  kInclusive: out[i] = exclusive[i] + in[i] (postfix 1),
// else the exclusive scan (postfix 0); sums[block] = the up-sweep root (block total).  in == out
// is allowed (the reference scans its block totals in place).
template <bool kInclusive>
__global__ __launch_bounds__(256) void k_scan_block(const float* in, float* out, float* sums, int n) {
    extern __shared__ float a[];
    const int t = threadIdx.x, T = blockDim.x;
    const float* src = in + (size_t)blockIdx.x * n;
    for (int i = t; i < n; i += T) a[i] = src[i];
    int offset = 1;
    for (int d = n >> 1; d > 0; d >>= 1) {
        __syncthreads();
        for (int i = t; i < d; i += T) {
            const int ai = offset * (2 * i + 1) - 1, bi = offset * (2 * i + 2) - 1;
            a[bi] = a[bi] + a[ai];
        }
        offset *= 2;
    }
    __syncthreads();
    if (t == 0) {
        if (sums) sums[blockIdx.x] = a[n - 1];
        a[n - 1] = 0.0f;
    }
    for (int d = 1; d < n; d *= 2) {
        offset >>= 1;
        __syncthreads();
        for (int i = t; i < d; i += T) {
            const int ai = offset * (2 * i + 1) - 1, bi = offset * (2 * i + 2) - 1;
            const float tmp = a[ai];
            a[ai] = a[bi];
            a[bi] = a[bi] + tmp;
        }
    }
    __syncthreads();
    float* dst = out + (size_t)blockIdx.x * n;
    for (int i = t; i < n; i += T) dst[i] = kInclusive ? a[i] + src[i] : a[i];
}

__global__ __launch_bounds__(256) void k_scan_add(float* out, const float* sums, int n, int total) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < total) out[i] = out[i] + sums[i / n];
}

// Scan(in, out, tmp, size, blockSize, postfix) (scan.cuh:258-298): blocks of blockSize, the block
// totals scanned exclusively in one workgroup, then added to every block.  Sizes as the reference
// asserts: powers of two, blockSize and the block count each <= 8192.
extern "C" hipError_t rtk_launch_scan_ex(const float* in, float* out, float* sums, int size, int blockSize,
                                         int postfix, hipStream_t stream) {
    if (blockSize < 2 || blockSize > 8192 || (blockSize & (blockSize - 1)) || size < blockSize || size % blockSize)
        return hipErrorInvalidValue;
    const int blocks = size / blockSize;
    if (blocks > 8192 || (blocks & (blocks - 1)) || (blocks > 1 && !sums)) return hipErrorInvalidValue;
    const int thr = blockSize / 2 < 256 ? blockSize / 2 : 256;
    const size_t lds = (size_t)blockSize * sizeof(float);
    if (postfix)
        hipLaunchKernelGGL(k_scan_block<true>, dim3(blocks), dim3(thr), lds, stream, in, out, blocks > 1 ? sums : nullptr,
                           blockSize);
    else
        hipLaunchKernelGGL(k_scan_block<false>, dim3(blocks), dim3(thr), lds, stream, in, out,
                           blocks > 1 ? sums : nullptr, blockSize);
    if (blocks > 1) {
        const int st = blocks / 2 < 256 ? blocks / 2 : 256;
        hipLaunchKernelGGL(k_scan_block<false>, dim3(1), dim3(st), (size_t)blocks * sizeof(float), stream,
                           (const float*)sums, sums, (float*)nullptr, blocks);
        hipLaunchKernelGGL(k_scan_add, dim3((size + 255) / 256), dim3(256), 0, stream, out, (const float*)sums,
                           blockSize, size);
    }
    return hipGetLastError();
}

extern "C" hipError_t rtk_launch_scan(const float* in, float* out, float* sums, int size, int blockSize,
                                      hipStream_t stream) {
    return rtk_launch_scan_ex(in, out, sums, size, blockSize, 1, stream);
}

// heap node j of the bisection over [0, right0] of `cdf` (see kSkyTreeNodes); nodes the
// search can never reach (its interval already closed) hold NaN
__global__ void k_cdf_tree(const float* cdf, int right0, float* tree, int nodes) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nodes) return;
    if (j == 0) { tree[0] = __builtin_nanf(""); return; }
    const int depth = 31 - __clz(j);
    int left = 0, right = right0;
    bool live = right - left > 1;
    for (int b = depth - 1; b >= 0 && live; --b) {
        const int mid = (left + right) / 2;
        if ((j >> b) & 1) left = mid;
        else right = mid;
        live = right - left > 1;
    }
    tree[j] = live ? cdf[(left + right) / 2] : __builtin_nanf("");
}

// SampleLight's terms that depend only on the frame's light tables (shade.h sample_light), in its
// operation order: pSky = totalSky / (totalSky + totalSun), the CDF totals, and the sun's
// 2 pi (1 - cosThetaMax); the shading kernels read them as uniform loads
__global__ void k_light_select(const float* skyCdf, const float* sunCdf, float cosThetaMax, float* out) {
    const float maxSky = skyCdf[kSkySize - 1], maxSun = sunCdf[kSunSize - 1];
    const float totalSky = maxSky * kTwoPi / kSkySize;
    const float totalSun = maxSun * kTwoPi * (1.0f - cosThetaMax) / kSunSize;
    out[0] = totalSky / (totalSky + totalSun);
    out[1] = maxSky;
    out[2] = maxSun;
    out[3] = kTwoPi * (1.0f - cosThetaMax);
}

extern "C" hipError_t rtk_launch_sky(const SkyGenParams* p, hipStream_t stream) {
    hipLaunchKernelGGL(k_sky, dim3(kSkySize / 256), dim3(256), 0, stream, *p);
    hipError_t e = rtk_launch_scan(p->skyPdf, p->skyCdf, p->scanSums, kSkySize, kSkyScanBlock, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_sun, dim3(kSunSize / 256), dim3(256), 0, stream, *p);
    if ((e = rtk_launch_scan(p->sunPdf, p->sunCdf, p->scanSums, kSunSize, kSunScanBlock, stream)) != hipSuccess)
        return e;
    hipLaunchKernelGGL(k_cdf_tree, dim3(kSkyTreeNodes / 256), dim3(256), 0, stream, p->skyCdf, kSkySize - 2,
                       p->skyTree, kSkyTreeNodes);
    hipLaunchKernelGGL(k_cdf_tree, dim3(kSunTreeNodes / 256), dim3(256), 0, stream, p->sunCdf, kSunSize - 2,
                       p->sunTree, kSunTreeNodes);
    hipLaunchKernelGGL(k_light_select, dim3(1), dim3(1), 0, stream, (const float*)p->skyCdf, (const float*)p->sunCdf,
                       p->cosThetaMax, p->lightSel);
    return hipGetLastError();
}
