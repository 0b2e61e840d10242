// texture.hip — MipmapGen (mipgen.cu:121-182) for gfx950: the 11-level mip chain of a 16-bit
// texture, built on the device after its level 0 is uploaded (init.cu:524-580).
//
// Output texel (x, y) of level l is the mean of the 2x2 input texels (2x..2x+1, 2y..2y+1) of
// level l-1, read with the surface's clamp boundary, summed in float (exact: < 2^24), divided by
// 4, clamped to 65535 and truncated to ushort ((unsigned short)float, toType<ushort4, float4>).
// Levels are square powers of two (1024 -> 1) concatenated in one buffer; one launch per level,
// 16x16 workgroups as the reference's, C = 4 (ushort4) or 1 (ushort) channels.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

template <int C>
__global__ __launch_bounds__(256) void k_mipgen(const uint16_t* __restrict__ in, int inW, int inH,
                                                uint16_t* __restrict__ out, int outW, int outH) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= outW || y >= outH) return;
    const int x0 = 2 * x < inW - 1 ? 2 * x : inW - 1, x1 = 2 * x + 1 < inW - 1 ? 2 * x + 1 : inW - 1;
    const int y0 = 2 * y < inH - 1 ? 2 * y : inH - 1, y1 = 2 * y + 1 < inH - 1 ? 2 * y + 1 : inH - 1;
    const uint16_t* a = in + ((size_t)y0 * inW + x0) * C;
    const uint16_t* b = in + ((size_t)y0 * inW + x1) * C;
    const uint16_t* c = in + ((size_t)y1 * inW + x0) * C;
    const uint16_t* d = in + ((size_t)y1 * inW + x1) * C;
    uint16_t* o = out + ((size_t)y * outW + x) * C;
#pragma unroll
    for (int k = 0; k < C; ++k) {
        float v = (((float)a[k] + (float)b[k]) + (float)c[k]) + (float)d[k];
        v = v / 4.0f;
        v = __builtin_fminf(v, 65535.0f);
        o[k] = (uint16_t)v;
    }
}

}  // namespace

// levels 1..levels-1 of a square chain whose level 0 (size x size, C channels) is in place
extern "C" hipError_t rtk_launch_mipgen(uint16_t* chain, int size, int levels, int channels, hipStream_t s) {
    if (channels != 1 && channels != 4) return hipErrorInvalidValue;
    size_t off = 0;
    int w = size;
    for (int l = 1; l < levels && w > 1; ++l) {
        const int n = w / 2 > 1 ? w / 2 : 1;
        uint16_t* in = chain + off * channels;
        uint16_t* out = in + (size_t)w * w * channels;
        const dim3 grid((n + 15) / 16, (n + 15) / 16);
        if (channels == 4) hipLaunchKernelGGL(k_mipgen<4>, grid, dim3(256), 0, s, in, w, w, out, n, n);
        else hipLaunchKernelGGL(k_mipgen<1>, grid, dim3(256), 0, s, in, w, w, out, n, n);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        off += (size_t)w * w;
        w = n;
    }
    return hipSuccess;
}
