// fetch_calib.hip — calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// widths the denoiser uses.  MI355X_MICROARCH.md calibrates
// FETCH_SIZE only for 16-byte-per-lane streaming reads (it reports half the bytes there); the
// denoise kernels read 8-byte half4 texels.  Each kernel below moves a known number of bytes:
//
//   copy4 / copy8 / copy16   dst[i] = src[i] with 4 / 8 / 16 bytes per lane, N bytes each way
//   tile8                    16x16-pixel workgroups over a 1920x1080 half4 image, each thread
//                            reading its own texel (8 B) and writing it: the denoise passes' shape
//
// The buffers (512 MiB each way for the streaming copies) exceed the 256 MiB Infinity Cache, so
// every dispatch reads from HBM.  Build: hipcc --offload-arch=gfx950 -O3 -o fetch_calib.bin
// fetch_calib.hip; run each counter in its own pass: rocprofv3 --pmc FETCH_SIZE --kernel-trace --
// ./fetch_calib.bin (then WRITE_SIZE).  tools/pmc_report.py --calib reads the two passes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            return 1;                                                             \
        }                                                                         \
    } while (0)

template <typename T>
__global__ __launch_bounds__(256) void copy_k(const T* __restrict__ src, T* __restrict__ dst, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void tile8_k(const uint2* __restrict__ src, uint2* __restrict__ dst, int W, int H) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x < W && y < H) dst[(size_t)y * W + x] = src[(size_t)y * W + x];
}

int main() {
    const size_t bytes = 512ull << 20;
    void *a = nullptr, *b = nullptr;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMemset(a, 1, bytes));
    CHECK(hipMemset(b, 0, bytes));
    CHECK(hipDeviceSynchronize());
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(copy_k<uint32_t>, dim3((unsigned)(bytes / 4 / 256)), dim3(256), 0, 0, (const uint32_t*)a,
                           (uint32_t*)b, bytes / 4);
        hipLaunchKernelGGL(copy_k<uint2>, dim3((unsigned)(bytes / 8 / 256)), dim3(256), 0, 0, (const uint2*)a,
                           (uint2*)b, bytes / 8);
        hipLaunchKernelGGL(copy_k<uint4>, dim3((unsigned)(bytes / 16 / 256)), dim3(256), 0, 0, (const uint4*)a,
                           (uint4*)b, bytes / 16);
        // the denoise shape: 1920x1080 half4, 16x16 tiles (16.6 MB: it also fits the Infinity Cache,
        // so this one calibrates the counter for cache-resident 8-byte reads)
        hipLaunchKernelGGL(tile8_k, dim3(120, 68), dim3(256), 0, 0, (const uint2*)a, (uint2*)b, 1920, 1080);
        CHECK(hipGetLastError());
    }
    CHECK(hipDeviceSynchronize());
    printf("fetch_calib: copy4/copy8/copy16 %zu bytes each way, tile8 %d bytes each way, 3 repeats\n", bytes,
           1920 * 1080 * 8);
    CHECK(hipFree(a));
    CHECK(hipFree(b));
    return 0;
}
