// debug_math.hip — test entry for the denoiser's packed-pair transcendentals (rtmath_pk.h), which
// must give rtmath.h's scalar results bit for bit (no reference counterpart; tests/test_gpu_pk_math.py).
#include <hip/hip_runtime.h>

#include "rtmath_pk.h"
#include "rtx_amd.h"

namespace {
// element i and its partner i ^ 1 go through one register pair; the scalar function runs beside it
__global__ __launch_bounds__(256) void k_debug_pk(int fn, const float* x, float y, float c, float* outPk,
                                                  float* outScalar, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const size_t j = (i ^ 1) < n ? (i ^ 1) : i;
    const rtpk::F2 v = {x[i], x[j]};
    float pk = 0.0f, sc = 0.0f;
    if (fn == 0) {  // pow(x, y) for finite x >= 0, y finite > 0
        pk = rtpk::pow_pos2(v, y, rtpk::pow_y_odd(y)).x;
        sc = rt_powf(x[i], y);
    } else if (fn == 1) {  // expf
        pk = rtpk::expf2(v).x;
        sc = rt_expf(x[i]);
    } else {  // x / y through the reciprocal c = RN(1 / y)
        pk = rtpk::div_rcp2(v, y, c).x;
        sc = rt_div_rcp(x[i], y, c);
    }
    outPk[i] = pk;
    outScalar[i] = sc;
}
}  // namespace

extern "C" int rt_debug_pk_math(int fn, const float* x, float y, float c, float* out_pk, float* out_scalar, size_t n) {
    if (!x || !out_pk || !out_scalar || fn < 0 || fn > 2) return RT_ERR_ARG;
    if (fn == 0 && !(y > 0.0f && y < __builtin_inff())) return RT_ERR_ARG;
    if (n == 0) return RT_OK;
    hipLaunchKernelGGL(k_debug_pk, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, fn, x, y, c, out_pk, out_scalar, n);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) return RT_ERR_HIP;
    return RT_OK;
}
