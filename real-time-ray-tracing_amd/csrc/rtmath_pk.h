// rtmath_pk.h — two lanes' worth of the denoiser's per-tap transcendentals in one register pair.
//
// The denoise passes are bound by vector-instruction issue (bench.py roofline.valu_issue: a wave's
// f32 instruction holds its SIMD four cycles), and gfx950 issues f32 add / mul / fma on a register
// pair as one packed instruction (v_pk_add_f32, v_pk_mul_f32, v_pk_fma_f32).  These are rtmath.h's
// float cores restated on a pair of independent arguments — two taps of one pixel — so that the
// polynomial and compensated-product chains issue once per pair.  Each element goes through exactly
// the scalar function's sequence of IEEE operations (branches become per-element selects of values
// both sides compute), so a pair's results are the scalar results bit for bit, and the CPU oracle,
// which runs the scalar functions, stays the checker (tests/test_gpu_denoise.py).
#pragma once
#include "rtmath.h"

namespace rtpk {

typedef float F2 __attribute__((ext_vector_type(2)));
typedef int I2 __attribute__((ext_vector_type(2)));
typedef unsigned int U2 __attribute__((ext_vector_type(2)));

__device__ inline F2 fma2(F2 a, F2 b, F2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ inline F2 splat(float a) { return F2{a, a}; }
__device__ inline F2 sel(bool c0, bool c1, F2 a, F2 b) { return F2{c0 ? a.x : b.x, c1 ? a.y : b.y}; }
__device__ inline U2 bits2(F2 a) { return __builtin_bit_cast(U2, a); }
__device__ inline F2 from_bits2(U2 a) { return __builtin_bit_cast(F2, a); }

// rtm::exp2_core
__device__ inline F2 exp2_core2(F2 f) {
    F2 p = splat(1.5252733804059840e-05f);
    p = fma2(p, f, splat(1.5403530393381609e-04f));
    p = fma2(p, f, splat(1.3333558146428443e-03f));
    p = fma2(p, f, splat(9.6181291076284772e-03f));
    p = fma2(p, f, splat(5.5504108664821580e-02f));
    p = fma2(p, f, splat(2.4022650695910071e-01f));
    p = fma2(p, f, splat(6.9314718055994531e-01f));
    return fma2(p, f, splat(1.0f));
}

// rtm::scale2 (p * 2^n, one rounding) with its three cases as selects: n > 127 multiplies by
// 2^(n-1) and then by 2 (the scalar form doubles first; both products before the last are exact),
// n < -126 by 2^(n+64) and then 2^-64, else by 2^n
__device__ inline float scale2_one(float p, int n) {
    const bool hi = n > 127, lo = n < -126;
    const int n1 = hi ? n - 1 : lo ? n + 64 : n;
    const float f2 = hi ? 2.0f : lo ? rtm::bits_to_float((uint32_t)(-64 + 127) << 23) : 1.0f;
    return (p * rtm::bits_to_float((uint32_t)(n1 + 127) << 23)) * f2;
}
__device__ inline F2 scale2_2(F2 p, I2 n) {
    const bool h0 = n.x > 127, h1 = n.y > 127, l0 = n.x < -126, l1 = n.y < -126;
    const I2 n1 = I2{h0 ? n.x - 1 : l0 ? n.x + 64 : n.x, h1 ? n.y - 1 : l1 ? n.y + 64 : n.y};
    const float m64 = rtm::bits_to_float((uint32_t)(-64 + 127) << 23);
    const F2 f2 = F2{h0 ? 2.0f : l0 ? m64 : 1.0f, h1 ? 2.0f : l1 ? m64 : 1.0f};
    const U2 e = __builtin_bit_cast(U2, (n1 + 127) << 23);
    return (p * from_bits2(e)) * f2;
}

// rtm::exp2_pair: 2^(hi + lo); hi >= 128 gives +inf, hi < -152 gives +0.  The exponent arithmetic
// runs on hi clamped to [-160, 136] so that the lanes the selects discard stay in range.
__device__ inline F2 exp2_pair2(F2 hi, F2 lo) {
    const F2 hc = __builtin_elementwise_min(__builtin_elementwise_max(hi, splat(-160.0f)), splat(136.0f));
    const F2 n = __builtin_elementwise_rint(hc);
    const F2 f = (hc - n) + lo;
    const F2 r = scale2_2(exp2_core2(f), __builtin_convertvector(n, I2));
    const float inf = rtm::bits_to_float(0x7F800000u);
    return F2{hi.x >= 128.0f ? inf : hi.x < -152.0f ? 0.0f : r.x, hi.y >= 128.0f ? inf : hi.y < -152.0f ? 0.0f : r.y};
}

// rtm::recip_log_den
__device__ inline F2 recip_log_den2(F2 d) {
    F2 y = fma2(splat(-0.239016f), d, splat(0.985076f));
    y = fma2(y, fma2(-d, y, splat(1.0f)), y);
    return fma2(y, fma2(-d, y, splat(1.0f)), y);
}

// rtm::log2_pair for finite x > 0 (subnormal scaling and the mantissa fold as selects)
__device__ inline void log2_pair2(F2 x, F2& hi, F2& lo) {
    const U2 b0 = bits2(x);
    const bool s0 = b0.x < 0x00800000u, s1 = b0.y < 0x00800000u;
    const F2 xs = sel(s0, s1, x * splat(8388608.0f), x);
    const U2 b = bits2(xs);
    I2 e = I2{(int)(b.x >> 23) - (s0 ? 150 : 127), (int)(b.y >> 23) - (s1 ? 150 : 127)};
    F2 m = from_bits2((b & 0x007FFFFFu) | 0x3F800000u);
    const bool f0 = m.x > 1.41421354f, f1 = m.y > 1.41421354f;
    m = sel(f0, f1, m * splat(0.5f), m);
    e = e + I2{f0 ? 1 : 0, f1 ? 1 : 0};
    const F2 r = m - splat(1.0f);
    const F2 d = splat(2.0f) + r, dl = r - (d - splat(2.0f));
    const F2 y = recip_log_den2(d);
    const F2 s0v = r * y;
    const F2 s = fma2(fma2(-s0v, d, r), y, s0v);
    const F2 sl = (fma2(-s, d, r) - s * dl) * y;
    const F2 s2 = s * s;
    F2 q = splat(1.0f / 13.0f);
    q = fma2(q, s2, splat(1.0f / 11.0f));
    q = fma2(q, s2, splat(1.0f / 9.0f));
    q = fma2(q, s2, splat(1.0f / 7.0f));
    q = fma2(q, s2, splat(1.0f / 5.0f));
    q = fma2(q, s2, splat(1.0f / 3.0f));
    const F2 lnh = splat(2.0f) * s;
    const F2 lnl = splat(2.0f) * sl + (splat(2.0f) * s) * (s2 * q);
    const F2 Lh = splat(1.44269502162933349609f), Ll = splat(1.9259629911783e-08f);
    const F2 ph = lnh * Lh;
    const F2 pl = fma2(lnh, Lh, -ph) + fma2(lnh, Ll, lnl * Lh);
    const F2 fe = __builtin_convertvector(e, F2);
    const F2 sh = fe + ph;
    const F2 err = (fe - sh) + ph;
    hi = sh;
    lo = err + pl;
    const F2 t = hi + lo;
    lo = lo - (t - hi);
    hi = t;
}

// Whether rt_powf(x, y) takes its float path for every finite x >= 0: y finite and > 0 (uniform:
// the denoiser's sigmas; callers keep the scalar rt_powf otherwise), and whether y is an odd
// integer, which decides the sign of pow(-0, y).
__device__ inline bool pow_pos_ok(float y) { return y > 0.0f && y < rtm::bits_to_float(0x7F800000u); }
__device__ inline bool pow_y_odd(float y) {
    if (!(__builtin_fabsf(y) < 9007199254740992.0f)) return false;
    const double t = (double)(int64_t)y;
    return t == (double)y && (((int64_t)y) & 1) != 0;
}

// rt_powf(x, y) for finite x >= 0 (either zero), pow_pos_ok(y): 1 at x == 1, pow(+-0, y) = +0 or
// -0 (odd y, -0 x), else exp2(y log2 x) through the float pair
__device__ inline F2 pow_pos2(F2 x, float y, bool yOdd) {
    F2 lh, ll;
    log2_pair2(x, lh, ll);
    const F2 Y = splat(y);
    const F2 th = Y * lh;
    const F2 tl = fma2(Y, lh, -th) + Y * ll;
    const F2 r = exp2_pair2(th, tl);
    const U2 xb = bits2(x);
    const float z0 = (xb.x == 0x80000000u && yOdd) ? -0.0f : 0.0f, z1 = (xb.y == 0x80000000u && yOdd) ? -0.0f : 0.0f;
    return F2{x.x == 1.0f ? 1.0f : x.x == 0.0f ? z0 : r.x, x.y == 1.0f ? 1.0f : x.y == 0.0f ? z1 : r.y};
}

// rt_expf
__device__ inline F2 expf2(F2 x) {
    const F2 n = __builtin_elementwise_rint(x * splat(1.44269502162933349609f));
    F2 r = fma2(-n, splat(0.693145751953125f), x);
    r = fma2(-n, splat(1.428606765330187e-06f), r);
    F2 p = splat(2.4801587301587302e-05f);
    p = fma2(p, r, splat(1.9841269841269841e-04f));
    p = fma2(p, r, splat(1.3888888888888889e-03f));
    p = fma2(p, r, splat(8.3333333333333333e-03f));
    p = fma2(p, r, splat(4.1666666666666667e-02f));
    p = fma2(p, r, splat(1.6666666666666667e-01f));
    p = fma2(p, r, splat(0.5f));
    p = fma2(p, r, splat(1.0f));
    p = fma2(p, r, splat(1.0f));
    // n is only used where -104 <= x <= 89 (|n| <= 151); clamp it for the discarded lanes
    const F2 nc = __builtin_elementwise_min(__builtin_elementwise_max(n, splat(-160.0f)), splat(136.0f));
    const F2 s = scale2_2(p, __builtin_convertvector(nc, I2));
    const float inf = rtm::bits_to_float(0x7F800000u);
    return F2{x.x != x.x ? x.x : x.x > 89.0f ? inf : x.x < -104.0f ? 0.0f : s.x,
              x.y != x.y ? x.y : x.y > 89.0f ? inf : x.y < -104.0f ? 0.0f : s.y};
}

// inner3(a, b, c, d, e, f) — rt_device.h's compensated dot product, element for element
__device__ inline F2 inner3_2g(F2 A, F2 b, F2 C, F2 d, F2 E, F2 f) {
    const F2 ef = E * f, efe = fma2(E, f, -ef);
    const F2 cd = C * d, cde = fma2(C, d, -cd);
    const F2 s2 = cd + ef, dl2 = s2 - cd, s2e = (cd - (s2 - dl2)) + (ef - dl2);
    const F2 tpv = s2, tpe = cde + (efe + s2e);
    const F2 ab = A * b, abe = fma2(A, b, -ab);
    const F2 s1 = ab + tpv, dl1 = s1 - ab, s1e = (ab - (s1 - dl1)) + (tpv - dl1);
    const F2 rv = s1, re = abe + (tpe + s1e);
    return rv + re;
}
// with a, c, e shared by both elements (the centre normal)
__device__ inline F2 inner3_2(float a, F2 b, float c, F2 d, float e, F2 f) {
    return inner3_2g(splat(a), b, splat(c), d, splat(e), f);
}

// rt_div_rcp(a, b, c) (c = RN(1 / b), b in its range: rt_div_rcp_ok)
__device__ inline F2 div_rcp2(F2 a, float b, float c) {
    const F2 B = splat(b), C = splat(c);
    const F2 q0 = a * C;
    const F2 q1 = fma2(fma2(-q0, B, a), C, q0);
    const F2 q2 = fma2(fma2(-q1, B, a), C, q1);
    const float inf = rtm::bits_to_float(0x7F800000u);
    return F2{(a.x != 0.0f && __builtin_fabsf(q0.x) < inf) ? q2.x : q0.x,
              (a.y != 0.0f && __builtin_fabsf(q0.y) < inf) ? q2.y : q0.y};
}

}  // namespace rtpk
