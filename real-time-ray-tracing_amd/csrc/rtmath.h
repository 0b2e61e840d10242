// rtmath.h — deterministic transcendental functions, bit-identical on gfx950 and x86-64.
//
// The reference calls CUDA libdevice sinf/cosf/expf/powf/acosf/... on the device and
// MSVC's libm on the host (e.g. bsdf.cuh:33, sky.cuh:167-191, kernel.cuh:105-109).
// Neither is available here, and ROCm's ocml and glibc disagree in the last ulp, which
// would flip Monte-Carlo decisions between the GPU kernels and the CPU oracle.  Every
// transcendental on the hot path therefore goes through this header, written with plain
// +,-,*,/, explicit fma and sqrt only (no contraction: every translation unit that includes this
// header is built with -ffp-contract=off), so each function returns the same bits on gfx950 and
// on x86-64 and kernel-vs-oracle parity can be tested bit-exact.
//
// Two families: float cores (sin/cos for |x| <= 64, atan, atan2, exp, log, pow — the per-sample
// and per-tap hot trig) in float arithmetic with error-free float-pair steps, faithful (within
// 1 ulp; tests/test_rtmath.py); and double-precision cores rounded once to float (correctly
// rounded in all but rare ties) for the rest (asin/acos, tan, large sin/cos arguments).
//
// sqrtf and float division stay native: both are correctly rounded on both sides
// (hipcc's default -fhip-fp32-correctly-rounded-divide-sqrt, SSE2 on the host).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD static inline
#endif

namespace rtm {

RT_HD double bits_to_double(uint64_t u) { union { uint64_t u; double d; } c; c.u = u; return c.d; }
RT_HD uint64_t double_to_bits(double d) { union { uint64_t u; double d; } c; c.d = d; return c.u; }
RT_HD float bits_to_float(uint32_t u) { union { uint32_t u; float f; } c; c.u = u; return c.f; }
RT_HD uint32_t float_to_bits(float f) { union { uint32_t u; float f; } c; c.f = f; return c.u; }

RT_HD bool d_isnan(double x) { return x != x; }
RT_HD double d_inf() { return bits_to_double(0x7FF0000000000000ull); }
RT_HD double d_nan() { return bits_to_double(0x7FF8000000000000ull); }
RT_HD double d_abs(double x) { return bits_to_double(double_to_bits(x) & 0x7FFFFFFFFFFFFFFFull); }

// pi/2 in double.  On the device it is materialised where it is used: as a plain constant the
// compiler hoists it into a VGPR pair for the whole kernel (it serves only the rare double
// paths below), and in the register-bound path-trace kernels that pair was spilled to scratch.
RT_HD double d_pio2() {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t lo, hi;
    asm volatile("v_mov_b32 %0, 0x54442d18" : "=v"(lo));
    asm volatile("v_mov_b32 %0, 0x3ff921fb" : "=v"(hi));
    return bits_to_double(((uint64_t)hi << 32) | lo);
#else
    return 1.57079632679489661923;
#endif
}

RT_HD double d_pi() {  // pi in double, materialised at its use on the device like d_pio2
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t lo, hi;
    asm volatile("v_mov_b32 %0, 0x54442d18" : "=v"(lo));
    asm volatile("v_mov_b32 %0, 0x400921fb" : "=v"(hi));
    return bits_to_double(((uint64_t)hi << 32) | lo);
#else
    return 3.14159265358979323846;
#endif
}

// round-half-away for the reduction index; exact for |x| < 2^52
RT_HD double d_round(double x) {
    double a = d_abs(x);
    if (a >= 4503599627370496.0) return x;
    double r = (double)(int64_t)(a + 0.5);
    return x < 0 ? -r : r;
}

// Horner step: product and sum rounded separately (no contraction), identically on both sides.
// (A fused v_fma_f64 chain measured 40+ more VGPRs in the shading kernels: the 64-bit
// coefficients then live in registers across the whole inlined path.)
RT_HD double d_mad(double a, double b, double c) { return a * b + c; }

// ---------------------------------------------------------------- exp2 / log2
RT_HD double exp2d(double x) {
    if (d_isnan(x)) return x;
    if (x >= 1024.0) return d_inf();
    if (x <= -1075.0) return 0.0;
    double n = d_round(x);
    double f = x - n;  // [-0.5, 0.5]
    // 2^f = sum (f ln2)^k / k!, k <= 11: truncation < 1e-14
    const double L = 0.69314718055994530942;
    const double c2 = L * L / 2.0, c3 = c2 * L / 3.0, c4 = c3 * L / 4.0, c5 = c4 * L / 5.0, c6 = c5 * L / 6.0;
    const double c7 = c6 * L / 7.0, c8 = c7 * L / 8.0, c9 = c8 * L / 9.0, c10 = c9 * L / 10.0, c11 = c10 * L / 11.0;
    double p = c11;
    p = d_mad(p, f, c10);
    p = d_mad(p, f, c9);
    p = d_mad(p, f, c8);
    p = d_mad(p, f, c7);
    p = d_mad(p, f, c6);
    p = d_mad(p, f, c5);
    p = d_mad(p, f, c4);
    p = d_mad(p, f, c3);
    p = d_mad(p, f, c2);
    p = d_mad(p, f, L);
    p = d_mad(p, f, 1.0);
    int ni = (int)n;
    if (ni > 1023) { p *= 2.0; ni -= 1; }
    if (ni >= -1022) return p * bits_to_double((uint64_t)(ni + 1023) << 52);
    // subnormal range: scale in two steps
    p *= bits_to_double((uint64_t)(ni + 600 + 1023) << 52);
    return p * bits_to_double((uint64_t)(-600 + 1023) << 52);
}

// natural log of x in (0, inf), exact exponent split + atanh series
RT_HD double logd_pos(double x) {
    uint64_t b = double_to_bits(x);
    int e = (int)((b >> 52) & 0x7FF);
    if (e == 0) {  // subnormal double (cannot come from a float input, kept for safety)
        x *= 18014398509481984.0;  // 2^54
        b = double_to_bits(x);
        e = (int)((b >> 52) & 0x7FF) - 54;
    }
    e -= 1023;
    double m = bits_to_double((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);  // [1,2)
    if (m > 1.41421356237309504880) { m *= 0.5; e += 1; }
    double s = (m - 1.0) / (m + 1.0);  // |s| <= 0.1716
    double s2 = s * s;
    // 2 atanh(s) = 2 sum s^(2k+1)/(2k+1), k <= 7: truncation < 1e-15
    double p = 1.0 / 15.0;
    p = d_mad(p, s2, 1.0 / 13.0);
    p = d_mad(p, s2, 1.0 / 11.0);
    p = d_mad(p, s2, 1.0 / 9.0);
    p = d_mad(p, s2, 1.0 / 7.0);
    p = d_mad(p, s2, 1.0 / 5.0);
    p = d_mad(p, s2, 1.0 / 3.0);
    p = d_mad(p, s2, 1.0);
    double lnm = 2.0 * s * p;
    return d_mad((double)e, 0.69314718055994530942, lnm);
}

RT_HD double logd(double x) {
    if (d_isnan(x)) return x;
    if (x < 0.0) return d_nan();
    if (x == 0.0) return -d_inf();
    if (x == d_inf()) return x;
    return logd_pos(x);
}

RT_HD double log2d(double x) {
    if (d_isnan(x)) return x;
    if (x < 0.0) return d_nan();
    if (x == 0.0) return -d_inf();
    if (x == d_inf()) return x;
    // split exponent exactly so log2 of powers of two is exact
    uint64_t b = double_to_bits(x);
    int e = (int)((b >> 52) & 0x7FF) - 1023;
    double m = bits_to_double((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
    if (m > 1.41421356237309504880) { m *= 0.5; e += 1; }
    return d_mad(logd_pos(m), 1.44269504088896340736, (double)e);
}

RT_HD double expd(double x) {
    if (d_isnan(x)) return x;
    return exp2d(x * 1.44269504088896340736);
}

// ---------------------------------------------------------------- trig
RT_HD void sincosd(double x, double& s, double& c) {
    if (d_isnan(x) || d_abs(x) == d_inf()) { s = d_nan(); c = d_nan(); return; }
    double k = d_round(x * 0.63661977236758134308);  // 2/pi
    // Cody-Waite, fdlibm constants (pio2_1 has 33 bits: k*pio2_1 exact for |k| < 2^20)
    double r = x - k * 1.57079632673412561417e+00;
    r = r - k * 6.07710050650619224932e-11;
    double r2 = r * r;
    // |r| <= pi/4: sin to r^13, cos to r^14 (truncation < 1e-13)
    double sp = 1.0 / 6227020800.0;  // 1/13!
    sp = d_mad(sp, r2, -1.0 / 39916800.0);
    sp = d_mad(sp, r2, 1.0 / 362880.0);
    sp = d_mad(sp, r2, -1.0 / 5040.0);
    sp = d_mad(sp, r2, 1.0 / 120.0);
    sp = d_mad(sp, r2, -1.0 / 6.0);
    double sr = d_mad(r * r2, sp, r);
    double cp = -1.0 / 87178291200.0;  // -1/14!
    cp = d_mad(cp, r2, 1.0 / 479001600.0);
    cp = d_mad(cp, r2, -1.0 / 3628800.0);
    cp = d_mad(cp, r2, 1.0 / 40320.0);
    cp = d_mad(cp, r2, -1.0 / 720.0);
    cp = d_mad(cp, r2, 1.0 / 24.0);
    cp = d_mad(cp, r2, -0.5);
    double cr = d_mad(r2, cp, 1.0);
    int q = (int)((int64_t)k & 3);
    if (q == 0) { s = sr; c = cr; }
    else if (q == 1) { s = cr; c = -sr; }
    else if (q == 2) { s = -sr; c = -cr; }
    else { s = -cr; c = sr; }
}

// atan on [0, inf)
RT_HD double atan_pos(double x) {
    bool inv = x > 1.0;
    if (inv) x = 1.0 / x;
    // atan(x) = pi/6 + atan((sqrt3 x - 1)/(x + sqrt3)) for x > tan(pi/12)
    bool shift = x > 0.26794919243112270647;
    if (shift) x = (x * 1.73205080756887729353 - 1.0) / (x + 1.73205080756887729353);
    double x2 = x * x;  // <= 0.0718
    // sum (-1)^k x^(2k+1)/(2k+1), k <= 9: truncation < 1e-13
    double p = -1.0 / 19.0;
    p = d_mad(p, x2, 1.0 / 17.0);
    p = d_mad(p, x2, -1.0 / 15.0);
    p = d_mad(p, x2, 1.0 / 13.0);
    p = d_mad(p, x2, -1.0 / 11.0);
    p = d_mad(p, x2, 1.0 / 9.0);
    p = d_mad(p, x2, -1.0 / 7.0);
    p = d_mad(p, x2, 1.0 / 5.0);
    p = d_mad(p, x2, -1.0 / 3.0);
    p = d_mad(p, x2, 1.0);
    double a = x * p;
    if (shift) a = 0.52359877559829887308 + a;
    if (inv) a = d_pio2() - a;
    return a;
}

RT_HD double atand(double x) {
    if (d_isnan(x)) return x;
    if (x == d_inf()) return d_pio2();
    if (x == -d_inf()) return -d_pio2();
    return x < 0 ? -atan_pos(-x) : atan_pos(x);
}

RT_HD double atan2d(double y, double x) {
    if (d_isnan(x) || d_isnan(y)) return d_nan();
    bool yneg = (double_to_bits(y) >> 63) != 0;
    bool xneg = (double_to_bits(x) >> 63) != 0;
    double ay = d_abs(y), ax = d_abs(x);
    double r;
    if (ay == 0.0) r = xneg ? d_pi() : 0.0;
    else if (ax == 0.0) r = d_pio2();
    else if (ax == d_inf() && ay == d_inf()) r = xneg ? d_pi() * 0.75 : d_pi() * 0.25;
    else if (ax == d_inf()) r = xneg ? d_pi() : 0.0;
    else if (ay == d_inf()) r = d_pio2();
    else {
        double a = atan_pos(ay / ax);
        r = xneg ? d_pi() - a : a;
    }
    return yneg ? -r : r;
}

// ---- float-result cores (the kernels' hot trig): double internals, short polynomials
//
// sin/cos for |x| <= 1e5: the same Cody-Waite reduction as sincosd, then minimax kernels on
// |r| <= pi/4 with relative error < 2^-37 (the sin/cos kernels of musl / FreeBSD
// k_sinf.c / k_cosf.c, coefficients in hex-float form), so the float result is the correctly
// rounded one except within ~2^-13 ulp of a rounding boundary.
RT_HD void sincosf_core(double x, double& s, double& c) {
    const double k = d_round(x * 0.63661977236758134308);
    const double r = (x - k * 1.57079632673412561417e+00) - k * 6.07710050650619224932e-11;
    const double z = r * r, w = z * z;
    const double S1 = -0x15555554cbac77.0p-55, S2 = 0x111110896efbb2.0p-59, S3 = -0x1a00f9e2cae774.0p-65,
                 S4 = 0x16cd878c3b46a7.0p-71;
    const double C0 = -0x1ffffffd0c5e81.0p-54, C1 = 0x155553e1053a42.0p-57, C2 = -0x16c087e80f1e27.0p-62,
                 C3 = 0x199342e0ee5069.0p-68;
    const double zr = z * r;
    const double sr = (r + zr * (S1 + z * S2)) + zr * w * (S3 + z * S4);
    const double cr = ((1.0 + z * C0) + w * C1) + (w * z) * (C2 + z * C3);
    const int q = (int)((int64_t)k & 3);
    if (q == 0) { s = sr; c = cr; }
    else if (q == 1) { s = cr; c = -sr; }
    else if (q == 2) { s = -sr; c = -cr; }
    else { s = -cr; c = sr; }
}

// atan(num / den) for 0 <= num, den finite, not both 0: one double division.  The ratio
// q = num/den is split as atan(c) + atan((num - c den) / (den + c num)) with c = i/8 nearest to
// min(q, 1/q) (i from a float estimate; any i keeps the identity exact), so |t| <= 1/16 + eps
// and five odd terms leave < 1e-15.
RT_HD double atan_ratio(double num, double den) {
    const bool swap = num > den;
    const double a = swap ? den : num, b = swap ? num : den;  // a <= b, a / b in [0, 1]
    const float qf = (float)a / (float)b;
    const int i = (int)(qf * 8.0f + 0.5f);
    const double c = (double)i * 0.125;
    const double t = (a - c * b) / (b + c * a);
    const double t2 = t * t;
    double p = 1.0 / 9.0;
    p = d_mad(p, t2, -1.0 / 7.0);
    p = d_mad(p, t2, 1.0 / 5.0);
    p = d_mad(p, t2, -1.0 / 3.0);
    const double at = d_mad(t * t2, p, t);
    // atan(i / 8), i = 0..8
    const double kAtan8[9] = {0.0, 0.12435499454676144, 0.24497866312686414, 0.35877067027057225, 0.4636476090008061, 0.5585993153435624, 0.6435011087932844, 0.7188299996216245, 0.7853981633974483};
    const double r = kAtan8[i] + at;
    return swap ? d_pio2() - r : r;
}

RT_HD double atan2f_core(double y, double x) {
    if (d_isnan(x) || d_isnan(y)) return d_nan();
    const bool yneg = (double_to_bits(y) >> 63) != 0;
    const bool xneg = (double_to_bits(x) >> 63) != 0;
    const double ay = d_abs(y), ax = d_abs(x);
    double r;
    if (ay == 0.0) r = xneg ? d_pi() : 0.0;
    else if (ax == 0.0) r = d_pio2();
    else if (ax == d_inf() && ay == d_inf()) r = xneg ? d_pi() * 0.75 : d_pi() * 0.25;
    else if (ax == d_inf()) r = xneg ? d_pi() : 0.0;
    else if (ay == d_inf()) r = d_pio2();
    else {
        const double a = atan_ratio(ay, ax);
        r = xneg ? d_pi() - a : a;
    }
    return yneg ? -r : r;
}

}  // namespace rtm

// ------------------------------------------------------------------ float API
// ---- float cores of exp / log / pow (the denoiser's per-tap weights, texture gamma, LOD).
// Single-precision arithmetic with explicit fmaf (v_fma_f32 on gfx950, the correctly rounded
// fmaf of libm on the host) and correctly rounded division: the same bits on both sides at
// about a quarter of the double path's latency.  log2 is carried as a float pair
// (hi + lo, ~2^-40 relative) so that pow stays within about one ulp even for large exponents.
namespace rtm {
RT_HD float f_fma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

// 2^f for |f| <= 0.5 + 2^-20: Taylor series of e^(f ln2) to degree 8 (truncation < 2e-10)
RT_HD float exp2_core(float f) {
    float p = 1.5252733804059840e-05f;  // ln2^7/7!
    p = f_fma(p, f, 1.5403530393381609e-04f);
    p = f_fma(p, f, 1.3333558146428443e-03f);
    p = f_fma(p, f, 9.6181291076284772e-03f);
    p = f_fma(p, f, 5.5504108664821580e-02f);
    p = f_fma(p, f, 2.4022650695910071e-01f);
    p = f_fma(p, f, 6.9314718055994531e-01f);
    return f_fma(p, f, 1.0f);
}

// p * 2^n for p in [0.7, 1.5], n in [-151, 128], one rounding (into the subnormal range too)
RT_HD float scale2(float p, int n) {
    if (n > 127) return p * 2.0f * bits_to_float((uint32_t)(n - 1 + 127) << 23);
    if (n >= -126) return p * bits_to_float((uint32_t)(n + 127) << 23);
    return (p * bits_to_float((uint32_t)(n + 64 + 127) << 23)) * bits_to_float((uint32_t)(-64 + 127) << 23);
}

// 2^(hi + lo), |lo| <= ulp(hi)
RT_HD float exp2_pair(float hi, float lo) {
    if (hi >= 128.0f) return bits_to_float(0x7F800000u);
    if (hi < -152.0f) return 0.0f;
    const float n = __builtin_rintf(hi);
    const float f = (hi - n) + lo;  // hi - n is exact
    return scale2(exp2_core(f), (int)n);
}

// 1 / d for d in [1.70, 2.42] (log2_pair's 2 + r) to ~2^-24 relative: the linear minimax seed
// (relative error 1.5 %) and two Newton steps, fma only — the same bits on the GPU and the host,
// unlike the hardware reciprocal, and without the division's scale / fixup sequence.
RT_HD float recip_log_den(float d) {
    float y = f_fma(-0.239016f, d, 0.985076f);  // c1 (a + b) = 0.98508, c1 = 2 / (ab + (a + b)^2 / 4)
    y = f_fma(y, f_fma(-d, y, 1.0f), y);
    return f_fma(y, f_fma(-d, y, 1.0f), y);
}

// log2(x) = hi + lo for finite x > 0 (~2^-44 relative).  Division-free (kDiv false): r / (2 + r)
// is r times the Newton reciprocal above, corrected once by its exact remainder to within an ulp (so
// the second remainder, which carries the low part, is exact as well).  kDiv: the two correctly
// rounded divisions instead — the path tracer's variant (rt_powf_div / rt_log2f_div): the
// reciprocal's extra registers pushed the fused bounce chain, which holds 168 VGPRs, into scratch.
// The two variants can differ in the last bit; each call site uses the same one on the GPU and in
// the oracle.
template <bool kDiv = false>
RT_HD void log2_pair_t(float x, float& hi, float& lo) {
    uint32_t b = float_to_bits(x);
    int e = 0;
    if (b < 0x00800000u) {  // subnormal: scale by 2^23
        x *= 8388608.0f;
        b = float_to_bits(x);
        e = -23;
    }
    e += (int)(b >> 23) - 127;
    float m = bits_to_float((b & 0x007FFFFFu) | 0x3F800000u);  // [1, 2)
    if (m > 1.41421354f) { m *= 0.5f; e += 1; }
    const float r = m - 1.0f;  // exact
    // ln(1 + r) = 2 atanh(s), s = r / (2 + r), s carried as s_hi + s_lo
    const float d = 2.0f + r, dl = r - (d - 2.0f);  // 2 + r exactly as d + dl
    float s, sl;
    if (kDiv) {
        s = r / d;
        sl = (f_fma(-s, d, r) - s * dl) / d;
    } else {
        const float y = recip_log_den(d);
        const float s0 = r * y;
        s = f_fma(f_fma(-s0, d, r), y, s0);    // r / d within an ulp
        sl = (f_fma(-s, d, r) - s * dl) * y;  // the exact remainder over d: r / (2 + r) - s
    }
    const float s2 = s * s;
    float q = 1.0f / 13.0f;
    q = f_fma(q, s2, 1.0f / 11.0f);
    q = f_fma(q, s2, 1.0f / 9.0f);
    q = f_fma(q, s2, 1.0f / 7.0f);
    q = f_fma(q, s2, 1.0f / 5.0f);
    q = f_fma(q, s2, 1.0f / 3.0f);
    const float lnh = 2.0f * s;                       // exact
    const float lnl = 2.0f * sl + (2.0f * s) * (s2 * q);
    // times log2(e) = Lh + Ll, plus the exponent
    const float Lh = 1.44269502162933349609f, Ll = 1.9259629911783e-08f;
    const float ph = lnh * Lh;
    const float pl = f_fma(lnh, Lh, -ph) + (f_fma(lnh, Ll, lnl * Lh));
    const float fe = (float)e;
    const float sh = fe + ph;
    const float err = (fe - sh) + ph;  // |fe| >= 1 > |ph| or fe == 0: exact two-sum
    hi = sh;
    lo = err + pl;
    const float t = hi + lo;  // renormalise
    lo = lo - (t - hi);
    hi = t;
}
RT_HD void log2_pair(float x, float& hi, float& lo) { log2_pair_t<false>(x, hi, lo); }

// ---- float cores of sin / cos / atan / atan2 (the path tracer's per-sample trig: the aperture
// disk, cosine-weighted and light directions, the sky lookup's longitude).  Float arithmetic with
// explicit fmaf and error-free float-pair steps where the last bits are decided, so the result is
// the same on the GPU and the host and faithful (within 1 ulp of the exact value; the double path
// above is kept for arguments outside the reduced range).  Constants: pi/2 = C1 + C2 + C3 + C4
// with C1..C3 of 18 significant bits; musl's __sindf / __cosdf kernels (relative error < 2^-37 on
// |r| <= pi/4) rounded to float; atan(i/8) and pi/2 - atan(i/8) as float pairs.
constexpr float kPio2C1 = 0x1.921f8p+0f, kPio2C2 = 0x1.aa22p-19f, kPio2C3 = 0x1.68c2p-39f, kPio2C4 = 0x1.a62634p-58f;
constexpr float kSinS1 = -0x1.555556p-3f, kSinS2 = 0x1.111108p-7f, kSinS3 = -0x1.a00f9ep-13f, kSinS4 = 0x1.6cd878p-19f;
constexpr float kCosC0d = 0x1.79d0cp-29f, kCosC1 = 0x1.55553ep-5f, kCosC2 = -0x1.6c087ep-10f, kCosC3 = 0x1.99342ep-16f;  // kCosC0d = C0 + 1/2
constexpr float kPiHi = 0x1.921fb6p+1f, kPiLo = -0x1.777a5cp-24f, kPio2Hi = 0x1.921fb6p+0f, kPio2Lo = -0x1.777a5cp-25f;

RT_HD void two_sum(float a, float b, float& s, float& e) {
    s = a + b;
    const float bb = s - a;
    e = (a - (s - bb)) + (b - bb);
}

// sin x, cos x for |x| <= 64 (|k| <= 41: k C1, k C2, k C3 are exact, C1..C3 having 18 significant
// bits), the reduced argument x - k pi/2 carried as the float pair rh + rl
RT_HD void sincosf_fcore(float x, float& sn, float& cs) {
    const float k = __builtin_rintf(x * 0.636619772f);
    const float r1 = f_fma(-k, kPio2C1, x);  // exact
    float rh, rl, e;
    two_sum(r1, -(k * kPio2C2), rh, rl);
    two_sum(rh, -(k * kPio2C3), rh, e);
    rl = f_fma(-k, kPio2C4, rl + e);
    two_sum(rh, rl, rh, rl);  // renormalise: |rl| <= ulp(rh) / 2
    const float z = rh * rh;
    const float zl = f_fma(rh, rh, -z);                // z + zl = rh^2 exactly
    const float hz = 0.5f * z;
    // sin(rh + rl) = rh + rh z S(z) + rl (1 - z/2)
    const float sp = z * f_fma(z, f_fma(z, f_fma(z, kSinS4, kSinS3), kSinS2), kSinS1);
    const float s = rh + f_fma(rh, sp, rl * (1.0f - hz));
    // cos(rh + rl) = (1 - z/2) + [z (C0 + 1/2) + z^2 C(z) - zl/2 - rh rl], 1 - z/2 split exactly
    const float w = 1.0f - hz;
    const float we = (1.0f - w) - hz;
    const float cp = f_fma(z * z, f_fma(z, f_fma(z, kCosC3, kCosC2), kCosC1), z * kCosC0d);
    const float c = w + (((we - 0.5f * zl) + cp) - rh * rl);
    const int q = (int)k & 3;
    sn = q == 0 ? s : q == 1 ? c : q == 2 ? -s : -c;
    cs = q == 0 ? c : q == 1 ? -s : q == 2 ? -c : s;
}

// atan(num / den) as hi + lo (hi a table value, lo the rest) for 0 <= num, den finite, not both 0:
// with a <= b the smaller and larger of the two, atan(a / b) = atan(c) + atan(t),
// t = (a - c b) / (b + c a), c = i / 8 nearest to a / b (i = 1 taken as 0, so that |atan t| stays
// below a third of the result when i > 0), and the odd series of atan t to t^13 (|t| < 3/16).
RT_HD void atan_ratio_f(float num, float den, float& hi, float& lo) {
    const bool swap = num > den;
    const float a = swap ? den : num, b = swap ? num : den;
    int i = (int)((a / b) * 8.0f + 0.5f);
    if (i == 1) i = 0;
    const float c = (float)i * 0.125f;
    const float t = f_fma(-c, b, a) / f_fma(c, a, b);
    const float t2 = t * t;
    float p = 1.0f / 13.0f;
    p = f_fma(p, t2, -1.0f / 11.0f);
    p = f_fma(p, t2, 1.0f / 9.0f);
    p = f_fma(p, t2, -1.0f / 7.0f);
    p = f_fma(p, t2, 1.0f / 5.0f);
    p = f_fma(p, t2, -1.0f / 3.0f);
    const float at = f_fma(t * t2, p, t);
    // atan(i/8) (row 0) and pi/2 - atan(i/8) (row 1) as float pairs, i = 0, 2..8 (entry 1 repeats
    // entry 0): one table read per value (a select chain here became a dozen exec-mask branches)
    static constexpr float kTh[2][9] = {
        {0.0f, 0.0f, 0x1.f5b76p-3f, 0x1.6f6194p-2f, 0x1.dac67p-2f, 0x1.1e00bap-1f, 0x1.4978fap-1f, 0x1.700a7cp-1f, 0x1.921fb6p-1f},
        {0x1.921fb6p+0f, 0x1.921fb6p+0f, 0x1.5368cap+0f, 0x1.36475p+0f, 0x1.1b6e1ap+0f, 0x1.031f58p+0f, 0x1.dac67p-1f, 0x1.b434eep-1f, 0x1.921fb6p-1f}};
    static constexpr float kTl[2][9] = {
        {0.0f, 0.0f, -0x1.b4dfc8p-29f, 0x1.e4defp-30f, 0x1.586ed4p-28f, 0x1.7bdfd6p-26f, 0x1.934f7p-28f, 0x1.5e118cp-27f, -0x1.777a5cp-26f},
        {-0x1.777a5cp-25f, -0x1.777a5cp-25f, -0x1.5c2c6p-25f, 0x1.e57aaep-27f, -0x1.a28838p-25f, -0x1.ab5242p-28f, 0x1.586ed4p-27f, 0x1.8809fep-28f, -0x1.777a5cp-26f}};
    const int row = swap ? 1 : 0;
    const float tl = kTl[row][i];
    hi = kTh[row][i];
    lo = swap ? tl - at : tl + at;
}

RT_HD float atan2f_fcore(float y, float x) {
    const uint32_t yb = float_to_bits(y), xb = float_to_bits(x);
    const float ay = bits_to_float(yb & 0x7FFFFFFFu), ax = bits_to_float(xb & 0x7FFFFFFFu);
    float hi, lo;
    atan_ratio_f(ay, ax, hi, lo);
    float r;
    if (xb >> 31) {  // pi - atan(|y| / |x|)
        float s, e;
        two_sum(kPiHi, -hi, s, e);
        r = s + ((e + kPiLo) - lo);
    } else {
        r = hi + lo;
    }
    return (yb >> 31) ? -r : r;
}
}  // namespace rtm

// a / b for a divisor b that many lanes share (the denoiser's sigmas), with c = RN(1 / b) computed
// once: two remainder corrections (Markstein) turn a * c into the IEEE quotient as long as the
// quotient and the remainders stay normal — for 2^-20 <= |b| <= 2^20 and a = 0 or
// 2^-30 <= |a| <= 2^30 (every such float a, for the denoiser's default sigmas and a sample of
// others: tools/div_exhaustive.c, tests/test_rtmath.py).  Zero, infinite and NaN a return a * c,
// which is the quotient there too.  Five instructions instead of the division's ten and its
// reciprocal; callers keep the division for a divisor outside that range.
RT_HD float rt_div_rcp(float a, float b, float c) {
    const float q0 = a * c;
    const float q1 = rtm::f_fma(rtm::f_fma(-q0, b, a), c, q0);
    const float q2 = rtm::f_fma(rtm::f_fma(-q1, b, a), c, q1);
    return (a != 0.0f && __builtin_fabsf(q0) < rtm::bits_to_float(0x7F800000u)) ? q2 : q0;
}
// whether rt_div_rcp may stand for a / b (host side, once per divisor)
inline bool rt_div_rcp_ok(float b) {
    const float ab = b < 0.0f ? -b : b;
    return ab >= 0x1p-20f && ab <= 0x1p20f;
}

// x / 65535 for a 16-bit texel value x (Load2DFuncUshort4's unorm conversion), correctly rounded:
// the product with c = RN(1/65535) corrected by one fma step (Markstein).  Equal to the IEEE
// division for every x in [0, 65535] (checked exhaustively: tests/test_rtmath.py); 3 instructions
// instead of the division's ~10, four times per texel tap.
RT_HD float rt_unorm16(uint32_t x) {
    const float xf = (float)x, c = rtm::bits_to_float(0x37800080u);  // RN(1 / 65535)
    const float q = xf * c;
    return rtm::f_fma(rtm::f_fma(-q, 65535.0f, xf), c, q);
}

RT_HD float rt_exp2f(float x) {
    if (x != x) return x;
    return rtm::exp2_pair(x, 0.0f);
}

RT_HD float rt_expf(float x) {
    if (x != x) return x;
    if (x > 89.0f) return rtm::bits_to_float(0x7F800000u);
    if (x < -104.0f) return 0.0f;
    // Cody-Waite: x = n ln2 + r, ln2 = 0.693145752 (16 bits) + 1.42860677e-06
    const float n = __builtin_rintf(x * 1.44269502162933349609f);
    float r = rtm::f_fma(-n, 0.693145751953125f, x);
    r = rtm::f_fma(-n, 1.428606765330187e-06f, r);
    // e^r, |r| <= 0.35: Taylor to degree 8
    float p = 2.4801587301587302e-05f;
    p = rtm::f_fma(p, r, 1.9841269841269841e-04f);
    p = rtm::f_fma(p, r, 1.3888888888888889e-03f);
    p = rtm::f_fma(p, r, 8.3333333333333333e-03f);
    p = rtm::f_fma(p, r, 4.1666666666666667e-02f);
    p = rtm::f_fma(p, r, 1.6666666666666667e-01f);
    p = rtm::f_fma(p, r, 0.5f);
    p = rtm::f_fma(p, r, 1.0f);
    p = rtm::f_fma(p, r, 1.0f);
    return rtm::scale2(p, (int)n);
}

template <bool kDiv = false>
RT_HD float rt_log2f_t(float x) {
    if (x != x) return x;
    if (x < 0.0f) return rtm::bits_to_float(0x7FC00000u);
    if (x == 0.0f) return rtm::bits_to_float(0xFF800000u);
    if (x == rtm::bits_to_float(0x7F800000u)) return x;
    float h, l;
    rtm::log2_pair_t<kDiv>(x, h, l);
    return h + l;
}
RT_HD float rt_log2f(float x) { return rt_log2f_t<false>(x); }
RT_HD float rt_log2f_div(float x) { return rt_log2f_t<true>(x); }

RT_HD float rt_logf(float x) {
    if (x != x) return x;
    if (x < 0.0f) return rtm::bits_to_float(0x7FC00000u);
    if (x == 0.0f) return rtm::bits_to_float(0xFF800000u);
    if (x == rtm::bits_to_float(0x7F800000u)) return x;
    float h, l;
    rtm::log2_pair(x, h, l);
    // times ln2 = 0.693147182 + -1.90465421e-09
    const float Nh = 0.693147182464599609375f, Nl = -1.904654212125e-09f;
    const float ph = h * Nh;
    return ph + (rtm::f_fma(h, Nh, -ph) + rtm::f_fma(h, Nl, l * Nh));
}
RT_HD float rt_log10f(float x) { return (float)(rtm::logd((double)x) * 0.43429448190325182765); }
RT_HD void rt_sincos_d(float x, double& s, double& c) {
    if (rtm::d_abs((double)x) <= 1e5) rtm::sincosf_core((double)x, s, c);  // NaN and inf fail the test
    else rtm::sincosd((double)x, s, c);
}
RT_HD void rt_sincosf(float x, float* s, float* c) {
    if (__builtin_fabsf(x) <= 64.0f) {  // NaN and inf fail the test
        rtm::sincosf_fcore(x, *s, *c);
        return;
    }
    double sd, cd;
    rt_sincos_d(x, sd, cd);
    *s = (float)sd;
    *c = (float)cd;
}
RT_HD float rt_sinf(float x) { float s, c; rt_sincosf(x, &s, &c); return s; }
RT_HD float rt_cosf(float x) { float s, c; rt_sincosf(x, &s, &c); return c; }
RT_HD float rt_tanf(float x) { double s, c; rt_sincos_d(x, s, c); return (float)(s / c); }
RT_HD float rt_atanf(float x) {
    if (x != x) return x;
    if (x == 0.0f) return x;
    const float ax = __builtin_fabsf(x);
    if (ax == rtm::bits_to_float(0x7F800000u)) return x > 0.0f ? 1.57079632679489661923f : -1.57079632679489661923f;
    float hi, lo;
    rtm::atan_ratio_f(ax, 1.0f, hi, lo);
    const float r = hi + lo;
    return x < 0.0f ? -r : r;
}
RT_HD float rt_atan2f(float y, float x) {
    const float ay = __builtin_fabsf(y), ax = __builtin_fabsf(x);
    // finite, not both zero and neither zero: the float core; the rest (zeros, infinities, NaN)
    // take the double path's C99 special cases
    if (ay > 0.0f && ax > 0.0f && ay < rtm::bits_to_float(0x7F800000u) && ax < rtm::bits_to_float(0x7F800000u))
        return rtm::atan2f_fcore(y, x);
    return (float)rtm::atan2f_core((double)y, (double)x);
}
RT_HD float rt_asinf(float x) {
    double d = (double)x;
    if (!(d >= -1.0 && d <= 1.0)) return (float)rtm::d_nan();
    return (float)rtm::atan2f_core(d, __builtin_sqrt((1.0 - d) * (1.0 + d)));
}
RT_HD float rt_acosf(float x) {
    double d = (double)x;
    if (!(d >= -1.0 && d <= 1.0)) return (float)rtm::d_nan();
    return (float)rtm::atan2f_core(__builtin_sqrt((1.0 - d) * (1.0 + d)), d);
}

// powf with the C99 special cases that matter on the path (x >= 0 in practice); kDiv: log2_pair_t's
// division variant (rt_powf_div, the path tracer's)
template <bool kDiv = false>
RT_HD float rt_powf_t(float xf, float yf) {
    // common case first (textures' ^2.2, the tone mapper's gamma): x positive and finite, y not
    // NaN.  None of the special cases below applies to it, so this is the same computation as
    // the tail of the general path, without its double-precision classification.
    if (xf > 0.0f && xf < rtm::bits_to_float(0x7F800000u) && yf == yf) {
        if (xf == 1.0f) return 1.0f;  // exact (the denoiser's equal normals: a whole wave skips the log)
        float lh, ll;
        rtm::log2_pair_t<kDiv>(xf, lh, ll);
        const float th = yf * lh;
        const float tl = rtm::f_fma(yf, lh, -th) + yf * ll;
        return rtm::exp2_pair(th, tl);
    }
    // +0 to a positive power (the denoiser's clamped normal weights at right angles): the general
    // path's answer, without its double-precision classification
    if (rtm::float_to_bits(xf) == 0u && yf > 0.0f) return 0.0f;
    double x = (double)xf, y = (double)yf;
    if (y == 0.0) return 1.0f;
    if (x == 1.0) return 1.0f;
    if (rtm::d_isnan(x) || rtm::d_isnan(y)) return (float)rtm::d_nan();
    bool yint = false, yodd = false;
    if (rtm::d_abs(y) < 9007199254740992.0) {
        double t = (double)(int64_t)y;
        yint = (t == y);
        if (yint) yodd = ((int64_t)y & 1) != 0;
    } else {
        yint = true;
    }
    if (x == 0.0) {
        bool neg0 = (rtm::double_to_bits(x) >> 63) != 0;
        if (y > 0) return (neg0 && yodd) ? -0.0f : 0.0f;
        return (neg0 && yodd) ? (float)-rtm::d_inf() : (float)rtm::d_inf();
    }
    double sign = 1.0;
    if (x < 0.0) {
        if (!yint) return (float)rtm::d_nan();
        if (yodd) sign = -1.0;
        x = -x;
    }
    if (x == rtm::d_inf()) return (float)(sign * (y > 0 ? rtm::d_inf() : 0.0));
    // exp2(y log2 x) with log2 x as a float pair and the product's rounding error kept
    float lh, ll;
    rtm::log2_pair_t<kDiv>((float)x, lh, ll);
    const float th = yf * lh;
    const float tl = rtm::f_fma(yf, lh, -th) + yf * ll;
    const float r = rtm::exp2_pair(th, tl);
    return sign < 0.0 ? -r : r;
}
RT_HD float rt_powf(float xf, float yf) { return rt_powf_t<false>(xf, yf); }
RT_HD float rt_powf_div(float xf, float yf) { return rt_powf_t<true>(xf, yf); }

// IEEE float -> binary16, round to nearest even (matches __float2half_rn / v_cvt_f16_f32)
//
// On gfx950 both conversions are the hardware v_cvt_f16_f32 / v_cvt_f32_f16 (round to nearest
// even, half denormals preserved in the default float mode): the same bits as the integer
// restatements below for every non-NaN input.  NaNs are canonicalised to sign | 0x7E00 after the
// hardware float -> half conversion, by a select (a branch here costs a dozen instructions per
// conversion in the per-tap loops); half -> float quiets a NaN and keeps its payload, as IEEE 754
// conversion does on both sides.
RT_HD uint16_t rt_f2h(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint16_t hv = __builtin_bit_cast(uint16_t, (_Float16)f);
    const uint16_t qn = (uint16_t)(((rtm::float_to_bits(f) >> 16) & 0x8000u) | 0x7E00u);
    return f != f ? qn : hv;
#endif
    uint32_t x = rtm::float_to_bits(f);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t ax = x & 0x7FFFFFFFu;
    if (ax >= 0x7F800000u) return (uint16_t)(sign | (ax > 0x7F800000u ? 0x7E00u : 0x7C00u));
    if (ax >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u);  // rounds to >= 65520 -> inf
    if (ax < 0x38800000u) {                                      // half subnormal or zero
        if (ax < 0x33000000u) return (uint16_t)sign;             // < 2^-25 rounds to 0
        uint32_t mant = (ax & 0x7FFFFFu) | 0x800000u;
        int shift = 126 - (int)(ax >> 23);                       // 14..24
        uint32_t h = mant >> (shift);
        uint32_t rem = mant & ((1u << shift) - 1u);
        uint32_t half = 1u << (shift - 1);
        if (rem > half || (rem == half && (h & 1u))) h += 1u;
        return (uint16_t)(sign | h);
    }
    uint32_t h = ((ax >> 13) - ((127u - 15u) << 10));
    uint32_t rem = ax & 0x1FFFu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h += 1u;
    return (uint16_t)(sign | h);
}

RT_HD float rt_h2f(uint16_t h) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (float)__builtin_bit_cast(_Float16, h);
#endif
    uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
    uint32_t e = ((uint32_t)h >> 10) & 0x1Fu;
    uint32_t m = (uint32_t)h & 0x3FFu;
    if (e == 0x1F) return rtm::bits_to_float(sign | 0x7F800000u | (m << 13) | (m ? 0x00400000u : 0u));  // NaN quieted
    if (e == 0) {
        if (m == 0) return rtm::bits_to_float(sign);
        // subnormal: m * 2^-24
        float v = (float)m * 5.9604644775390625e-08f;
        return sign ? -v : v;
    }
    return rtm::bits_to_float(sign | ((e + 112u) << 23) | (m << 13));
}
