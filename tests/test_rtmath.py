"""rtmath.h (the deterministic transcendentals shared by kernels and oracle) vs float64 numpy."""
import math

import numpy as np
import pytest

FNS = {
    "sin": (np.sin, (-50, 50)), "cos": (np.cos, (-50, 50)), "tan": (np.tan, (-1.5, 1.5)),
    "atan": (np.arctan, (-100, 100)), "acos": (np.arccos, (-1, 1)), "asin": (np.arcsin, (-1, 1)),
    "exp": (np.exp, (-80, 80)), "exp2": (np.exp2, (-120, 120)), "log": (np.log, (1e-30, 1e30)),
    "log2": (np.log2, (1e-30, 1e30)), "log2_div": (np.log2, (1e-30, 1e30)),
}


def ulp_err(got, ref):
    ref32 = np.float32(ref)
    if not np.isfinite(ref32):
        return 0 if got == ref32 else 99
    return abs(int(np.float32(got).view(np.int32)) - int(ref32.view(np.int32)))


@pytest.mark.parametrize("name", sorted(FNS))
def test_rtmath_faithful(oracle, name):
    f, (lo, hi) = FNS[name]
    rng = np.random.default_rng(7)
    if name in ("log", "log2", "log2_div"):
        xs = np.float32(10.0) ** rng.uniform(-30, 30, 3000).astype(np.float32)
    else:
        xs = rng.uniform(lo, hi, 3000).astype(np.float32)
    worst = 0
    for x in xs:
        worst = max(worst, ulp_err(oracle.rtmath(name, float(x)), f(np.float64(x))))
    assert worst <= 1, "%s worst ulp %d" % (name, worst)


def test_rtmath_pow_atan2(oracle):
    rng = np.random.default_rng(3)
    worst = 0
    for _ in range(3000):
        x, y = np.float32(rng.uniform(0, 20)), np.float32(rng.uniform(-8, 8))
        worst = max(worst, ulp_err(oracle.rtmath("pow", float(x), float(y)), np.float64(x) ** np.float64(y)))
        worst = max(worst, ulp_err(oracle.rtmath("pow_div", float(x), float(y)), np.float64(x) ** np.float64(y)))
        a, b = np.float32(rng.uniform(-5, 5)), np.float32(rng.uniform(-5, 5))
        worst = max(worst, ulp_err(oracle.rtmath("atan2", float(a), float(b)), np.arctan2(np.float64(a), np.float64(b))))
    assert worst <= 1


def test_rtmath_special_cases(oracle):
    assert oracle.rtmath("pow", 0.0, 2.0) == 0.0
    assert oracle.rtmath("pow", 2.0, 0.0) == 1.0
    assert math.isinf(oracle.rtmath("pow", 0.0, -1.0))
    assert math.isnan(oracle.rtmath("acos", 1.5))
    assert oracle.rtmath("acos", 1.0) == 0.0
    assert oracle.rtmath("exp", -200.0) == 0.0
    assert math.isinf(oracle.rtmath("exp", 200.0))
    assert oracle.rtmath("log2", 8.0) == 3.0
    assert math.isinf(oracle.rtmath("log", 0.0)) and oracle.rtmath("log", 0.0) < 0
    assert oracle.rtmath("atan2", 0.0, -1.0) == np.float32(np.pi)


def test_rtmath_float_pow_large_exponent(oracle):
    """powf(x, 100) (the denoiser's normal weight): float-pair log2 keeps it within 2 ulp."""
    rng = np.random.default_rng(11)
    worst = 0
    for x in rng.uniform(0, 1, 3000).astype(np.float32):
        worst = max(worst, ulp_err(oracle.rtmath("pow", float(x), 100.0), np.float64(x) ** 100.0))
    assert worst <= 2, worst


def test_rtmath_subnormal_range(oracle):
    rng = np.random.default_rng(5)
    worst = 0
    for x in rng.uniform(-149, -126, 2000).astype(np.float32):
        worst = max(worst, ulp_err(oracle.rtmath("exp2", float(x)), np.exp2(np.float64(x))))
    for x in (np.float32(2.0) ** rng.uniform(-149, -126, 2000)).astype(np.float32):
        worst = max(worst, ulp_err(oracle.rtmath("log2", float(x)), np.log2(np.float64(x))))
    assert worst <= 1, worst


def test_rtmath_float_trig_cores_near_quadrant_boundaries(oracle):
    """sin/cos through the float core (|x| <= 64) stay faithful where the reduced argument is
    tiny: floats within a few hundred ulps of k pi/2, k = -40..40 (the float-pair reduction)."""
    worst = 0
    for k in range(-40, 41, 3):
        c = np.float32(k * np.pi / 2)
        for d in range(-60, 61, 7):
            x = (c.view(np.int32) + np.int32(d)).view(np.float32)
            if abs(float(x)) > 64:
                continue
            worst = max(worst, ulp_err(oracle.rtmath("sin", float(x)), np.sin(np.float64(x))))
            worst = max(worst, ulp_err(oracle.rtmath("cos", float(x)), np.cos(np.float64(x))))
    assert worst <= 1, worst


def test_rtmath_atan2_quadrants_and_ratios(oracle):
    """atan2 through the float core over all four quadrants and |y/x| from 1e-6 to 1e6."""
    rng = np.random.default_rng(13)
    worst = 0
    for _ in range(3000):
        x = np.float32(rng.choice([-1, 1]) * 10.0 ** rng.uniform(-3, 3))
        y = np.float32(rng.choice([-1, 1]) * 10.0 ** rng.uniform(-3, 3))
        worst = max(worst, ulp_err(oracle.rtmath("atan2", float(y), float(x)), np.arctan2(np.float64(y), np.float64(x))))
    assert worst <= 1, worst


def test_unorm16_equals_division(oracle):
    """rt_unorm16 (x * RN(1/65535) with one fma correction) is the IEEE quotient x / 65535 for all
    65,536 texel values: the texture path's conversion is exact, not approximate."""
    assert oracle.lib().orc_unorm16_mismatches() == 0


@pytest.mark.parametrize("d", [np.float32(3.1415926535897932), np.float32(6.2831853071795865)])
def test_div_by_pi_constants_equal_division(oracle, d):
    """pt_common.h div_pi / div_two_pi: x * RN(1/d) plus one fma correction is the IEEE quotient x / d
    for finite |x| >= 2^-100 (tools/div_exhaustive.c checks all 2^32 patterns; here every 4,099th)."""
    assert oracle.lib().orc_div_const_mismatches(float(d), 4099) == 0


_SIGMAS = [0.1, 0.01, 100.0] + [float(np.float32(2.0) ** e) for e in np.random.default_rng(17).uniform(-20, 20, 6)]


@pytest.mark.parametrize("d", _SIGMAS)
def test_div_rcp_equals_division(oracle, d):
    """rtmath.h rt_div_rcp (x * RN(1/d) with two remainder corrections: the denoiser's depth weights
    (dV - d) / sigma) is the IEEE quotient for x = 0, +-inf, NaN and every 2^-30 <= |x| <= 2^30, for
    divisors in [2^-20, 2^20]: the defaults 0.1, 0.01 (tools/div_exhaustive.c checks all 2^32 patterns
    for those) and six random ones; here every 4,099th pattern."""
    assert oracle.lib().orc_div_rcp_mismatches(float(np.float32(d)), 4099) == 0
