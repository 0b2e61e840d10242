"""The denoiser's packed-pair transcendentals (csrc/rtmath_pk.h: two taps' pow / expf / depth ratio
in one register pair) against their scalar rtmath.h forms on the GPU and against the CPU oracle,
bit for bit, over edge values (zeros of both signs, 1, subnormals, the range ends of exp and of
the reciprocal division) and random arguments.  The full-frame denoise tests cover the same code
inside the passes; this pins the functions on their own."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def run(lib, fn, x, y=0.0, c=0.0):
    import torch

    xd = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).cuda()
    pk = torch.empty_like(xd)
    sc = torch.empty_like(xd)
    assert lib.rt_debug_pk_math(fn, xd.data_ptr(), y, c, pk.data_ptr(), sc.data_ptr(), xd.numel()) == 0
    return pk.cpu().numpy(), sc.cpu().numpy()


def same_bits(a, b):
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.fixture(scope="module")
def lib():
    import rtx

    return rtx.load_library()


def pow_inputs(rng):
    edge = np.array([0.0, -0.0, 1.0, 1e-45, 1e-40, 1.17549435e-38, 1e-30, 0.5, 0.9999999, 1.0000001, 2.0,
                     65504.0, 1e10, 3.4e38], np.float32)
    return np.concatenate([edge, rng.random(200000, dtype=np.float32),
                           (10.0 ** rng.uniform(-44, 38, 200000)).astype(np.float32)])


@pytest.mark.parametrize("y", [128.0, 64.0, 16.0, 2.2, 1.0 / 2.2, 1.0, 3.0, 7.0, 0.5, 1e-3, 64.5])
def test_pow_pairs_equal_scalar_and_oracle(lib, oracle, y):
    x = pow_inputs(np.random.default_rng(int(y * 1000)))
    pk, sc = run(lib, 0, x, y)
    assert same_bits(pk, sc), np.nonzero(pk.view(np.uint32) != sc.view(np.uint32))[0][:8]
    ref = oracle.rtmath_n(0, x, y)
    assert same_bits(sc, ref), np.nonzero(sc.view(np.uint32) != ref.view(np.uint32))[0][:8]
    assert np.signbit(pk[1]) == (y in (1.0, 3.0, 7.0))  # pow(-0, odd integer) = -0


def test_expf_pairs_equal_scalar_and_oracle(lib, oracle):
    rng = np.random.default_rng(5)
    edge = np.array([0.0, -0.0, 88.7, 89.0, 89.01, -103.9, -104.0, -104.01, -87.3, -100.0, np.inf, -np.inf,
                     np.nan, -1e-30], np.float32)
    x = np.concatenate([edge, rng.uniform(-110, 95, 400000).astype(np.float32),
                        -(rng.random(100000, dtype=np.float32) ** 2) * 50])
    pk, sc = run(lib, 1, x)
    nan = np.isnan(sc)
    assert np.array_equal(np.isnan(pk), nan)
    assert same_bits(pk[~nan], sc[~nan])
    ref = oracle.rtmath_n(1, x)
    assert same_bits(sc[~nan], ref[~nan])


@pytest.mark.parametrize("sigma", [1.0, 0.1, 4.0, 1e-3, 1e5])
def test_depth_ratio_pairs_equal_scalar_and_oracle(lib, oracle, sigma):
    rng = np.random.default_rng(11)
    c = np.float32(1.0) / np.float32(sigma)
    x = np.concatenate([np.array([0.0, -0.0, 1e-30, -1e-30, 1e30, np.inf, -np.inf], np.float32),
                        rng.standard_normal(300000).astype(np.float32) * np.float32(10.0) ** rng.integers(-6, 6, 300000).astype(np.float32)])
    pk, sc = run(lib, 2, x, sigma, float(c))
    assert same_bits(pk, sc)
    assert same_bits(sc, oracle.rtmath_n(2, x, sigma, float(c)))
