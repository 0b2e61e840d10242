"""The half <-> float conversions the kernels rely on (csrc/rtmath.h rt_f2h / rt_h2f use the hardware
v_cvt_f16_f32 / v_cvt_f32_f16 on the device, with NaN canonicalised to sign|0x7E00 after float ->
half) against the oracle's integer restatements, over every bit pattern: all 65,536 halves and all
2^32 floats (the conversions of torch's float32 <-> float16 casts on the GPU are the same hardware
instructions)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_half_to_float_all_halves(oracle):
    import torch

    h = np.arange(65536, dtype=np.uint32).astype(np.uint16)
    got = torch.from_numpy(h.view(np.int16)).cuda().view(torch.float16).float().cpu().numpy().view(np.uint32)
    ref = oracle.h2f(h).view(np.uint32)
    assert np.array_equal(got, ref), np.nonzero(got != ref)[0][:8]


def test_float_to_half_all_floats(oracle):
    import torch

    chunk = 1 << 26
    for base in range(0, 1 << 32, chunk):
        bits = torch.arange(base, base + chunk, dtype=torch.int64, device="cuda").to(torch.int32)
        got = bits.view(torch.float32).half().view(torch.int16).cpu().numpy().view(np.uint16)
        f = np.arange(base, base + chunk, dtype=np.uint64).astype(np.uint32).view(np.float32)
        ref = oracle.f2h(f)
        nan = np.isnan(f)
        bad = (got != ref) & ~nan  # NaN: the kernels canonicalise after the hardware conversion
        assert not bad.any(), (hex(base), np.nonzero(bad)[0][:8])
        assert ((got[nan] & 0x7C00) == 0x7C00).all() and ((got[nan] & 0x3FF) != 0).all()
