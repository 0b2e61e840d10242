"""The reference's only test, test/scan/main.cu:5-68, applied to the product's scan kernels (sky.hip
k_scan_block / k_scan_add behind rt_scan_device, the drop-in for Scan, scan.cuh:258-298):
262,144 floats of rand()/RAND_MAX scanned with blockSize 128 (2,048 blocks, their totals scanned in
one workgroup), postfix 1, against CpuScan (scan.cuh:235-251) with ArrayAlmostEqual at 5 %
(testCommon.h:37-59).  Beyond the reference's rule the GPU result must equal the oracle's Blelloch
restatement (oracle/sky.cpp scan_blocks) bit for bit at every size, as the sky/sun CDFs do."""
import numpy as np
import pytest

from test_ref_data_pins import array_almost_equal

pytestmark = pytest.mark.gpu


def rand_array(n, seed):
    """RandomArray (testCommon.h:12-22): rand() / (float)RAND_MAX, seeded here (the reference uses time(0))."""
    r = np.random.default_rng(seed).integers(0, 2**31 - 1, n)
    return (r.astype(np.float32) / np.float32(2**31 - 1)).astype(np.float32)


def gpu_scan(rtx, x, block, postfix):
    import torch
    dev = torch.device("cuda", 0)
    t_in = torch.from_numpy(x).to(dev)
    t_out = torch.empty_like(t_in)
    t_tmp = torch.zeros(max(1, x.size // block), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    lib = rtx.load_library()
    rc = lib.rt_scan_device(t_in.data_ptr(), t_out.data_ptr(), t_tmp.data_ptr(), x.size, block, postfix, None)
    torch.cuda.synchronize()
    return rc, t_out.cpu().numpy()


@pytest.mark.parametrize("postfix", [1, 0])
def test_reference_scan_test(rtx, oracle, postfix):
    x = rand_array(128 * 2048, 7)
    rc, y = gpu_scan(rtx, x, 128, postfix)
    assert rc == 0
    seq = oracle.cpu_scan(x, postfix)
    a, b = (seq, y) if postfix else (seq[1:], y[1:])
    assert array_almost_equal(a, b, 5)  # the reference test's acceptance rule
    assert np.array_equal(y.view(np.uint32), oracle.scan(x, 128, postfix).view(np.uint32))


@pytest.mark.parametrize("size,block", [(131072, 256), (1024, 32), (8192, 8192), (2 * 8192, 8192), (8192 * 8, 8),
                                        (4096, 2), (64, 64), (2048 * 4096, 4096)])
def test_scan_sizes_bit_exact(rtx, oracle, size, block):
    x = rand_array(size, size + block)
    for postfix in (1, 0):
        rc, y = gpu_scan(rtx, x, block, postfix)
        assert rc == 0
        assert np.array_equal(y.view(np.uint32), oracle.scan(x, block, postfix).view(np.uint32)), (size, block, postfix)


def test_scan_rejects_what_the_reference_asserts(rtx):
    x = rand_array(3 * 128, 1)
    for size, block in ((3 * 128, 128), (1024, 48), (1024, 16384), (16384 * 2, 2)):
        rc, _ = gpu_scan(rtx, np.resize(x, size), block, 1)
        assert rc == -1, (size, block)
