"""More pins to data the reference itself holds (VERDICT r3 "what's missing" 1):

* the denoiser's precomputed Gaussian tables, gaussian.cuh:12-43: tests/golden/ref_gaussian.json
  holds each literal as written and its float32 bits (tests/golden/make_ref_fixtures.py reads them
  from the header's text); the product's tables (rt_filter_kernel: the same list the device
  __constant__ tables are built from, csrc/gaussian_tables.h) and the oracle's (oracle/denoise.cpp,
  its own literals) must equal them bit for bit;
* the data files tools/extract_reference_data.py extracted once from the reference tree
  (real-time-ray-tracing_amd/data: the blue-noise tables of blueNoiseRandGenData.h, the round-cube
  tiles of resources/models/roundcubes/2, the sky tables of skyData.h): where /root/reference is
  present the extraction is re-run and must reproduce data/MANIFEST.json and every shipped byte;
* the reference's only test, test/scan/main.cu:5-68, has its CPU side here (CpuScan,
  scan.cuh:235-251) checked against the oracle's Blelloch restatement with the test's own rule
  (ArrayAlmostEqual 5 %, testCommon.h:37-59); tests/test_gpu_scan.py applies it to the GPU kernels.
"""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
ROOT = os.path.dirname(HERE)
DATA = os.path.join(ROOT, "real-time-ray-tracing_amd", "data")
REF = "/root/reference"


def gaussian_fixture():
    raw = open(os.path.join(GOLD, "ref_gaussian.json"), "rb").read()
    man = json.load(open(os.path.join(GOLD, "ref_fixtures.json")))
    assert hashlib.sha256(raw).hexdigest() == man["ref_gaussian.json"]["sha256"]
    return json.loads(raw)


def array_almost_equal(a, b, pct):
    """ArrayAlmostEqual (test/testCommon.h:37-59): larger / smaller - 1 <= pct / 100 at every index."""
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    c, d = np.maximum(a, b), np.minimum(a, b)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = c / d - np.float32(1.0)
    return not bool((r > np.float32(pct / 100.0)).any())


@pytest.mark.parametrize("n", [3, 5, 7])
def test_gaussian_tables_product_and_oracle_match_reference(rtx, oracle, n):
    want = np.array(gaussian_fixture()["%dx%d" % (n, n)]["float32_bits"], np.uint32)
    got = np.zeros(n * n, np.float32)
    lib = rtx.load_library()
    assert lib.rt_filter_kernel(n, got.ctypes.data, n * n) == 0
    assert np.array_equal(got.view(np.uint32), want)
    assert np.array_equal(oracle.filter_kernel(n).view(np.uint32), want)
    assert lib.rt_filter_kernel(4, got.ctypes.data, 16) == -1 and lib.rt_filter_kernel(7, got.ctypes.data, 48) == -1


def test_gaussian_tables_are_the_slightly_asymmetric_ones():
    """The precomputed tables are not symmetric: e.g. 3x3 [2] 0.0584323 vs [6] 0.0584322."""
    g = gaussian_fixture()
    t3 = g["3x3"]["literals"]
    assert t3[2] == "0.0584323" and t3[6] == "0.0584322"
    # the 5x5's centre 3x3 block is the 3x3 table, and the 7x7's centre 5x5 block the 5x5 table
    t5 = np.array(g["5x5"]["float32_bits"]).reshape(5, 5)
    t7 = np.array(g["7x7"]["float32_bits"]).reshape(7, 7)
    assert np.array_equal(t5[1:4, 1:4].ravel(), g["3x3"]["float32_bits"])
    assert np.array_equal(t7[1:6, 1:6][:4, :4], t5[:4, :4])


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "src", "gaussian.cuh")),
                    reason="reference tree not present (GPU box)")
def test_reference_gaussian_reproduces_fixture():
    sys.path.insert(0, GOLD)
    import make_ref_fixtures as M
    assert M.gaussian_tables(open(os.path.join(REF, "src", "gaussian.cuh")).read()) == gaussian_fixture()


def test_shipped_data_matches_manifest():
    man = json.load(open(os.path.join(DATA, "MANIFEST.json")))
    for name, e in man.items():
        assert hashlib.sha256(open(os.path.join(DATA, name), "rb").read()).hexdigest() == e["sha256"], name


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "src", "blueNoiseRandGenData.h")),
                    reason="reference tree not present (GPU box)")
def test_reference_extraction_reproduces_shipped_data(tmp_path):
    """Re-run tools/extract_reference_data.py against /root/reference into a scratch directory: the
    manifest equals data/MANIFEST.json and every file equals the shipped one byte for byte."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import extract_reference_data as X
    man = X.extract(str(tmp_path))
    assert json.loads(json.dumps(man)) == json.load(open(os.path.join(DATA, "MANIFEST.json")))
    for name in man:
        assert open(str(tmp_path / name), "rb").read() == open(os.path.join(DATA, name), "rb").read(), name


@pytest.mark.parametrize("postfix", [1, 0])
def test_reference_scan_rule_on_oracle(oracle, postfix):
    """test/scan/main.cu:12-55 on the oracle: 262,144 floats of rand()/RAND_MAX, Scan with blockSize 128
    (2,048 blocks) against CpuScan, ArrayAlmostEqual at 5 % (seeded here; the reference seeds with time(0))."""
    x = (np.random.default_rng(2024).integers(0, 2**31 - 1, 128 * 2048) / np.float32(2**31 - 1)).astype(np.float32)
    blel = oracle.scan(x, 128, postfix)
    seq = oracle.cpu_scan(x, postfix)
    if not postfix:  # the exclusive scans' first element is 0 in both: compare from index 1
        assert blel[0] == 0 and seq[0] == 0
        blel, seq = blel[1:], seq[1:]
    assert array_almost_equal(seq, blel, 5)
    # the rule is loose: the two orders differ only by float rounding (sequential error grows ~n eps)
    assert float(np.max(np.abs(blel / seq - 1))) < 1e-3
