"""bench.py's CPU-baseline legs on a small size (no GPU): BASELINE config 1's host frame and the
thread-count rule the JSON reports."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_c1_frame_small(oracle):
    r = bench.c1_frame(oracle, threads=2, size=64)
    assert r["size"] == [64, 64] and r["spp"] == 1
    assert r["rays"] >= 64 * 64  # every pixel traces its camera ray
    for k in ("lbvh_build_ms", "path_trace_ms", "denoise_post_ms", "hdr_dump_ms"):
        assert r[k] > 0.0
    assert abs(r["frame_ms"] - (r["lbvh_build_ms"] + r["path_trace_ms"] + r["denoise_post_ms"] + r["hdr_dump_ms"])) < 1.0


def test_host_threads_respects_cap(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert 1 <= bench.host_threads() <= 3
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.host_threads() >= 1
