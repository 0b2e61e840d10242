#!/usr/bin/env python3
"""Serial per-kernel and per-stage times of the bench workload (1080p 4 spp, default view) for one
library: rt_time_path_trace_kernels and rt_time_stage (build 0, path trace 2, full serial frame 3, denoise+post 4).
Usage: python tools/stage_probe.py [lib.so]  -> one JSON line."""
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]
import rtx  # noqa: E402


def main():
    if len(sys.argv) > 1:
        rtx.load_library(sys.argv[1])
    W, H = 1920, 1080
    rt = rtx.RayTracer(W, H, rtx.write_config(os.path.join(tempfile.mkdtemp(), "s.toml"), W, H, spp=4)).init()
    rt.set_delta_time(16.667)
    for f in range(1, 4):
        rt.build_bvh()
        rt.path_trace(f)
        rt.denoise_post(f)
    rt.sync()
    k = rt.time_path_trace_kernels(20)
    out = {"kernels_ms": {a: round(b, 4) for a, b in k.items() if b > 0},
           "build_ms": round(rt.time_stage(0, 20) / 20, 4), "path_trace_ms": round(rt.time_stage(2, 20) / 20, 4),
           "denoise_post_ms": round(rt.time_stage(4, 20) / 20, 4), "frame_ms": round(rt.time_stage(3, 20) / 20, 4)}
    print(json.dumps(out))
    rt.cleanup()


if __name__ == "__main__":
    main()
