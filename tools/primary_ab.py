#!/usr/bin/env python3
"""Primary-ray stage (rt_trace_primary, 1080p, 1 spp, default view) of one librtx build (RTX_LIB
selects it): ms over 5 x 20 serial stages, as bench.py's primary_rays_1spp.  Ablation aid."""
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]


def main():
    import rtx

    W, H = 1920, 1080
    sr = rtx.RayTracer(W, H, rtx.write_config(os.path.join(tempfile.mkdtemp(), "s.toml"), W, H,
                                              dynamic=False, spp=4)).init()
    for f in range(1, 4):
        sr.build_bvh()
        sr.path_trace(f)
    sr.sync()
    ms = sorted(sr.time_stage(1, 20) / 20 for _ in range(5))
    print(json.dumps({"lib": os.environ.get("RTX_LIB", "in-tree"), "ms": ms,
                      "mray_s_best": round(W * H / (ms[0] * 1e-3) / 1e6, 1)}))
    sr.cleanup()


if __name__ == "__main__":
    main()
