#!/usr/bin/env python3
"""Denoise + post under a profiler: serial frames of the bench workload (1080p 4 spp, default or
terrain view) with each stage synchronised, then the gating statistics of the frame's wide and
local spatial filters (16x16 tiles whose noise level passes noise_threshold_large / _local) and the
fraction of surface (non-sky) pixels.  Run it as
  rocprofv3 --kernel-trace --stats -- python3 tools/denoise_probe.py [frames] [view]
(RTX_LIB selects an ablation build).  Prints one JSON line."""
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]


def main():
    import rtx

    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    view = sys.argv[2] if len(sys.argv) > 2 else "default"
    W, H = 1920, 1080
    rt = rtx.RayTracer(W, H, rtx.write_config(os.path.join(tempfile.mkdtemp(), "d.toml"), W, H, spp=4)).init()
    rt.set_delta_time(16.667)
    if os.environ.get("DN_PASS"):  # e.g. DN_PASS=enableSharpening=0,enableToneMapping=0
        pr = rt.params
        for kv in os.environ["DN_PASS"].split(","):
            k, v = kv.split("=")
            setattr(pr.pass_, k, int(v))
        rt.params = pr
    if view == "terrain":
        c = rt.camera
        c.pos[:] = (8.0, 15.0, -6.0)
        c.yaw, c.pitch = 0.0, -0.7
        rt.camera = c
    for f in range(1, frames + 1):
        rt.build_bvh()
        rt.path_trace(f)
        rt.sync()
        rt.denoise_post(f)
        rt.sync()
    p = rt.params.denoise
    W16, H16 = (W + 15) // 16, (H + 15) // 16
    n16 = rt.get_buffer("NOISE_LEVEL16", (H16, W16), np.float16).astype(np.float32)
    depth = rt.get_buffer("DEPTH", (H, W), np.float16).astype(np.float32)
    out = dict(view=view, frames=frames, tiles=int(n16.size),
               wide_active_tiles=round(float((~(n16 < p.noise_threshold_large)).mean()), 4),
               local_active_tiles=round(float((~(n16 < p.noise_threshold_local)).mean()), 4),
               surface_px=round(float((depth < 10e9).mean()), 4),
               denoise_post_ms=round(rt.time_stage(4, 20) / 20, 4),
               path_trace_ms=round(rt.time_stage(2, 20) / 20, 4))
    print(json.dumps(out), flush=True)
    rt.cleanup()


if __name__ == "__main__":
    main()
