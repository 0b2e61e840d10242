#!/usr/bin/env python3
"""The workload of BASELINE configs 2 and 4 alone, for rocprofv3 (--kernel-trace --stats and one
--pmc pass per run, tools/prof_r04_c2c4.sh):

  config 2  1920x1080, 1 spp primary rays, default scene and camera: rt_time_stage(1, N) = N
            back-to-back k_trace_primary launches (frames 1..N) between HIP events;
  config 4  the 958,720-triangle scene (chunkDim 4): rt_time_stage(0, N) = N k_build_bvh launches.

Prints one JSON line with the event times, so that the rocprof average of each kernel can be set
beside the events of the same run.  The default scene's own init-time build (60,800 triangles, 60
workgroups) is told apart from config 4's (937 workgroups) by its grid size."""
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]


def main():
    import torch  # noqa: F401  (one HIP runtime: torch's)
    import rtx
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    tmp = tempfile.mkdtemp()
    W, H = 1920, 1080
    rt = rtx.RayTracer(W, H, rtx.write_config(os.path.join(tmp, "c2.toml"), W, H, dynamic=False)).init()
    rt.build_bvh()
    rt.sync()
    out = {"c2_primary_ms": round(rt.time_stage(1, n) / n, 5), "c2_launches": n, "c2_rays": W * H}
    rt.cleanup()
    r4 = rtx.RayTracer(256, 144, rtx.write_config(os.path.join(tmp, "c4.toml"), 256, 144, chunk_dim=4)).init()
    r4.build_bvh()
    r4.sync()
    out.update(c4_build_ms=round(r4.time_stage(0, n) / n, 5), c4_launches=n, c4_tris=int(r4.info().triCount))
    r4.cleanup()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
