#!/usr/bin/env python3
"""Per-kernel path-trace times (HIP events) of the default 1080p 4-spp frame for several
librtx builds.  Usage: [PITCH=p] tools/kprobe.py [lib.so ...]  (no argument: the in-tree build;
PITCH overrides the camera pitch, e.g. -1.2 looks down at the terrain, 0.9 up at the sky)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys, tempfile, json
sys.path[:0] = [%r, %r]
import rtx
lib = %r
if lib:
    rtx.load_library(lib)
d = tempfile.mkdtemp()
rt = rtx.RayTracer(1920, 1080, rtx.write_config(os.path.join(d, "c.toml"), 1920, 1080, spp=4)).init()
rt.set_delta_time(16.667)
pitch = os.environ.get("PITCH")
if pitch:
    c = rt.camera
    c.pitch = float(pitch)
    rt.camera = c
rt.build_bvh()
rt.path_trace(1)
ks = rt.time_path_trace_kernels(20)
tot = rt.time_stage(2, 20) / 20
fr = rt.time_stage(3, 20) / 20
print(json.dumps(dict(kernels={k: round(v * 1e3, 1) for k, v in ks.items()}, stage_us=round(tot * 1e3, 1),
                      frame_us=round(fr * 1e3, 1))))
rt.cleanup()
'''

for lib in (sys.argv[1:] or [""]):
    code = CHILD % (ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd"), lib)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    print(lib or "in-tree", out.stdout.strip() or out.stderr[-2000:])
