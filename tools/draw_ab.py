#!/usr/bin/env python3
"""rt_draw_device ms/frame, synchronous and asynchronous, of the bench's two views (default and
terrain camera), 1080p 4 spp, timed as bench.py's time_draw does; for A/B runs of environment
switches or ablation builds (RTX_LIB).  Prints one JSON line.  Usage: python3 tools/draw_ab.py [frames] [tag]"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]

TERRAIN = dict(pos=(8.0, 15.0, -6.0), yaw=0.0, pitch=-0.7)


def main():
    import torch

    import rtx

    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    out = {"tag": sys.argv[2] if len(sys.argv) > 2 else ""}
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    W, H, S = 1920, 1080, 4
    target = torch.empty((H, W, 4), dtype=torch.uint8, device=dev)
    for view in ("default", "terrain"):
        for mode in ("sync", "async"):
            d = rtx.RayTracer(W, H, rtx.write_config(os.path.join(tempfile.mkdtemp(), "d.toml"), W, H,
                                                     dynamic=False, spp=S)).init()
            d.set_delta_time(16.667)
            if view == "terrain":
                cam = d.camera
                cam.pos[:] = TERRAIN["pos"]
                cam.yaw, cam.pitch = TERRAIN["yaw"], TERRAIN["pitch"]
                d.camera = cam
            asy = mode == "async"
            for _ in range(3):
                d.draw_device(target.data_ptr(), 0, asynchronous=asy)
            d.sync()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(frames):
                d.draw_device(target.data_ptr(), 0, asynchronous=asy)
            d.sync()
            torch.cuda.synchronize()
            out["%s_%s" % (view, mode)] = round((time.perf_counter() - t0) * 1e3 / frames, 4)
            d.cleanup()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
