#!/usr/bin/env python3
"""Pipelined ms/frame of the bench's two views (default and terrain camera), 1080p 4 spp, timed the
way bench.py times its frames (no per-kernel marks).  For A/B runs of environment switches or
ablation builds (RTX_LIB): prints one JSON line.  Usage: python3 tools/view_ab.py [frames] [tag]"""
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
    from rtx.frames import FramePipeline

    nt = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    tag = sys.argv[2] if len(sys.argv) > 2 else ""
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    W, H, S = 1920, 1080, 4
    out = {"tag": tag}
    for view in ("default", "terrain"):
        cfg = rtx.write_config(os.path.join(tempfile.mkdtemp(), "v.toml"), W, H, dynamic=False, chunk_dim=1, spp=S)
        rt = rtx.RayTracer(W, H, cfg).init()
        rt.set_delta_time(16.667)
        if view == "terrain":
            cam = rt.camera
            cam.pos[:] = TERRAIN["pos"]
            cam.yaw, cam.pitch = TERRAIN["yaw"], TERRAIN["pitch"]
            rt.camera = cam
        fp = FramePipeline(rt, dev, pipelined=True)
        for f in range(1, 4):
            fp.frame(f)
        fp.finish()
        res = []
        for rep in range(2):
            torch.cuda.synchronize()
            ta = time.perf_counter()
            for k in range(nt):
                fp.frame(4 + rep * nt + k)
            fp.finish()
            torch.cuda.synchronize()
            res.append(round((time.perf_counter() - ta) * 1e3 / nt, 4))
        out[view] = res
        rt.cleanup()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
