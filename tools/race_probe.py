#!/usr/bin/env python3
"""Repeat pipelined renders and compare every frame's RGBA8 with a serial render (race probe).
Usage: tools/race_probe.py [reps] [frames] [mode: pipe|pipe-sync]"""
import hashlib
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]
import torch  # noqa: E402
import rtx  # noqa: E402

W, H = 256, 144


def render(pipelined, frames, per_frame_sync):
    d = tempfile.mkdtemp()
    rt = rtx.RayTracer(W, H, rtx.write_config(os.path.join(d, "c.toml"), W, H, spp=2)).init()
    rt.set_delta_time(16.667)
    rt.set_stream(torch.cuda.current_stream().cuda_stream)
    if pipelined:
        post = torch.cuda.Stream()
        rt.set_post_stream(post.cuda_stream)
    cam0 = rt.camera
    out = []
    for f in range(1, frames + 1):
        c = rt.camera
        c.yaw = cam0.yaw + 0.02 * f
        rt.camera = c
        rt.build_bvh()
        rt.path_trace(f)
        if per_frame_sync:
            rt.sync()
        rt.denoise_post(f)
        out.append(hashlib.sha1(rt.download("RGBA8", np.uint8).tobytes()).hexdigest()[:12] if per_frame_sync else None)
    final = hashlib.sha1(rt.download("RGBA8", np.uint8).tobytes() + rt.get_buffer("RENDER_COLOR").tobytes()).hexdigest()[:12]
    rt.cleanup()
    return out, final


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    torch.cuda.set_device(0)
    ref_frames, ref = render(False, frames, True)
    print("serial", ref)
    bad = 0
    for r in range(reps):
        for mode in ("pipe", "pipe-sync"):
            fr, fin = render(True, frames, mode == "pipe-sync")
            ok = fin == ref and (mode == "pipe" or fr == ref_frames)
            bad += not ok
            print(r, mode, fin, "ok" if ok else "MISMATCH", "" if ok or mode == "pipe" else
                  [i + 1 for i, (a, b) in enumerate(zip(fr, ref_frames)) if a != b])
    print("mismatches", bad)


if __name__ == "__main__":
    main()
