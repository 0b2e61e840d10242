#!/usr/bin/env python3
"""Probe: k_pathtrace time at 1080p 4 spp under three cameras (default view ~8% terrain,
looking down = all terrain, looking up = all sky), plus the frame's stage times.
Usage: python tools/pt_probe.py [--iters N]"""
import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-ray-tracing_amd"))
import numpy as np  # noqa: E402
import rtx  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--lib", default=None, help="alternative librtx.so (ablation builds)")
    ap.add_argument("--torch-stream", action="store_true", help="run on torch's current stream, as bench.py does")
    ap.add_argument("--only-default", action="store_true")
    a = ap.parse_args()
    if a.lib:
        rtx.load_library(a.lib)
    d = tempfile.mkdtemp()
    rt = rtx.RayTracer(a.width, a.height, rtx.write_config(os.path.join(d, "p.toml"), a.width, a.height, spp=4)).init()
    rt.set_delta_time(16.667)
    if a.torch_stream:
        import torch
        torch.cuda.set_device(0)
        rt.set_stream(torch.cuda.current_stream().cuda_stream)
    rt.build_bvh()
    out = {}
    base = rt.camera
    cams = (("default", None),) if a.only_default else (("default", None), ("down", -1.2), ("up", 0.9))
    for name, pitch in cams:
        c = rtx.Camera.from_buffer_copy(base)
        if pitch is not None:
            c.pos[1] = 12.0 if name == "down" else base.pos[1]
            c.pitch = pitch
        rt.camera = c
        rt.path_trace(1, detail=True)
        st = rt.download("PT_STATS", np.uint32).reshape(-1, 4).astype(np.uint64)
        qc = rt.download("PT_QUEUE", np.uint32)
        out[name + "_queues"] = {"q3": int(qc[0]), "q4": int(qc[1]), "pending": int(qc[4]),
                                 "max_iter3": int(qc[8]), "max_iter4": int(qc[9])}
        rt.time_stage(2, 3)
        ms = rt.time_stage(2, a.iters) / a.iters
        H8, W8 = a.height // 8, a.width // 8
        vis = st[:, 1].reshape(a.height, a.width)[:H8 * 8, :W8 * 8].reshape(H8, 8, W8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
        out[name + "_tiles"] = {"mean_visits_px": round(float(vis.mean()), 2),
                                "mean_tile_max_visits_px": round(float(vis.max(1).mean()), 2),
                                "p99_px": float(np.percentile(vis, 99)), "max_px": int(vis.max())}
        out[name] = {"ms": round(ms, 4), "rays": int(st[:, 0].sum()), "visits": int(st[:, 1].sum()),
                     "tests": int(st[:, 2].sum()), "diffuse": int(st[:, 3].sum())}
    rt.camera = base
    out["stage_ms"] = {"build": rt.time_stage(0, 20) / 20, "denoise_post": rt.time_stage(4, 20) / 20}
    out["lib"] = a.lib or "librtx.so"
    print(json.dumps(out))
    rt.cleanup()


if __name__ == "__main__":
    main()
