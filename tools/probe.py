#!/usr/bin/env python3
"""Measurement probes of the bench workload (1920x1080, 4 spp unless given), one JSON line each.
RTX_LIB selects a library build (tools/abl_build.sh); run under rocprofv3 for kernel stats / PMC
passes (tools/prof.sh).  DESIGN.md §4-§9 cite the subcommands.

  probe.py frames  [--view default|terrain] [--n 30] [--reps 2] [--split]   pipelined ms/frame
                   (FramePipeline, as bench.py runs it); --split adds every kernel's HIP-event ms in
                   20 pipelined frames and the serial denoise + post
  probe.py serial  [--view ...] [--n 10]                                      serial frames, each
                   stage synchronised (per-kernel profiles without overlap)
  probe.py stages  [--view ...]                                               serial per-kernel and
                   per-stage times (rt_time_path_trace_kernels, rt_time_stage 0 / 2 / 3 / 4; RTX_TUNING=chain=off
                   for the four bounce kernels instead of the fused chain)
  probe.py denoise [--view ...] [--n 20]                                      serial frames, then the
                   noise gating (active tiles) and the serial denoise + post ms
  probe.py draw    [--modes sync,async,pipe] [--view ...] [--n 30]           rt_draw_device ms/frame
  probe.py primary [--n 20]                                                   config 2 (1 spp primary
                   rays), best of 5 x n launches
  probe.py lbvh    [--n 30]                                                   LBVH build of the
                   60,800- and 958,720-triangle scenes, best of 5 x n builds
  probe.py c2c4    [--n 20]                                                   configs 2 and 4 for the
                   PMC passes (one timed stage each)
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]

VIEWS = {"default": None, "terrain": dict(pos=(8.0, 15.0, -6.0), yaw=0.0, pitch=-0.7)}
DELTA_MS = 16.667


def renderer(W, H, S, view="default", **kw):
    import rtx

    rt = rtx.RayTracer(W, H, rtx.write_config(os.path.join(tempfile.mkdtemp(), "p.toml"), W, H, dynamic=False,
                                              spp=S, **kw)).init()
    rt.set_delta_time(DELTA_MS)
    v = VIEWS[view]
    if v:
        cam = rt.camera
        cam.pos[:] = v["pos"]
        cam.yaw, cam.pitch = v["yaw"], v["pitch"]
        rt.camera = cam
    return rt


def serial_frames(rt, first, n):
    for f in range(first, first + n):
        rt.build_bvh()
        rt.sync()
        rt.path_trace(f)
        rt.sync()
        rt.denoise_post(f)
        rt.sync()


def cmd_frames(a):
    import torch

    from rtx.frames import FramePipeline

    dev = torch.device("cuda", 0)
    rt = renderer(a.width, a.height, a.spp, a.view)
    fp = FramePipeline(rt, dev, pipelined=True)
    for f in range(1, 4):
        fp.frame(f)
    fp.finish()
    res, nxt = [], 4
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.n):
            fp.frame(nxt + k)
        fp.finish()
        torch.cuda.synchronize()
        res.append(round((time.perf_counter() - t0) * 1e3 / a.n, 4))
        nxt += a.n
    out = {"view": a.view, "ms_frame": res, "lib": os.environ.get("RTX_LIB", "in-tree")}
    if a.split:
        out["kernels_ms"] = {k: round(v, 4) for k, v in rt.time_frame_kernels(nxt + 1, 20).items()}
        out["denoise_serial_ms"] = round(rt.time_stage(4, 20) / 20, 4)
    rt.cleanup()
    return out


def cmd_serial(a):
    rt = renderer(a.width, a.height, a.spp, a.view)
    serial_frames(rt, 1, a.n)
    rt.cleanup()
    return {"view": a.view, "frames": a.n}


def cmd_stages(a):
    rt = renderer(a.width, a.height, a.spp, a.view)
    for f in range(1, 4):
        rt.build_bvh()
        rt.path_trace(f)
        rt.denoise_post(f)
    rt.sync()
    k = rt.time_path_trace_kernels(20)
    out = {"kernels_ms": {x: round(y, 4) for x, y in k.items() if y > 0},
           "build_ms": round(rt.time_stage(0, 20) / 20, 4), "path_trace_ms": round(rt.time_stage(2, 20) / 20, 4),
           "denoise_post_ms": round(rt.time_stage(4, 20) / 20, 4), "frame_ms": round(rt.time_stage(3, 20) / 20, 4)}
    rt.cleanup()
    return out


def cmd_denoise(a):
    import numpy as np

    W, H = a.width, a.height
    rt = renderer(W, H, a.spp, a.view)
    serial_frames(rt, 1, a.n)
    p = rt.params.denoise
    W16, H16 = (W + 15) // 16, (H + 15) // 16
    n16 = rt.get_buffer("NOISE_LEVEL16", (H16, W16), np.float16).astype(np.float32)
    depth = rt.get_buffer("DEPTH", (H, W), np.float16).astype(np.float32)
    out = dict(view=a.view, frames=a.n, tiles=int(n16.size),
               wide_active_tiles=round(float((~(n16 < p.noise_threshold_large)).mean()), 4),
               local_active_tiles=round(float((~(n16 < p.noise_threshold_local)).mean()), 4),
               surface_px=round(float((depth < 10e9).mean()), 4),
               denoise_post_ms=round(rt.time_stage(4, 20) / 20, 4))
    rt.cleanup()
    return out


def cmd_draw(a):
    import torch

    from rtx.frames import FramePipeline

    dev = torch.device("cuda", 0)
    out = {"view": a.view}
    for mode in a.modes.split(","):
        rt = renderer(a.width, a.height, a.spp, a.view)
        target = torch.empty((a.height, a.width, 4), dtype=torch.uint8, device=dev)
        fp = FramePipeline(rt, dev) if mode == "pipe" else None

        def step(f):
            if fp:
                fp.frame(f)
            else:
                rt.draw_device(target.data_ptr(), 0, asynchronous=mode == "async")

        for f in range(1, 4):
            step(f)
        rt.sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for f in range(4, 4 + a.n):
            step(f)
        rt.sync()
        torch.cuda.synchronize()
        out[mode + "_ms_frame"] = round((time.perf_counter() - t0) * 1e3 / a.n, 4)
        rt.cleanup()
        if fp:
            torch.cuda.set_stream(torch.cuda.default_stream(dev))
    return out


def cmd_primary(a):
    import torch  # noqa: F401  (one HIP runtime: torch's)

    rt = renderer(a.width, a.height, a.spp)
    for f in range(1, 4):
        rt.build_bvh()
        rt.path_trace(f)
    rt.sync()
    ms = sorted(rt.time_stage(1, a.n) / a.n for _ in range(5))
    rt.cleanup()
    return {"ms": [round(m, 5) for m in ms], "mray_s_best": round(a.width * a.height / (ms[0] * 1e-3) / 1e6, 1)}


def cmd_lbvh(a):
    import torch  # noqa: F401

    out = {}
    for cd in (1, 4):
        rt = renderer(256, 144, 1, chunk_dim=cd)
        rt.build_bvh()
        rt.sync()
        best = min(rt.time_stage(0, a.n) / a.n for _ in range(5))
        out["%d_tris_ms" % rt.info().triCount] = round(best, 5)
        rt.cleanup()
    return out


def cmd_c2c4(a):
    import torch  # noqa: F401

    rt = renderer(1920, 1080, 1)
    rt.build_bvh()
    rt.sync()
    out = {"c2_primary_ms": round(rt.time_stage(1, a.n) / a.n, 5), "c2_launches": a.n, "c2_rays": 1920 * 1080}
    rt.cleanup()
    r4 = renderer(256, 144, 1, chunk_dim=4)
    r4.build_bvh()
    r4.sync()
    out.update(c4_build_ms=round(r4.time_stage(0, a.n) / a.n, 5), c4_launches=a.n, c4_tris=int(r4.info().triCount))
    r4.cleanup()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=("frames", "serial", "stages", "denoise", "draw", "primary", "lbvh", "c2c4"))
    ap.add_argument("--view", default="default", choices=tuple(VIEWS))
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--split", action="store_true")
    ap.add_argument("--modes", default="sync,async")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=4)
    a = ap.parse_args()
    if a.n is None:
        a.n = {"frames": 30, "serial": 10, "denoise": 20, "draw": 30, "primary": 20, "lbvh": 30, "c2c4": 20}.get(a.cmd, 20)
    out = globals()["cmd_" + a.cmd](a)
    out["probe"] = a.cmd
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
