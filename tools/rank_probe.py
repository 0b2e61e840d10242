#!/usr/bin/env python3
"""One rank's share of the N-GPU frame on a single GPU: the interleaved strip of rank 0 of N
(stripCount = N), pipelined exactly as bench.py runs it, without the G-buffer all-gather itself.
The rows other ranks would deliver are filled once with a full-frame render (the denoiser's cost
depends on them: sky pixels skip the filters), so the denoise sees the frame it would see after
the gather.  STRIP_DN=1: each rank denoises only its strip (+ halo), with the collective hook a
no-op (compute only: the exchanges are left out).  Prints ms per frame for each N, one fresh process
per N.  Usage: [W=3840 H=2160] [QUICK=1] [STRIP_DN=1] [STAGES=1] [FRAMES=30] tools/rank_probe.py [N ...]
(default 1 2 4 8; QUICK: the pipelined frame with denoise only; STAGES: serial stage split too)."""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtx  # noqa: E402
from rtx.dist import GBUFFERS, StripGather, strip_config  # noqa: E402

_FULL = {}


def full_frame(W, H, spp):
    """G-buffers of frame 1 rendered by one full-frame context (host bytes per buffer)."""
    key = (W, H, spp)
    if key not in _FULL:
        d = tempfile.mkdtemp()
        rt = rtx.RayTracer(W, H, rtx.write_config(os.path.join(d, "c.toml"), W, H, spp=spp)).init()
        rt.build_bvh()
        rt.path_trace(1)
        rt.sync()
        _FULL[key] = {name: rt.get_buffer(name, (W * H * bpp,), np.uint8) for name, bpp in GBUFFERS}
        rt.cleanup()
    return _FULL[key]


def run(n, frames=int(os.environ.get("FRAMES", "30")), warm=3, W=int(os.environ.get("W", "1920")),
        H=int(os.environ.get("H", "1080")), spp=4, pipeline=True, denoise=True):
    d = tempfile.mkdtemp()
    rt = rtx.RayTracer(W, H, rtx.write_config(os.path.join(d, "c.toml"), W, H, spp=spp,
                                              extra=strip_config(n, 0))).init()
    rt.set_delta_time(16.667)
    lo, hi = torch.cuda.Stream.priority_range()
    main, post = torch.cuda.Stream(priority=hi), torch.cuda.Stream(priority=lo)
    torch.cuda.set_stream(main)
    rt.set_stream(main.cuda_stream)
    if pipeline:
        rt.set_post_stream(post.cuda_stream)
    if n > 1 and os.environ.get("STRIP_DN"):  # strip-local denoise, exchanges left out (no-op hook)
        rt.set_collective_hook(lambda stage, stream, x: None)
    if n > 1:  # bound full-frame G-buffers holding the other ranks' rows, as after the gather
        sg = StripGather(W, H, n, 0, torch.device("cuda", 0), rt, sets=rtx.GBUFFER_SETS if pipeline else 1)
        full = full_frame(W, H, spp)
        for tensors in sg.sets:
            for name, _ in GBUFFERS:
                tensors[name][:full[name].size].copy_(torch.from_numpy(full[name]))
        torch.cuda.synchronize()
    for f in range(1, warm + 1):
        rt.build_bvh()
        rt.path_trace(f)
        rt.denoise_post(f)
    rt.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for f in range(warm + 1, warm + frames + 1):
        rt.build_bvh()
        rt.path_trace(f)
        if denoise:
            rt.denoise_post(f)
    rt.sync()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / frames
    if os.environ.get("STAGES"):  # serial stage times of this rank's share (primary rays, path trace, denoise)
        st = [rt.time_stage(k, 20) / 20 for k in (1, 2, 4)]
        print("  N=%d stages serial: primary rays %.3f  path trace %.3f  denoise %.3f ms" % (n, *st), flush=True)
    rt.cleanup()
    return ms


if __name__ == "__main__":
    ns = [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]
    if len(ns) > 1:  # one fresh process per N: a second context in one process can land in a slower schedule
        import subprocess
        for n in ns:
            rc = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), str(n)], timeout=300).returncode
            if rc:
                sys.exit(rc)
        sys.exit(0)
    for n in ns:
        variants = ((True, True), (False, True), (True, False), (False, False))
        for pipe, dn in variants[:1] if os.environ.get("QUICK") else variants:
            print("N=%d rank-0 strip (%sx%s), %s, %s: %.3f ms/frame" % (n, os.environ.get("W", "1920"),
                                                                       os.environ.get("H", "1080"),
                                                                       "pipelined" if pipe else "serial",
                                                              "with denoise" if dn else "no denoise",
                                                              run(n, pipeline=pipe, denoise=dn)), flush=True)
