#!/usr/bin/env python3
"""ms/frame of rt_draw_device (sync / async) and of the bench's FramePipeline, each in its own
context, in the order given (e.g. `async pipe async`): shows whether a later context in the same
process runs slower.  Usage: tools/draw_probe.py MODE [MODE ...]  (MODE: sync | async | pipe)"""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]

import torch  # noqa: E402

import rtx  # noqa: E402
from rtx.frames import FramePipeline  # noqa: E402

W, H, S, N = 1920, 1080, 4, 30


def run(mode, tmp, dev):
    rt = rtx.RayTracer(W, H, rtx.write_config(os.path.join(tmp, mode + ".toml"), W, H, dynamic=False, spp=S)).init()
    rt.set_delta_time(16.667)
    target = torch.empty((H, W, 4), dtype=torch.uint8, device=dev)
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
    for f in range(4, 4 + N):
        step(f)
    rt.sync()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / N
    rt.cleanup()
    if fp:
        torch.cuda.set_stream(torch.cuda.default_stream(dev))
    return ms


def main():
    dev = torch.device("cuda", 0)
    tmp = tempfile.mkdtemp()
    for i, mode in enumerate(sys.argv[1:] or ["async"]):
        print("%d %s %.4f ms/frame" % (i, mode, run(mode, tmp, dev)), flush=True)


if __name__ == "__main__":
    main()
