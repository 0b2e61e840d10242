#!/usr/bin/env python3
"""Host-side cost of the bench loop: wall time of FramePipeline.frame() calls (enqueue only)
against the synchronised frame time.  If enqueueing takes as long as the GPU work, the host, not
the GPU, sets the frame rate.  Tuning aid."""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]


def main():
    import torch

    import rtx
    from rtx.frames import FramePipeline

    W, H = 1920, 1080
    cfg = rtx.write_config(os.path.join(tempfile.mkdtemp(), "h.toml"), W, H, spp=4)
    rt = rtx.RayTracer(W, H, cfg).init()
    rt.set_delta_time(16.667)
    fp = FramePipeline(rt, torch.device("cuda", 0))
    for f in range(1, 6):
        fp.frame(f)
    fp.finish()
    torch.cuda.synchronize()
    for n in (30, 120):
        t0 = time.perf_counter()
        enq = 0.0
        for f in range(6, 6 + n):
            a = time.perf_counter()
            fp.frame(f)
            enq += time.perf_counter() - a
        t1 = time.perf_counter()
        fp.finish()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print("frames %d: enqueue %.4f ms/frame (loop %.4f), total %.4f ms/frame" % (n, enq * 1e3 / n, (t1 - t0) * 1e3 / n, (t2 - t0) * 1e3 / n), flush=True)
    rt.cleanup()


if __name__ == "__main__":
    main()
