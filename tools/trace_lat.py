#!/usr/bin/env python3
"""Latency anatomy of the queue tracer: trace the default frame's step-3 bounce rays through
rt_trace_rays in subsets (all, without the longest, the longest alone, copies of it, the k
longest) and report kernel ms and ms per TraverseBvh iteration of the longest ray."""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]
import rtx  # noqa: E402


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else None
    if lib:
        rtx.load_library(lib)
    w, h = 1920, 1080
    d = tempfile.mkdtemp()
    rt = rtx.RayTracer(w, h, rtx.write_config(os.path.join(d, "c.toml"), w, h, spp=4)).init()
    rt.set_delta_time(16.667)
    rt.build_bvh()
    rt.path_trace(1)
    rt.sync()
    cnt = rt.download("PT_QUEUE", np.uint32)
    res = {}
    for q, key in ((3, 0), (4, 1)):
        n = int(cnt[key])
        o = rt.download("PT_Q%d_ORIGINS" % q, np.float32).reshape(-1, 4)[:n, :3].copy()
        dd = rt.download("PT_Q%d_DIRS" % q, np.float32).reshape(-1, 4)[:n, :3].copy()
        res[q] = (o, dd)
    for q in (3, 4):
        o, dd = res[q]
        n = len(o)
        *_, iters, ms = rt.trace_rays(o, dd, want_iters=True)
        for _ in range(3):
            *_, ms = rt.trace_rays(o, dd)
        order = np.argsort(iters)[::-1]
        L = order[0]
        print("queue %d: n=%d  all %.1f us  max iters %d  mean %.1f  p99 %d  p999 %d" % (
            q, n, ms * 1e3, iters[L], iters.mean(), np.percentile(iters, 99), np.percentile(iters, 99.9)))

        def run(sel, label):
            best = 1e9
            for _ in range(5):
                *_, m = rt.trace_rays(o[sel], dd[sel])
                best = min(best, m)
            it = iters[sel].max()
            print("  %-28s rays %7d  max iters %4d  %8.1f us  %.3f us/iter" % (label, len(sel), it, best * 1e3,
                                                                          best * 1e3 / max(1, it)))
        run(order[:1], "longest alone")
        run(np.repeat(order[:1], 64), "longest x64 (one wave)")
        run(order[:64], "64 longest (one wave)")
        run(order[:4096], "4096 longest")
        run(order[n // 100:], "all but the longest 1%")
        run(order[n // 10:], "all but the longest 10%")
        mid = order[len(order) // 2]
        run(np.array([mid]), "median ray alone")
    rt.cleanup()


if __name__ == "__main__":
    main()
