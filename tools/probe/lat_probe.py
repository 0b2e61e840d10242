#!/usr/bin/env python3
"""Anatomy of a lone ray's TraverseBvh iteration (tools/probe/lat_probe.hip, the product's
trav_step on the product's record arena): per iteration the load wait left at its start and its
own work, in core clocks, by iteration kind, for the longest, the p99 and the median step-3 bounce
ray of the default 1080p frame.  The probe's hit must equal the queue tracer's (rt_trace_rays)."""
import ctypes as C
import os
import sys
import tempfile

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]
import rtx  # noqa: E402


def unwrap(c):
    """low 32 bits of s_memtime -> monotone counts"""
    c = c.astype(np.int64) & 0xFFFFFFFF
    d = np.diff(c) % (1 << 32)
    return np.concatenate([[0], np.cumsum(d)])


def main():
    w, h = 1920, 1080
    d = tempfile.mkdtemp()
    rt = rtx.RayTracer(w, h, rtx.write_config(os.path.join(d, "c.toml"), w, h, spp=4)).init()
    rt.set_delta_time(16.667)
    rt.build_bvh()
    rt.path_trace(1)
    rt.sync()
    n = int(rt.download("PT_QUEUE", np.uint32)[0])
    o = rt.download("PT_Q3_ORIGINS", np.float32).reshape(-1, 4)[:n, :3].copy()
    dd = rt.download("PT_Q3_DIRS", np.float32).reshape(-1, 4)[:n, :3].copy()
    t, tri, u, v, iters, _ = rt.trace_rays(o, dd, want_iters=True)
    dev = torch.device("cuda:0")
    B = len(rt.download("TLAS_NODES", np.uint8)) // 64
    root, triBase = B * 1024, B * 1024 + B
    arena = torch.from_numpy(rt.download("BVH_ARENA", np.uint8).copy()).to(dev)
    lib = C.CDLL(os.environ.get("LATPROBE_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblatprobe.so"))
    lib.lp_run.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32] + [C.c_void_p] * 5
    maxIt = 1100
    order = np.argsort(iters)[::-1]
    for label, i in (("longest", order[0]), ("p99", order[n // 100]), ("median", order[n // 2])):
        ray = torch.tensor(list(o[i]) + list(dd[i]) + [0.0, 0.0], dtype=torch.float32, device=dev)
        hit = torch.zeros(4, dtype=torch.float32, device=dev)
        it = torch.zeros(2, dtype=torch.int32, device=dev)
        ts = torch.zeros(2 * maxIt, dtype=torch.int32, device=dev)
        kind = torch.zeros(maxIt, dtype=torch.int32, device=dev)
        for rep in range(3):  # the last run is the warm one reported
            rc = lib.lp_run(arena.data_ptr(), root, triBase, ray.data_ptr(), hit.data_ptr(), it.data_ptr(),
                            ts.data_ptr(), kind.data_ptr())
            if rc != 0:
                raise SystemExit("lp_run failed: %d" % rc)
        hh = hit.cpu().numpy()
        k, cal = (int(x) for x in it.cpu().numpy())
        same = (hh[0] == t[i]) and (int(hh[1].view(np.int32)) == int(tri[i])) and k == int(iters[i])
        T = unwrap(ts.cpu().numpy()[:2 * k]).reshape(k, 2)
        K = kind.cpu().numpy()[:k]
        wait = T[1:, 1] - T[1:, 0]            # iterations 1..k-1 (0 is the setup's)
        work = T[2:, 0] - T[1:-1, 1]          # start of the next minus arrival
        kk = K[1:-1]
        print("%s ray %d: iters %d (queue tracer %d), hit equal: %s, total %.0f clocks, %.0f per iteration "
              "(one reading costs %d)" % (label, i, k, iters[i], same, T[-1, 0] - T[1, 0],
                                          (T[-1, 0] - T[1, 0]) / max(1, k - 2), cal))
        for kname, kv in (("node", 0), ("triangle", 1), ("tlas leaf", 2)):
            m = kk == kv
            if m.any():
                print("   %-10s n=%4d  wait mean %6.0f med %6.0f   work mean %6.0f med %6.0f" % (
                    kname, m.sum(), wait[:-1][m].mean(), np.median(wait[:-1][m]), work[m].mean(), np.median(work[m])))
    rt.cleanup()


if __name__ == "__main__":
    main()
