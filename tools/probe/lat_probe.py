#!/usr/bin/env python3
"""Anatomy of a lone ray's TraverseBvh iteration (tools/probe/lat_probe.hip): per iteration the
load wait left at its start and its own work, in core clocks, by iteration kind, for the longest
and the median step-3 bounce ray of the default 1080p frame.  The probe's hit must equal the
queue tracer's (rt_trace_rays) for the same ray."""
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


def joint_nodes(nodes, tlas):
    """The candidate record format of k_probe2: [BLAS nodes | TLAS nodes], child words in q3.xy."""
    LEAF, BLAS = np.uint32(0x80000000), np.uint32(0x40000000)
    B = len(tlas) // 16
    nodes = nodes.reshape(-1, 16)[:B * 1024]
    tlas = tlas.reshape(-1, 16)[:B]
    joint = np.concatenate([nodes, tlas]).astype(np.uint32)
    b = (np.arange(B * 1024, dtype=np.uint32) // 1024) * 1024
    for c in (0, 1):
        idx, leaf = nodes[:, 12 + c], nodes[:, 14 + c] != 0
        joint[:B * 1024, 12 + c] = np.where(leaf, LEAF | BLAS | (b + idx), BLAS | (b + idx))
        idx, leaf = tlas[:, 12 + c], tlas[:, 14 + c] != 0
        joint[B * 1024:, 12 + c] = np.where(leaf, LEAF | (idx * 1024), np.uint32(B * 1024) + idx)
    return np.ascontiguousarray(joint), B * 1024


def joint4_nodes(nodes, tlas, tripos):
    """step4's format: [BLAS nodes | TLAS nodes | triangles as 64-B records (v0 v1 v2, (index, 0, 0, 0))];
    BLAS-leaf words index the triangle records."""
    joint, root = joint_nodes(nodes, tlas)
    LEAF, BLAS = np.uint32(0x80000000), np.uint32(0x40000000)
    nrec = len(joint)
    tp = tripos.view(np.uint32).reshape(-1, 12)
    T = np.zeros((len(tp), 16), np.uint32)
    T[:, :12] = tp
    T[:, 12] = np.arange(len(tp), dtype=np.uint32)
    B = len(tlas) // 16
    blas = joint[:B * 1024, 12:14]
    tri = (blas & (LEAF | BLAS)) == (LEAF | BLAS)
    blas[tri] = (LEAF | BLAS) | ((blas[tri] & np.uint32(0x3FFFFFFF)) + np.uint32(nrec))
    joint[:B * 1024, 12:14] = blas
    return np.ascontiguousarray(np.concatenate([joint, T])), root


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
    arrs = {k: torch.from_numpy(rt.download(k, np.uint8).copy()).to(dev) for k in ("TRI_POS", "NODES", "TLAS_NODES")}
    lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblatprobe.so"))
    lib.lp_run.argtypes = [C.c_void_p] * 8
    lib.lp_run2.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32] + [C.c_void_p] * 5 + [C.c_int]
    joint, root = joint_nodes(rt.download("NODES", np.uint32), rt.download("TLAS_NODES", np.uint32))
    arrs["JOINT"] = torch.from_numpy(joint.view(np.uint8).reshape(-1)).to(dev)
    joint4, _ = joint4_nodes(rt.download("NODES", np.uint32), rt.download("TLAS_NODES", np.uint32),
                             rt.download("TRI_POS", np.uint32))
    arrs["JOINT4"] = torch.from_numpy(joint4.view(np.uint8).reshape(-1)).to(dev)
    maxIt = 1100
    order = np.argsort(iters)[::-1]
    for (label, i), fmt in [(x, f) for x in (("longest", order[0]), ("p99", order[n // 100]), ("median", order[n // 2]))
                            for f in ("product", "joint", "joint3", "joint4")]:
        ray = torch.tensor(list(o[i]) + list(dd[i]) + [0.0, 0.0], dtype=torch.float32, device=dev)
        hit = torch.zeros(4, dtype=torch.float32, device=dev)
        it = torch.zeros(2, dtype=torch.int32, device=dev)
        ts = torch.zeros(2 * maxIt, dtype=torch.int32, device=dev)
        kind = torch.zeros(maxIt, dtype=torch.int32, device=dev)
        for rep in range(3):  # the last run is the warm one reported
            if fmt == "product":
                rc = lib.lp_run(arrs["TRI_POS"].data_ptr(), arrs["NODES"].data_ptr(), arrs["TLAS_NODES"].data_ptr(),
                                ray.data_ptr(), hit.data_ptr(), it.data_ptr(), ts.data_ptr(), kind.data_ptr())
            else:
                rc = lib.lp_run2(arrs["TRI_POS"].data_ptr(), arrs["JOINT4" if fmt == "joint4" else "JOINT"].data_ptr(),
                                 root, ray.data_ptr(), hit.data_ptr(), it.data_ptr(), ts.data_ptr(), kind.data_ptr(),
                                 {"joint": 2, "joint3": 3, "joint4": 4}[fmt])
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
        print("[%s] %s ray %d: iters %d (queue tracer %d), hit equal: %s, total %.0f clocks, %.0f per iteration "
              "(one reading costs %d)" % (fmt, label, i, k, iters[i], same, T[-1, 0] - T[1, 0],
                                          (T[-1, 0] - T[1, 0]) / max(1, k - 2), cal))
        for kname, kv in (("node", 0), ("triangle", 1), ("tlas leaf", 2)):
            m = kk == kv
            if m.any():
                print("   %-10s n=%4d  wait mean %6.0f med %6.0f   work mean %6.0f med %6.0f" % (
                    kname, m.sum(), wait[:-1][m].mean(), np.median(wait[:-1][m]), work[m].mean(), np.median(work[m])))
    rt.cleanup()


if __name__ == "__main__":
    main()
