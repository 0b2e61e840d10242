#!/usr/bin/env python3
"""Phase anatomy of the config-4 LBVH build (958,720 triangles, 937 batches) from a stamped build
(-DRTX_BVH_STAMPS, tools/abl_build.sh bvhstamps): per workgroup the s_memtime clocks of gather +
Morton, the radix sort, Karras, the refit + node stores, the arrival; the s_memrealtime (100 MHz)
start / end spread across workgroups and the TLAS tail.  Usage: RTX_LIB=<stamped lib> python tools/lbvh_stamps.py"""
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]


def main():
    import rtx
    chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    r4 = rtx.RayTracer(256, 144, rtx.write_config(os.path.join(tempfile.mkdtemp(), "c4.toml"), 256, 144,
                                                   chunk_dim=chunk)).init()
    for _ in range(3):
        r4.build_bvh()
    r4.sync()
    B = int(r4.info().batchCount) if hasattr(r4.info(), "batchCount") else len(r4.download("TLAS_NODES", np.uint8)) // 64
    m = r4.download("MORTON", np.uint32).reshape(-1, 1024)[:B, 1016:1024].astype(np.int64)
    tl = int(r4.download("TLAS_SCENE_AABB", np.uint32)[0])
    r4.cleanup()
    d = lambda a, b: (m[:, b] - m[:, a]) % (1 << 32)  # noqa: E731
    phases = {"gather_morton": d(1, 2), "sort": d(2, 3), "karras": d(3, 4), "refit_stores": d(4, 5),
              "arrival": d(5, 6), "workgroup_total": d(1, 6)}
    rt0 = m[:, 0]
    base = rt0.min()
    start = (rt0 - base) % (1 << 32)
    end = (m[:, 7] - base) % (1 << 32)
    out = {"batches": B,
           "clocks": {k: {"mean": float(v.mean()), "p50": float(np.median(v)), "max": float(v.max())}
                      for k, v in phases.items()},
           "realtime_us": {"starts_spread": float(start.max()) / 100, "last_end": float(end.max()) / 100,
                           "tlas_end": float(((tl - base) % (1 << 32))) / 100,
                           "start_quantiles": [float(np.quantile(start, q)) / 100 for q in (0.25, 0.5, 0.75, 0.9)]}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
