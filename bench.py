#!/usr/bin/env python3
"""Benchmark of the hot path on MI355X; prints ONE JSON line (rank 0).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload primary]

Workload "primary" = BASELINE config 2 on the default procedural scene: per step one
per-frame LBVH rebuild (the reference rebuilds every frame, kernel.cu:330-331) plus
GenerateRay + RaySceneIntersect for every pixel of a 1920x1080 frame (1 spp).  The metric
is BASELINE.json's: Mray/s (+ ms/frame and the LBVH build ms as extra fields).

With N ranks (torch.distributed.run, one per GPU) the frame is split into N horizontal
strips (screen-tile split): each rank traces its rows; no collective sits on
the data path of this workload.  Timing: barrier + device sync on both sides of exactly K
steps, max over ranks.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "real-time-ray-tracing_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="primary", choices=["primary"])
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(width, height):
    """Oracle (CPU restatement) traversal of a bounded sample of the same primary rays."""
    from oracle import oracle as O

    threads = min(16, os.cpu_count() or 1)
    v, i, n = O.scene(1)
    bvh = O.build_bvh(v, i, n, O.smooth_normals(v, i))
    rows = min(height, 540)
    rays, _ = O.primary_rays(width, height, 1)
    sample = np.ascontiguousarray(rays[: width * rows])
    reps = 0
    t0 = time.perf_counter()
    while True:
        O.intersect(bvh, sample, threads)
        reps += 1
        if time.perf_counter() - t0 > 10.0 or reps >= 200:
            break
    dt = time.perf_counter() - t0
    return {"value": round(sample.shape[0] * reps / dt / 1e6, 3), "unit": "Mray/s", "cores": threads,
            "kind": "port",
            "sample": "%d x %d primary rays of the 1080p default-camera frame, traversed %d times by the "
                      "oracle (oracle/traverse.cpp) on %d host threads" % (width, rows, reps, threads)}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import rtx

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    W, H = args.width, args.height
    tmp = tempfile.mkdtemp(prefix="rtxbench")
    y0, rows = (H * rank) // world, (H * (rank + 1)) // world - (H * rank) // world
    cfg = rtx.write_config(os.path.join(tmp, "bench.toml"), W, H, dynamic=False, chunk_dim=1,
                           extra="stripY0 = %d\nstripRows = %d\n" % (y0, rows))
    rt = rtx.RayTracer(W, H, cfg).init()

    def step(frame):
        rt.build_bvh()
        rt.trace_primary(frame, detail=False)

    for k in range(args.warmup):
        step(1 + k)
    rt.sync()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(1 + k)
    rt.sync()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    dt = t1 - t0
    if world > 1:
        tt = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms_per_step = dt * 1e3 / args.steps
    rays_total = W * H * args.steps
    value = rays_total / dt / 1e6

    # ---- roofline of the dominant kernel (primary traversal), HIP events on the ctx stream
    rt.trace_primary(1, detail=True)
    stats = rt.download("HIT_STATS", np.uint32).reshape(-1, 4)[y0 * W:(y0 + rows) * W]
    visits, tests = int(stats[:, 0].sum(dtype=np.uint64)), int(stats[:, 1].sum(dtype=np.uint64))
    nrays = W * rows
    alg_bytes = 24 * nrays + 16 * nrays + 64 * visits + 48 * tests
    iters = 100
    ms = rt.time_stage(1, iters) / iters
    achieved = alg_bytes / (ms * 1e-3) / 1e9
    build_ms = rt.time_stage(0, 50) / 50
    info = rt.info()
    build_bytes = 348 * info.triCount  # BASELINE.md algorithmic bytes per triangle
    rt.cleanup()

    result = {
        "metric": "Mray/s + ms/frame at 1080p 4spp (1/2/4/8 GPU); LBVH build ms",
        "value": round(value, 3),
        "unit": "Mray/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: the reference's default procedural scene (Perlin terrain, 60,800 triangles) "
                "and default camera",
        "config": {"workload": "BASELINE config 2: 1920x1080, 1 spp primary rays only + per-frame LBVH rebuild",
                   "width": W, "height": H, "spp": 1, "parallelism": "screen strips x%d" % world},
        "lbvh_build_ms": round(build_ms, 5),
        "lbvh_build_roofline": {"bound": "hbm", "achieved": round(build_bytes / (build_ms * 1e-3) / 1e9, 2),
                                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": round(build_bytes / (build_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                                "traffic": None},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                     "kernel": "k_trace_primary", "kernel_ms": round(ms, 5),
                     "algorithmic_bytes": alg_bytes, "node_visits": visits, "tri_tests": tests},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(W, H)
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
