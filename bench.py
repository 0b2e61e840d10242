#!/usr/bin/env python3
"""Benchmark of the per-frame hot path on MI355X; prints ONE JSON line (rank 0).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--width 1920 --height 1080 --spp 4]

A step is one full frame of BASELINE config 3 on the reference's default procedural scene and
camera: per-frame two-level LBVH rebuild (kernel.cu:330-331), the path tracer at 4 spp
(4 reference PathTrace evaluations per pixel), the SVGF-style denoiser and the post chain
(auto-exposure, scale, sharpen, tone map, dither to RGBA8).  The metric is BASELINE.json's:
Mray/s (every RaySceneIntersect that ran a traversal: primary, bounce and shadow rays, counted
on the GPU) with ms/frame and the LBVH build ms as extra fields.

N ranks (torch.distributed.run, one per GPU): each rank rebuilds the BVH, path traces its rows
of the frame (16-row blocks dealt round-robin, so every rank gets its share of the geometry
rows), the ranks' G-buffer blocks are all-gathered over RCCL (rtx/dist.py, one collective per
frame), and every rank runs the denoise/post chain on the full frame (exact vs 1 GPU).
Total work per frame is fixed as N grows ("strong" scaling).  Timing: barrier + device sync on
both sides of exactly K frames, max over ranks; value = rays of all ranks / that time.

Frames are pipelined (rt_set_post_stream; --no-pipeline for serial frames): the denoise/post
chain of frame f runs on a second stream beside the trace kernels of frame f+1, and the LBVH
build + camera rays of frame f+1 on a third beside the trace tails of frame f.  Every frame's
full work is inside the timed region: the last frame's deferred denoise is issued and waited
for (rt.sync) before the closing device sync.
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

HBM_PEAK_GBS = 8000.0  # /opt/skills/guides/MI355X_MICROARCH.md (spec peak)
DELTA_MS = 16.667      # fixed AutoExposure step (SURVEY §8d determinism settings)
PMC_FILE = os.path.join(ROOT, "profiles", "r01_pmc_pathtrace.json")

# algorithmic bytes of one path-trace stage launch: per traced ray the node and
# triangle records a traversal must read, per pixel the G-buffer it writes, per diffuse event
# the 48 texel taps of the triplanar soil textures
NODE_B, TRI_B, GBUF_B, TEX_B = 64, 48, 30, 48 * 8


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the per-stage and 1M-triangle side measurements")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="gloo: rehearse the multi-rank path with ranks sharing a GPU (not a measurement)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="serial frames (no post stream): denoise of frame f does not overlap the trace of f+1")
    return ap.parse_args()


def cpu_baseline(width, height, spp):
    """Oracle (CPU restatement) path trace of a bounded sample of the same frame."""
    from oracle import oracle as O

    threads = 16
    v, i, n = O.scene(1)
    bvh = O.build_bvh(v, i, n, O.smooth_normals(v, i))
    sky, tex = O.sky(), O.textures()
    rows = min(height, 32)
    y0 = height // 2 - rows // 2
    rays = 0
    reps = 0
    t0 = time.perf_counter()
    while True:
        g = O.pathtrace(bvh, width, height, frame_num=1 + reps, spp=spp, sky_out=sky, tex=tex, y0=y0, rows=rows,
                        threads=threads)
        rays += int(g["rays"].sum(dtype=np.uint64))
        reps += 1
        if time.perf_counter() - t0 > 10.0 or reps >= 400:
            break
    dt = time.perf_counter() - t0
    return {"value": round(rays / dt / 1e6, 3), "unit": "Mray/s", "cores": threads, "kind": "port",
            "sample": "%d x %d centre rows of the %dx%d frame at %d spp, path traced %d times by the oracle "
                      "(oracle/pathtrace.cpp, full PathTrace incl. traversal, textures, sky) on %d host threads"
                      % (width, rows, width, height, spp, reps, threads)}


def pmc_traffic():
    if not os.path.exists(PMC_FILE):
        return None, None
    with open(PMC_FILE) as f:
        d = json.load(f)
    return d.get("hbm_bytes_per_launch"), os.path.relpath(PMC_FILE, ROOT)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import rtx
    from rtx.dist import StripGather, strip_blocks, strip_config

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dist_backend == "gloo":  # rehearsal of the N-rank path with ranks sharing GPUs
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    W, H, S = args.width, args.height, args.spp
    rows = sum(r for _, r in strip_blocks(H, world, rank))
    tmp = tempfile.mkdtemp(prefix="rtxbench")
    cfg = rtx.write_config(os.path.join(tmp, "bench.toml"), W, H, dynamic=False, chunk_dim=1, spp=S,
                           extra=strip_config(world, rank))
    rt = rtx.RayTracer(W, H, cfg).init()
    rt.set_delta_time(DELTA_MS)
    pipeline = not args.no_pipeline
    if pipeline:  # the trace chain is the critical path: its stream outranks the denoise stream
        lo, hi = torch.cuda.Stream.priority_range()
        main_stream = torch.cuda.Stream(dev, priority=hi)
        post = torch.cuda.Stream(dev, priority=lo)
        torch.cuda.set_stream(main_stream)
    else:
        post = None
    rt.set_stream(torch.cuda.current_stream(dev).cuda_stream)  # collectives order with the renderer
    if pipeline:  # denoise/post of frame f on a second stream, overlapping the trace of frame f+1
        rt.set_post_stream(post.cuda_stream)
    sg = StripGather(W, H, world, rank, dev, rt, sets=rtx.GBUFFER_SETS if pipeline else 1) if world > 1 else None
    # RCCL gathers on a stream of their own: the next frame's path trace does not wait for the
    # collective, only the frame's own denoise does (rt_set_gather_stream)
    gs = torch.cuda.Stream(dev) if (sg is not None and args.dist_backend == "nccl") else None
    if gs is not None:
        rt.set_gather_stream(gs.cuda_stream)

    def frame(f):
        rt.build_bvh()
        rt.path_trace(f)
        if sg is not None:
            if gs is not None:
                gs.wait_stream(torch.cuda.current_stream(dev))  # this frame's path trace
                with torch.cuda.stream(gs):
                    sg.gather()
            else:
                rt.sync()  # gloo copies through the host: the strip must be complete
                sg.gather()
        rt.denoise_post(f)

    for k in range(args.warmup):
        frame(1 + k)
    rt.sync()
    rt.ray_count(reset=True)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        frame(args.warmup + 1 + k)
    rt.sync()  # issues the last frame's deferred denoise/post and waits for every renderer stream
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    dt = t1 - t0
    rays = rt.ray_count()
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        r = torch.tensor([rays], device=dev, dtype=torch.int64)
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        rays = int(r.item())
    ms_per_step = dt * 1e3 / args.steps
    value = rays / dt / 1e6

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
        "data": "synthetic: the reference's default procedural scene (Perlin terrain, 60,800 triangles), "
                "default camera and sky, deterministic stand-in soil textures",
        "config": {"workload": "BASELINE config 3: %dx%d, %d spp path trace + SVGF denoise + auto-exposure/"
                               "tone map, per-frame LBVH rebuild" % (W, H, S),
                   "width": W, "height": H, "spp": S,
                   "parallelism": ("interleaved 16-row strips x%d + RCCL all-gather of G-buffers" % world if world > 1
                                   else "single GPU")
                                  + ("; pipelined frames: denoise/post of f-1 and LBVH build + camera rays of "
                                     "f+1 on their own streams beside the trace kernels of f" if pipeline
                                     else "; serial frames")},
        "fps": round(1000.0 / ms_per_step, 2),
        "rays_per_frame": int(rays // args.steps),
    }

    # ---- roofline of the path-trace stage over this rank's strip: the stage is the
    # dominant part of the frame; its seven kernels hand rays to each other through queues in HBM,
    # so the stage, not one kernel of it, is the unit whose algorithmic bytes are defined
    rt.path_trace(args.warmup + args.steps + 1, detail=True)
    st = rt.download("PT_STATS", np.uint32).reshape(-1, 4).astype(np.uint64)  # zero outside this rank's rows
    n_rays, visits, tests, diffuse = (int(st[:, k].sum()) for k in range(4))
    alg_bytes = NODE_B * visits + TRI_B * tests + GBUF_B * W * rows + TEX_B * diffuse
    iters = 20
    pt_ms = rt.time_stage(2, iters) / iters
    kernels_ms = rt.time_path_trace_kernels(iters)
    achieved = alg_bytes / (pt_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic() if (W, H, S) == (1920, 1080, 4) else (None, None)  # PMC file's workload
    result["roofline"] = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                          "kernel": "path-trace stage (" + " -> ".join(kernels_ms) + ")",
                          "kernel_ms": round(pt_ms, 5),
                          "kernels_ms": {k: round(v, 5) for k, v in kernels_ms.items()},
                          "algorithmic_bytes": alg_bytes,
                          "rays": n_rays, "node_visits": visits, "tri_tests": tests, "diffuse_events": diffuse}
    if traffic_src:
        result["roofline"]["traffic_source"] = traffic_src

    if not args.no_extras:
        build_ms = rt.time_stage(0, 50) / 50
        info = rt.info()
        result["lbvh_build_ms"] = round(build_ms, 5)
        result["lbvh_build_tris"] = int(info.triCount)
        result["stage_ms"] = {"lbvh_build": round(build_ms, 5), "path_trace": round(pt_ms, 5),
                              "denoise_post": round(rt.time_stage(4, 20) / 20, 5),
                              "primary_rays_1spp": round(rt.time_stage(1, 20) / 20, 5)}
        result["primary_mray_s"] = round(W * rows / (result["stage_ms"]["primary_rays_1spp"] * 1e-3) / 1e6, 2)
    rt.cleanup()

    if not args.no_extras and rank == 0:
        # BASELINE config 4: per-frame rebuild of the ~1M-triangle variant (chunkDim 4)
        cfg4 = rtx.write_config(os.path.join(tmp, "c4.toml"), 256, 144, chunk_dim=4)
        r4 = rtx.RayTracer(256, 144, cfg4).init()
        r4.build_bvh()
        r4.sync()
        ms4 = r4.time_stage(0, 30) / 30
        n4 = r4.info().triCount
        r4.cleanup()
        result["lbvh_build_1m"] = {"tris": int(n4), "ms": round(ms4, 5),
                                   "roofline": {"bound": "hbm", "achieved": round(348 * n4 / (ms4 * 1e-3) / 1e9, 2),
                                                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                                "frac": round(348 * n4 / (ms4 * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                                                "traffic": None}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(W, H, S)
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
