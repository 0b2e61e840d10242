#!/usr/bin/env python3
"""Benchmark of the per-frame hot path on MI355X; prints ONE JSON line (rank 0).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--width 1920 --height 1080 --spp 4]

A step is one full frame of BASELINE config 3 on the reference's default procedural scene and
camera: per-frame two-level LBVH rebuild (kernel.cu:330-331), the path tracer at 4 spp
(4 reference PathTrace evaluations per pixel), the SVGF-style denoiser and the post chain
(auto-exposure, scale, sharpen, tone map, dither to RGBA8).  The metric is BASELINE.json's:
Mray/s (every RaySceneIntersect that ran a traversal: primary, bounce and shadow rays, counted
on the GPU) with ms/frame and the LBVH build ms as extra fields.

The frames run through rtx.frames.FramePipeline, the object tests/test_gpu_bench_path.py checks
against the oracle: pipelined frames (the denoise/post chain of frame f on a second stream
beside the trace kernels of frame f+1, the LBVH build + camera rays of frame f+1 on a third
beside the trace tails of frame f; --no-pipeline for serial frames).  Every frame's full work
is inside the timed region: the last frame's deferred denoise is issued and waited for before
the closing device sync.  After timing, rank 0 re-renders the same frame sequence serially in a
fresh single-GPU context and compares the last frame bit for bit (--no-self-check skips it); a
mismatch exits non-zero.

N ranks (torch.distributed.run, one per GPU): each rank rebuilds the BVH, path traces its rows
of the frame (16-row blocks dealt round-robin), the G-buffer blocks each rank's denoise reads are
sent to it in one RCCL all-to-all (its strip plus the halo its passes read: rtx/dist.py
StripGather.exchange), and each rank denoises only its own contiguous 64-row-block strip,
exchanging the histogram (all-reduce) and its rows of the accumulation, history (the final HDR)
and RGBA8 buffers (all-gather) with the others.
Rank 0's self-check compares its frame with a single-GPU serial render.  Total work per frame is
fixed as N grows ("strong" scaling).  Timing: barrier + device sync on both sides of exactly
K frames, max over ranks; value = rays of all ranks / that time.

Roofline: per path-trace kernel, algorithmic bytes from the GPU's own work
counters (node visits x 64 B, triangle tests x 48 B, texel taps, queue records); per denoise / post
kernel its compulsory G-buffer / colour bytes (denoise_bytes); each over the kernel's HIP-event
duration inside pipelined frames.  The top-level kernel is the longest kernel of the stream that
binds the pipelined frame — the stream whose kernels add up to the most time in the warm-up frames,
which have every kernel bracketed by HIP events (rt_frame_marks_begin / _read) — and it is timed in
every one of the K timed frames the same way.  The process running the timed frames launches nothing
else of the frame's kernels (the side measurements run in a child process), so a rocprofv3
--kernel-trace --stats of this command gives, in this process's stats file, averages over exactly
the warm-up + timed + detail + split frames.  The BVH and textures are cache-resident, so the memory
ceiling of the path-trace kernels is L2 (MI355X_MICROARCH.md: 34.5 TB/s) and their HBM traffic
(rocprofv3 PMC passes) sits far below the algorithmic bytes; the denoise kernels are priced against
HBM, with the PMC pass's VALU-busy share beside it.
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

HBM_PEAK_GBS = 8000.0   # /opt/skills/guides/MI355X_MICROARCH.md (spec peak)
L2_PEAK_GBS = 34500.0   # MI355X_MICROARCH.md, L2 (per XCD) section: aggregate L2 bandwidth
# vector-instruction issue: a wave's f32 VALU instruction holds its SIMD 4 cycles (8 for the
# transcendentals; MI355X_MICROARCH.md, 'vector-instruction ISSUE cost'); 256 CUs x 4 SIMDs at the
# 2.4 GHz peak clock.  A kernel's SQ_INSTS_VALU x 4 / (1024 x 2.4 GHz) is the least time its vector
# instruction stream takes on the whole chip (a lower bound: transcendentals and DVFS only add).
VALU_SIMDS, VALU_CYC, CLOCK_GHZ = 1024, 4, 2.4
DELTA_MS = 16.667       # fixed AutoExposure step (SURVEY §8d determinism settings)
PMC_FILE = os.path.join(ROOT, "profiles", "r06_pmc_kernels.json")  # tools/prof.sh pmc of the pipelined frames
PMC_C2C4 = os.path.join(ROOT, "profiles", "r06_pmc_c2c4.json")  # KEY=c2c4 tools/prof.sh pmc probe.py c2c4
TERRAIN_CAM = dict(pos=(8.0, 15.0, -6.0), yaw=0.0, pitch=-0.7)  # ~50 % primary hits (tests' camera)

# algorithmic bytes: per node visit the 64-B node record, per triangle test the
# 48-B vertex record, per diffuse event the 48 texel taps (8 B) of the triplanar soil textures,
# per queue entry its 80-B record (5 float4) written + read and its 20-B hit record, per camera
# sample its 20-B hit record, per pixel the 30-B G-buffer
NODE_B, TRI_B, TEX_B, QREC_B, HIT_B, GBUF_B = 64, 48, 48 * 8, 80, 20, 30

# the frame's three streams and the kernels each runs when pipelined
CONTEXT_KERNELS = ("k_trace_queue<3>", "k_pt_resume<3>", "k_trace_queue<4>", "k_pt_resume<4>", "k_pt_resolve")
DENOISE_KERNELS = ("k_temporal", "k_spatial7", "k_spatial5<3>", "k_spatial5<6>", "k_spatial5<12>", "k_temporal2",
                   "k_downscale_chain", "k_scale_post")


def denoise_stats(rt, W, H):
    """Inputs of the denoise kernels' algorithmic bytes, from the last denoised frame: surface pixels
    (G-buffer depth below the reference's sky depth) and the pixels of the 16x16 tiles above the
    local / large noise thresholds (the tiles SpatialFilter7x7 and the a-trous passes filter; the
    others copy through)."""
    p = rt.params.denoise
    W16, H16 = (W + 15) // 16, (H + 15) // 16
    n16 = rt.get_buffer("NOISE_LEVEL16", (H16, W16), np.float16).astype(np.float32)
    depth = rt.get_buffer("DEPTH", (H, W), np.float16).astype(np.float32)
    tile_px = np.full((H16, W16), 256.0)
    tile_px[-1, :] = 16 * (H - 16 * (H16 - 1))
    tile_px[:, -1] *= (W - 16 * (W16 - 1)) / 16.0
    act7 = ~(n16 < p.noise_threshold_local)
    act5 = ~(n16 < p.noise_threshold_large)
    return {"pixels": W * H, "surface_px": int((depth < 10e9).sum()), "local_active_px": int(tile_px[act7].sum()),
            "large_active_px": int(tile_px[act5].sum()), "local_active_tiles": round(float(act7.mean()), 4),
            "large_active_tiles": round(float(act5.mean()), 4)}


def denoise_bytes(st, Ws, Hs):
    """Compulsory bytes of each denoise / post kernel per launch of the whole-frame chain (DESIGN.md
    §4.2): every input pixel the kernel needs read once, every output written once; stencil taps'
    re-reads of neighbours are cache hits and not counted.  Colour / normal / albedo / accumulation /
    history texels are 8 B (half4), depth 2, motion 4, RGBA8 4.  The noise-gated passes run over the
    active-tile lists: SpatialFilter7x7 and the first two a-trous passes touch only their lists' tiles,
    TemporalFilter writes the other tiles' output into the accumulation buffer as well."""
    P, S, A7, A5 = st["pixels"], st["surface_px"], st["local_active_px"], st["large_active_px"]
    apron7 = 22 * 22 / 256.0 * (8 + 8 + 2)  # SpatialFilter7x7's LDS-staged colour, normal, depth apron
    return {
        # colour, normal, depth in, colour + history depth out; surface: motion, history; gated tiles
        # also into the accumulation buffer
        "k_temporal": 28 * P + 12 * S + 8 * (P - A7),
        "k_spatial7": int((apron7 + 8 + 2) * A7),  # list 0: apron, out, the noise epilogue's depth
        # list 1: colour, normal, depth in, colour out; the first pass also writes the last pass's
        # output for the tiles off list 1 (accumulation and albedo in, colour out)
        "k_spatial5<3>": 26 * A5 + 24 * (P - A5),
        "k_spatial5<6>": 26 * A5,
        "k_spatial5<12>": 34 * A5,                # list 1: colour, normal, depth, albedo in, colour out
        "k_temporal2": 28 * P,                    # colour, motion, history in, history out
        "k_downscale_chain": 8 * P + P // 2 + P // 32,  # colour in, 1/4 and 1/16 levels out
        "k_scale_post": 8 * P + 12 * Ws * Hs,     # render colour in, scaled half4 + RGBA8 out
    }


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the per-stage, terrain and 1M-triangle side measurements")
    ap.add_argument("--no-self-check", action="store_true", help="skip the serial re-render of the timed sequence")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="gloo: rehearse the multi-rank path with ranks sharing a GPU (not a measurement)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="serial frames (no post stream): denoise of frame f does not overlap the trace of f+1")
    ap.add_argument("--no-marks", action="store_true",
                    help="no HIP events in the timed frames (A/B of their cost; the roofline then has no kernel ms)")
    ap.add_argument("--extras-child", action="store_true", help=argparse.SUPPRESS)  # side legs, own process
    ap.add_argument("--check-file", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--check-frames", type=int, default=0, help=argparse.SUPPRESS)
    return ap.parse_args()


def host_threads():
    """Threads for the CPU legs: the CPUs this process may run on, capped by OMP_NUM_THREADS (the
    GPU box sets it to the job's CPU share; os.cpu_count() there is the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(width, height, spp):
    """The oracle (CPU restatement, kind "port") on this host's cores: the LBVH build of both
    scene sizes, primary-ray traversal of the full frame, and the full path trace of a bounded
    sample of the frame (the metric's unit)."""
    from oracle import oracle as O

    threads = host_threads()
    out = {"unit": "Mray/s", "cores": threads, "kind": "port", "nproc": os.cpu_count(), "cpu_model": cpu_model()}
    legs = {}
    for cd, key in ((1, "lbvh_build_60800"), (4, "lbvh_build_958720")):
        v, i, n = O.scene(cd)
        nrm = O.smooth_normals(v, i)
        O.build_bvh(v, i, n, nrm, threads=threads)  # warm
        reps, t0 = 0, time.perf_counter()
        while True:
            O.build_bvh(v, i, n, nrm, threads=threads)
            reps += 1
            if time.perf_counter() - t0 > 1.0 or reps >= 200:
                break
        legs[key] = {"tris": int(n), "ms": round((time.perf_counter() - t0) * 1e3 / reps, 3), "reps": reps}
    v, i, n = O.scene(1)
    bvh = O.build_bvh(v, i, n, O.smooth_normals(v, i), threads=threads)
    rays, _ = O.primary_rays(width, height, 1)
    reps, t0 = 0, time.perf_counter()
    while True:
        O.intersect(bvh, rays, threads=threads)
        reps += 1
        if time.perf_counter() - t0 > 3.0 or reps >= 20:
            break
    dt = time.perf_counter() - t0
    legs["primary_rays"] = {"mray_s": round(rays.shape[0] * reps / dt / 1e6, 3), "rays": int(rays.shape[0]),
                            "reps": reps, "what": "%dx%d primary rays, frame 1, default camera (GenerateRay + "
                                                  "TraverseBvh + hit tail)" % (width, height)}
    sky, tex = O.sky(), O.textures()
    rows = min(height, 32)
    y0 = height // 2 - rows // 2
    nrays = reps = 0
    t0 = time.perf_counter()
    while True:
        g = O.pathtrace(bvh, width, height, frame_num=1 + reps, spp=spp, sky_out=sky, tex=tex, y0=y0, rows=rows,
                        threads=threads)
        nrays += int(g["rays"].sum(dtype=np.uint64))
        reps += 1
        if time.perf_counter() - t0 > 10.0 or reps >= 400:
            break
    dt = time.perf_counter() - t0
    out["value"] = round(nrays / dt / 1e6, 3)
    out["sample"] = ("%d x %d centre rows of the %dx%d frame at %d spp, path traced %d times by the oracle "
                     "(oracle/pathtrace.cpp, full PathTrace incl. traversal, textures, sky) on %d host threads; "
                     "legs: LBVH build of both scenes (oracle/bvh.cpp, batches over threads), full-frame primary "
                     "traversal" % (width, rows, width, height, spp, reps, threads))
    legs["c1_frame_256"] = c1_frame(O, threads)
    out["legs"] = legs
    return out


def c1_frame(O, threads, size=256):
    """BASELINE config 1 on the host: the default scene at 256x256, 1 spp, one whole frame on the
    CPU (LBVH build, PathTrace, the 13-pass denoise + post), ending in an HDR dump (PFM of the
    pre-tone-map colour) - the oracle's restatement of the reference path, no GPU involved."""
    t0 = time.perf_counter()
    v, i, n = O.scene(1)  # init (init.cu): scene input, sky tables, textures, denoiser state
    nrm = O.smooth_normals(v, i)
    sky, tex = O.sky(), O.textures()
    dn = O.Denoiser(size, size)
    t1 = time.perf_counter()
    bvh = O.build_bvh(v, i, n, nrm, threads=threads)
    t2 = time.perf_counter()
    g = O.pathtrace(bvh, size, size, frame_num=1, spp=1, sky_out=sky, tex=tex, threads=threads)
    t3 = time.perf_counter()
    out = dn.draw(g, 1)
    t4 = time.perf_counter()
    hdr = out["scaled"].view(np.float16).astype(np.float32).reshape(size, size, 4)[::-1, :, :3]
    path = os.path.join(tempfile.gettempdir(), "rtx_c1_%d.pfm" % os.getpid())
    with open(path, "wb") as f:  # PFM: bottom row first, little-endian scale
        f.write(b"PF\n%d %d\n-1.0\n" % (size, size))
        f.write(np.ascontiguousarray(hdr, dtype="<f4").tobytes())
    t5 = time.perf_counter()
    os.remove(path)
    rays = int(g["rays"].sum(dtype=np.uint64))
    ms = lambda a, b: round((b - a) * 1e3, 3)
    return {"size": [size, size], "spp": 1, "threads": threads, "init_ms": ms(t0, t1),
            "lbvh_build_ms": ms(t1, t2), "path_trace_ms": ms(t2, t3), "denoise_post_ms": ms(t3, t4),
            "hdr_dump_ms": ms(t4, t5), "frame_ms": ms(t1, t5), "rays": rays,
            "path_trace_mray_s": round(rays / max(t3 - t2, 1e-9) / 1e6, 3)}


def pmc_kernels():
    if not os.path.exists(PMC_FILE):
        return None
    with open(PMC_FILE) as f:
        return json.load(f)


def kernel_roofline(q, W, rows, S, kernels_ms, pmc, workload_matches):
    """Per-kernel algorithmic bytes (from the detail launch's work counters q = RT_ARR_PT_QUEUE)
    over the kernel's HIP-event ms."""
    q = q.astype(np.int64)
    n3, n4 = int(q[0]), int(q[1])
    vc, tc, vs, ts, v3, t3, v4, t4, ds, d3 = (int(q[k]) for k in range(12, 22))
    surf = int(q[11])
    px = W * rows
    alg = {
        "k_pt_camera": NODE_B * vc + TRI_B * tc + HIT_B * px * S + GBUF_B * (px - surf),
        "k_pt_shade0": HIT_B * surf * S + TEX_B * ds + NODE_B * vs + TRI_B * ts + QREC_B * n3 + GBUF_B * surf,
        "k_trace_queue<3>": NODE_B * v3 + TRI_B * t3 + (32 + HIT_B) * n3,
        "k_pt_resume<3>": (QREC_B + HIT_B) * n3 + TEX_B * d3,
        "k_trace_queue<4>": NODE_B * v4 + TRI_B * t4 + (32 + HIT_B) * n4,
        "k_pt_resume<4>": (QREC_B + HIT_B) * n4,
        "k_pt_resolve": 16 * S * surf + 8 * surf,
    }
    work = {"k_pt_camera": {"node_visits": vc, "tri_tests": tc, "samples": px * S, "culled": int(q[22])},
            "k_pt_shade0": {"diffuse_events": ds, "surface_pixels": surf, "node_visits": vs, "tri_tests": ts},
            "k_trace_queue<3>": {"rays": n3, "node_visits": v3, "tri_tests": t3, "max_iterations": int(q[8])},
            "k_pt_resume<3>": {"rays": n3, "diffuse_events": d3},
            "k_trace_queue<4>": {"rays": n4, "node_visits": v4, "tri_tests": t4, "max_iterations": int(q[9])},
            "k_pt_resume<4>": {"rays": n4}, "k_pt_resolve": {}}
    out = {}
    for k, ms in kernels_ms.items():
        if k not in alg:
            continue
        a = alg[k] / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        e = {"ms": round(ms, 5), "algorithmic_bytes": int(alg[k]), "achieved_GBs": round(a, 1),
             "frac_l2": round(a / L2_PEAK_GBS, 4), "work": work[k]}
        add_pmc(e, k, pmc, workload_matches)
        out[k] = e
    return out


def valu_issue_us(insts):
    """least time a kernel's SQ_INSTS_VALU wave-instructions take to issue on the whole chip"""
    return insts * VALU_CYC / VALU_SIMDS / (CLOCK_GHZ * 1e3)


# the denoise kernels' HIP-event names (by position in the chain) -> their PMC names when the frame
# runs the active-tile-list chain: the list kernels (two threads per pixel since
# round 6, one before) replace the full-frame ones
PMC_LIST_NAMES = {"k_spatial7": ("k_spatial7_list2", "k_spatial7_list"),
                  "k_spatial5<3>": ("k_spatial5_list2<3>", "k_spatial5_list<3>"),
                  "k_spatial5<6>": ("k_spatial5_list2<6>", "k_spatial5_list<6>"),
                  "k_spatial5<12>": ("k_spatial5_list2<12>",)}


def pmc_entry(pmc, k):
    ks = pmc.get("kernels", {})
    for name in PMC_LIST_NAMES.get(k, ()) + (k,):
        if ks.get(name):
            return ks[name]
    return None


def add_pmc(e, k, pmc, workload_matches):
    if pmc and workload_matches and pmc_entry(pmc, k):
        pk = pmc_entry(pmc, k)
        for f in ("hbm_bytes", "l2_hit_rate", "wait_inst_any_frac", "wait_any_frac", "valu_busy_frac",
                  "valu_per_wave"):
            if f in pk:
                e[f] = pk[f]
        insts = pk.get("counters_median", {}).get("SQ_INSTS_VALU")
        if insts:
            e["valu_wave_insts"] = int(insts)
            e["valu_issue_us"] = round(valu_issue_us(insts), 2)


def frame_valu_issue(kernels, ms_per_step, pmc, workload_matches):
    """The frame's vector-instruction issue bound: the VALU wave-instructions of every kernel of a
    frame (PMC medians per dispatch, one dispatch each per frame) issued at the chip's full rate,
    against the measured frame time.  Near 1 means the frame is bound by instruction issue, not by
    memory: what shortens it is fewer instructions (or packed ones), not more overlap."""
    if not (pmc and workload_matches):
        return None
    per = {}
    for k in kernels:
        pk = pmc_entry(pmc, k)
        insts = (pk or {}).get("counters_median", {}).get("SQ_INSTS_VALU")
        if insts:
            per[k] = int(insts)
    if not per:
        return None
    tot = sum(per.values())
    us = valu_issue_us(tot)
    return {"valu_wave_insts": tot, "issue_ms": round(us / 1e3, 4), "frame_ms": ms_per_step,
            "frac": round(us / 1e3 / ms_per_step, 4),
            "by_kernel_us": {k: round(valu_issue_us(v), 2) for k, v in sorted(per.items(), key=lambda kv: -kv[1])},
            "model": "SQ_INSTS_VALU x %d cycles / (%d SIMDs x %.1f GHz)" % (VALU_CYC, VALU_SIMDS, CLOCK_GHZ),
            "source": os.path.relpath(PMC_FILE, ROOT)}


def denoise_roofline(st, Ws, Hs, kernels_ms, pmc, workload_matches):
    """Per denoise / post kernel: compulsory bytes (denoise_bytes) over its HIP-event ms against HBM.
    The active tiles' stencil arithmetic, not bandwidth, sets most of these kernels' time: the PMC
    pass's VALU-busy share says how far they are from their issue bound."""
    alg = denoise_bytes(st, Ws, Hs)
    out = {}
    for k in DENOISE_KERNELS:
        ms = kernels_ms.get(k)
        if ms is None:
            continue
        a = alg[k] / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        e = {"ms": round(ms, 5), "algorithmic_bytes": int(alg[k]), "achieved_GBs": round(a, 1),
             "frac_hbm": round(a / HBM_PEAK_GBS, 4)}
        add_pmc(e, k, pmc, workload_matches)
        out[k] = e
    return out


def stream_kernels(shade_on_side):
    """The kernels of each stream of a pipelined frame: side (camera rays [+ shade]), context (the
    bounce / shadow queue chain [+ shade]), post (denoise + post)."""
    side = ("k_pt_camera", "k_pt_shade0") if shade_on_side else ("k_pt_camera",)
    ctx = CONTEXT_KERNELS if shade_on_side else ("k_pt_shade0",) + CONTEXT_KERNELS
    return {"side": [k for k in side], "context": list(ctx), "post": list(DENOISE_KERNELS)}


def pmc_c2c4(kernel, key):
    """HBM bytes per launch and L2 hit rate of a config-2 / config-4 kernel from the committed PMC
    passes (KEY=c2c4 tools/prof.sh <dir> pmc tools/probe.py c2c4 -> profiles/r06_pmc_c2c4.json), when
    its workload matches: k_trace_primary of the 1920x1080 1-spp launch, and the LBVH build of the
    958,720-triangle scene (the build launch with the most workgroups of that run)."""
    if not os.path.exists(PMC_C2C4):
        return {}
    with open(PMC_C2C4) as f:
        pm = json.load(f)
    if pm.get("workload_key") != "c2c4":
        return {}
    ks = pm.get("kernels", {})
    if kernel.startswith("k_build_bvh"):
        builds = [k for k in ks if k.startswith("k_build_bvh@")]
        if not builds or key != "958720 tris":
            return {}
        kernel = max(builds, key=lambda k: int(k.split("@")[1].rstrip("wg")))
    elif key != "1920x1080x1 primary":
        return {}
    e = ks.get(kernel)
    if not e:
        return {}
    out = {k: e[k] for k in ("hbm_bytes", "l2_hit_rate", "valu_busy_frac", "wait_any_frac") if k in e}
    insts = e.get("counters_median", {}).get("SQ_INSTS_VALU")
    if insts:
        out["valu_issue_us"] = round(valu_issue_us(insts), 2)
    return out | {"pmc_kernel": kernel, "traffic_source": os.path.relpath(PMC_C2C4, ROOT)}


def primary_roofline(rt, W, H, ms, frames):
    """BASELINE config 2 (1920x1080, 1 spp primary rays, k_trace_primary alone): algorithmic bytes per
    launch from the kernel's own counters (24 B ray + 16 B hit per ray, 64 B per node visit,
    48 B per triangle test; detail launches of the same frames 1..`frames` the timing ran, averaged),
    over the launch's HIP-event ms, against L2 and HBM; PMC traffic from the committed passes."""
    visits = tests = past_root = 0
    for f in range(1, frames + 1):
        rt.trace_primary(f, detail=True)
        rt.sync()
        hs = rt.download("HIT_STATS", np.uint32).reshape(-1, 4).astype(np.int64)
        visits += int(hs[:, 0].sum())
        tests += int(hs[:, 1].sum())
        past_root += int((hs[:, 3] > 1).sum())
    rays = W * H
    v, t, pr = visits / frames, tests / frames, past_root / frames
    alg = (24 + 16) * rays + NODE_B * v + TRI_B * t
    a = alg / (ms * 1e-3) / 1e9
    out = {"kernel": "k_trace_primary", "workload": "BASELINE config 2: %dx%d, 1 spp primary rays (GenerateRay + "
                                                    "RaySceneIntersect), default scene and camera" % (W, H),
           "kernel_ms": round(ms, 5), "rays": rays, "node_visits": round(v, 1), "tri_tests": round(t, 1),
           "visits_per_ray": round(v / rays, 3), "algorithmic_bytes": int(alg), "achieved": round(a, 1),
           "unit": "GB/s", "bound": "l2", "limiter": "latency", "peak": L2_PEAK_GBS, "frac": round(a / L2_PEAK_GBS, 4),
           "frac_hbm": round(a / HBM_PEAK_GBS, 4), "mray_s": round(rays / (ms * 1e-3) / 1e6, 1),
           "rays_traversed": round(pr, 1), "mray_s_traversed": round(pr / (ms * 1e-3) / 1e6, 1),
           "traversed_definition": "rays whose TraverseBvh ran past the TLAS root (iterations > 1); the rest are "
                                   "settled at the root (by the scene cull or the exact root box test)",
           "counters": "HIT_STATS of detail launches of frames 1..%d (the timed launches' frames)" % frames,
           "timing": "rt_time_stage(1, %d): HIP events around %d back-to-back launches, frames 1..%d" % (
               frames, frames, frames)}
    pm = pmc_c2c4("k_trace_primary", "%dx%dx1 primary" % (W, H))
    out["traffic"] = pm.pop("hbm_bytes", None)
    out.update(pm)
    return out


def iteration_histogram(rt, frame):
    """TraverseBvh iterations of the frame's camera rays (rt_trace_primary detail: 1 spp, frame
    index `frame`): distribution, mean, max, and how many rays the scene cull settled (1 iteration)."""
    rt.trace_primary(frame, detail=True)
    rt.sync()
    hs = rt.download("HIT_STATS", np.uint32).reshape(-1, 4)
    it = hs[:, 3].astype(np.int64)
    edges = [1, 2, 8, 16, 32, 48, 64, 96, 128, 192, 256, 512, 1025]
    h, _ = np.histogram(it, bins=edges)
    return {"rays": int(it.size), "mean": round(float(it.mean()), 2), "p99": int(np.percentile(it, 99)),
            "max": int(it.max()), "dropped_pushes": int(hs[:, 2].sum()),
            "hist": {("%d" % a if b - a == 1 else "%d-%d" % (a, b - 1)): int(c) for a, b, c in zip(edges, edges[1:], h)}}


def time_draw(rtx, torch, dev, W, H, S, tmp, frames=20):
    """ms/frame of rt_draw_device, sync and async, BASELINE config 3 (fixed deltaTime)."""
    out = {}
    target = torch.empty((H, W, 4), dtype=torch.uint8, device=dev)
    for mode in ("sync", "async"):
        d = rtx.RayTracer(W, H, rtx.write_config(os.path.join(tmp, "draw_%s.toml" % mode), W, H, dynamic=False,
                                                 spp=S)).init()
        d.set_delta_time(DELTA_MS)
        asy = mode == "async"
        for _ in range(3):
            d.draw_device(target.data_ptr(), 0, asynchronous=asy)
        d.sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(frames):
            d.draw_device(target.data_ptr(), 0, asynchronous=asy)
        d.sync()
        torch.cuda.synchronize()
        out[mode + "_ms_per_frame"] = round((time.perf_counter() - t0) * 1e3 / frames, 4)
        d.cleanup()
    out["frames"] = frames
    return out


def self_check(rtx, W, H, S, tmp, last, final):
    """Serial re-render of frames 1..last in a fresh single-GPU context, compared with the timed
    sequence's last frame (RGBA8, final HDR, exposure state)."""
    ref = rtx.RayTracer(W, H, rtx.write_config(os.path.join(tmp, "check.toml"), W, H, dynamic=False, spp=S)).init()
    ref.set_delta_time(DELTA_MS)
    ref.set_stream(None)
    for f in range(1, last + 1):
        ref.build_bvh()
        ref.path_trace(f)
        ref.denoise_post(f)
    ref.sync()
    same = {"rgba8": bool(np.array_equal(ref.download("RGBA8", np.uint8), final["rgba"])),
            "hdr": bool(np.array_equal(ref.get_buffer("RENDER_COLOR"), final["color"])),
            "exposure": bool(np.array_equal(ref.download("EXPOSURE", np.uint8), final["exposure"]))}
    ref.cleanup()
    return dict(same, frames=last, against="serial single-GPU re-render of frames 1..%d" % last, ok=all(same.values()))


def extras_child(args):
    """The side measurements, in a process of their own (so that the timed process's rocprofv3 stats
    hold only the timed workload): traversal under load (the terrain camera, pipelined, with its own
    kernel split, work counters and camera-ray iteration histogram), serial stage and kernel times,
    rt_draw_device sync / async, the 1M-triangle LBVH rebuild (config 4), and the self-check."""
    import torch

    import rtx
    from rtx.frames import FramePipeline

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    W, H, S = args.width, args.height, args.spp
    tmp = tempfile.mkdtemp(prefix="rtxextras")
    out = {}
    cfg = rtx.write_config(os.path.join(tmp, "x.toml"), W, H, dynamic=False, chunk_dim=1, spp=S)
    rt = rtx.RayTracer(W, H, cfg).init()
    rt.set_delta_time(DELTA_MS)
    rt.build_bvh()
    out["camera_iterations_default_view"] = iteration_histogram(rt, 4)
    fp = FramePipeline(rt, dev, pipelined=True)
    cam = rt.camera
    cam.pos[:] = TERRAIN_CAM["pos"]
    cam.yaw, cam.pitch = TERRAIN_CAM["yaw"], TERRAIN_CAM["pitch"]
    rt.camera = cam
    for f in range(1, 4):
        fp.frame(f)
    fp.finish()
    rt.ray_count(reset=True)
    nt = 20
    rt.frame_marks_begin(nt, rtx.RayTracer.PT_KERNELS)
    torch.cuda.synchronize()
    ta = time.perf_counter()
    for k in range(nt):
        fp.frame(4 + k)
    fp.finish()
    torch.cuda.synchronize()
    tdt = time.perf_counter() - ta
    kms, _ = rt.frame_marks_read()
    trays = rt.ray_count()
    f = 4 + nt
    rt.path_trace(f, detail=True)
    q = rt.download("PT_QUEUE", np.uint32).copy()
    st = rt.download("PT_STATS", np.uint32).reshape(-1, 4).astype(np.uint64)
    rays_detail = int(st[:, 0].sum())
    per = kernel_roofline(q, W, H, S, kms, None, False)
    culled = int(q[22])
    out["terrain_camera"] = {
        "camera": TERRAIN_CAM, "frames": nt, "ms_per_frame": round(tdt * 1e3 / nt, 4),
        "mray_s": round(trays / tdt / 1e6, 2), "rays_per_frame": int(trays // nt),
        "mray_s_traversed": round(trays * (1.0 - culled / max(rays_detail, 1)) / tdt / 1e6, 2),
        "culled_camera_rays_per_frame": culled,
        "roofline": {"kernel": max((k for k in per if k != "k_pt_camera"), key=lambda k: per[k]["ms"]),
                     "kernels": per, "peak": L2_PEAK_GBS, "unit": "GB/s",
                     "timing": "HIP events around each kernel of the %d timed terrain frames" % nt},
        "camera_iterations": iteration_histogram(rt, f + 1)}
    rt.cleanup()
    # serial stages and kernels of the default view (rt_draw's mode: trace<3> .. resume<4> fused)
    sr = rtx.RayTracer(W, H, rtx.write_config(os.path.join(tmp, "s.toml"), W, H, dynamic=False, spp=S)).init()
    sr.set_delta_time(DELTA_MS)
    for f in range(1, 4):
        sr.build_bvh()
        sr.path_trace(f)
        sr.denoise_post(f)
    sr.sync()
    build_ms = sr.time_stage(0, 50) / 50
    out["lbvh_build_ms"] = round(build_ms, 5)
    out["lbvh_build_tris"] = int(sr.info().triCount)
    out["stage_ms_serial"] = {"lbvh_build": round(build_ms, 5), "path_trace": round(sr.time_stage(2, 20) / 20, 5),
                              "denoise_post": round(sr.time_stage(4, 20) / 20, 5),
                              "primary_rays_1spp": round(sr.time_stage(1, 20) / 20, 5)}
    out["primary_mray_s"] = round(W * H / (out["stage_ms_serial"]["primary_rays_1spp"] * 1e-3) / 1e6, 2)
    out["primary_roofline"] = primary_roofline(sr, W, H, out["stage_ms_serial"]["primary_rays_1spp"], 20)
    sk = sr.time_path_trace_kernels(20)
    names = list(sk)
    if all(sk[k] < 0.02 for k in names[3:6]):  # the fused chain k_pt_chain ran in kernel slot 2
        sk = {("k_pt_chain" if i == 2 else k): v for i, (k, v) in enumerate(sk.items()) if not 3 <= i <= 5}
    out["serial_kernels_ms"] = {k: round(v, 5) for k, v in sk.items()}
    out["serial_kernels_ms"]["sum"] = round(sum(sk.values()), 5)
    # the roofline of the path rt_draw runs (serial frames): the detail launch's work counters over
    # the serial kernel times; the fused chain carries the bytes of the four stages it runs
    sr.path_trace(4, detail=True)
    sq = sr.download("PT_QUEUE", np.uint32).copy()
    stages = ("k_trace_queue<3>", "k_pt_resume<3>", "k_trace_queue<4>", "k_pt_resume<4>")
    full = kernel_roofline(sq, W, H, S, {k: 1.0 for k in ("k_pt_camera", "k_pt_shade0", "k_pt_resolve") + stages},
                           None, False)
    ser = {}
    for k, ms in sk.items():
        b = sum(full[j]["algorithmic_bytes"] for j in stages) if k == "k_pt_chain" else full[k]["algorithmic_bytes"]
        a = b / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        ser[k] = {"ms": round(ms, 5), "algorithmic_bytes": int(b), "achieved_GBs": round(a, 1),
                  "frac_l2": round(a / L2_PEAK_GBS, 4)}
    out["serial_roofline"] = {"kernels": ser, "peak": L2_PEAK_GBS, "unit": "GB/s",
                              "kernel": max(ser, key=lambda k: ser[k]["ms"]),
                              "timing": "HIP events around each kernel of 20 serial frames (rt_time_path_trace_kernels)"}
    sr.cleanup()
    # the reference host's entry point, RayTracer::draw(SurfObj*) (kernel.cu:259): rt_draw_device into
    # a caller-owned device RGBA8 target, synchronous and asynchronous (RT_DRAW_ASYNC)
    out["draw_device"] = time_draw(rtx, torch, dev, W, H, S, tmp)
    # BASELINE config 4: per-frame rebuild of the ~1M-triangle variant (chunkDim 4)
    r4 = rtx.RayTracer(256, 144, rtx.write_config(os.path.join(tmp, "c4.toml"), 256, 144, chunk_dim=4)).init()
    r4.build_bvh()
    r4.sync()
    ms4 = r4.time_stage(0, 30) / 30
    n4 = r4.info().triCount
    r4.cleanup()
    a4 = 348 * n4 / (ms4 * 1e-3) / 1e9
    pm4 = pmc_c2c4("k_build_bvh@958720", "%d tris" % n4)
    out["lbvh_build_1m"] = {"tris": int(n4), "ms": round(ms4, 5),
                            "roofline": dict({"bound": "hbm", "achieved": round(a4, 2), "peak": HBM_PEAK_GBS,
                                              "unit": "GB/s", "frac": round(a4 / HBM_PEAK_GBS, 5),
                                              "traffic": pm4.pop("hbm_bytes", None), "bytes_per_tri": 348,
                                              "algorithmic_bytes": 348 * int(n4),
                                              "timing": "rt_time_stage(0, 30): HIP events around 30 builds"}, **pm4)}
    if args.check_file:
        fin = np.load(args.check_file)
        out["self_check"] = self_check(rtx, W, H, S, tmp, args.check_frames,
                                       {k: fin[k] for k in ("rgba", "color", "exposure")})
    print("EXTRAS " + json.dumps(out), flush=True)


def run_extras(args, check_file, check_frames):
    """extras_child in a fresh process (started before or after this one used the GPU: a child, not an
    exec); returns its JSON, or an error record."""
    import subprocess

    cmd = [sys.executable, os.path.abspath(__file__), "--extras-child", "--width", str(args.width), "--height",
           str(args.height), "--spp", str(args.spp)]
    if check_file:
        cmd += ["--check-file", check_file, "--check-frames", str(check_frames)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    for line in r.stdout.splitlines():
        if line.startswith("EXTRAS "):
            return json.loads(line[7:])
    return {"extras_error": "rc %d: %s" % (r.returncode, r.stderr[-2000:])}


def main():
    args = parse()
    if args.extras_child:
        return extras_child(args)
    import torch
    import torch.distributed as dist

    import rtx
    from rtx.dist import strip_blocks, strip_config
    from rtx.frames import FramePipeline

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
    fp = FramePipeline(rt, dev, pipelined=pipeline, world=world, rank=rank, backend=args.dist_backend)

    # warm-up; frames 2..W with every kernel (path trace and denoise / post) bracketed by HIP events
    # on its stream.  The stream whose kernels add up to the most time per frame binds the
    # pipelined frame (the denoise / post stream since round 4); the roofline's kernel
    # is that stream's longest.  Serial frames: every kernel is on the critical path.
    streams = stream_kernels(bool(rt.info().shadeOnSide)) if pipeline else {
        "serial": list(rtx.RayTracer.FRAME_KERNELS)}
    dom, bind, stream_ms, warm_ms = "k_trace_queue<3>", None, {}, {}
    if args.warmup >= 2:
        fp.frame(1)
        fp.finish()
        rt.frame_marks_begin(args.warmup - 1)
        for k in range(1, args.warmup):
            fp.frame(1 + k)
        fp.finish()
        warm_ms, _ = rt.frame_marks_read()
        stream_ms = {n: round(sum(warm_ms.get(k, 0.0) for k in ks), 5) for n, ks in streams.items()}
        bind = max(stream_ms, key=stream_ms.get)
        dom = max(streams[bind], key=lambda k: warm_ms.get(k, 0.0))
    else:
        for k in range(args.warmup):
            fp.frame(1 + k)
        fp.finish()
    rt.ray_count(reset=True)

    # ---- the timed region: K frames; that kernel is bracketed by HIP events on its stream in every
    # one of them (two events per frame: bracketing all seven kernels measured +2.4 % per frame)
    if not args.no_marks:
        rt.frame_marks_begin(args.steps, [dom])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        fp.frame(args.warmup + 1 + k)
    fp.finish()  # issues the last frame's deferred denoise/post and waits for every renderer stream
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    dt = t1 - t0
    kernels_ms, marked = rt.frame_marks_read() if not args.no_marks else (None, 0)
    rays = rt.ray_count()
    last = args.warmup + args.steps
    final = None
    if rank == 0 and not args.no_self_check:
        final = dict(rgba=rt.download("RGBA8", np.uint8).copy(), color=rt.get_buffer("RENDER_COLOR").copy(),
                     exposure=rt.download("EXPOSURE", np.uint8).copy())
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
        "config": {"workload": "BASELINE config %s: %dx%d, %d spp path trace + SVGF denoise + auto-exposure/"
                               "tone map, per-frame LBVH rebuild" % ("5" if (W, H) == (3840, 2160) else "3", W, H, S),
                   "width": W, "height": H, "spp": S,
                   "parallelism": ("interleaved 16-row strips x%d + RCCL all-to-all of the G-buffer rows each "
                                   "rank's strip-local denoise reads (64-row blocks + halo), histogram all-reduce "
                                   "and accumulation/history/RGBA8 row all-gathers" % world if world > 1
                                   else "single GPU")
                                  + ("; pipelined frames: denoise/post of f-1 and LBVH build + camera rays + "
                                     "shading of f+1 on their own streams beside the trace kernels of f" if pipeline
                                     else "; serial frames")},
        "fps": round(1000.0 / ms_per_step, 2),
        "rays_per_frame": int(rays // args.steps),
    }

    # ---- per-kernel roofline over this rank's strip: work counters of one detail launch (after the
    # timed frames), kernel durations from the timed frames' events; the denoise kernels' gating
    # statistics from the last timed frame (whole-frame denoise: one GPU)
    dst = denoise_stats(rt, W, H) if world == 1 else None
    rt.path_trace(last + 1, detail=True)
    st = rt.download("PT_STATS", np.uint32).reshape(-1, 4).astype(np.uint64)  # zero outside this rank's rows
    n_rays, visits, tests, diffuse = (int(st[:, k].sum()) for k in range(4))
    counters = rt.download("PT_QUEUE", np.uint32).copy()  # per-kernel work of this detail launch
    culled = int(counters[22])
    result["mray_s_traversed"] = round(value * (1.0 - culled / max(n_rays, 1)), 3)
    result["rays_traversed_fraction"] = round(1.0 - culled / max(n_rays, 1), 4)
    pmc = pmc_kernels()
    matches = pmc is not None and pmc.get("workload_key") == "%dx%dx%d" % (W, H, S) and world == 1
    if world > 1:  # what each rank receives per frame over the collectives (the G-buffer rows its
        # strip-local denoise reads, its peers' accumulation / history / RGBA8 rows, 256 B histogram)
        g = fp.gather.exchange_bytes_per_frame(fp.need) if fp.need else fp.gather.bytes_per_frame()
        r_ = fp.denoise.bytes_per_frame() if fp.denoise else 0
        result["comm_bytes_per_rank_per_frame"] = {"gbuffer_rows": int(g), "denoise_rows": int(r_),
                                                   "gbuffer_allgather_would_be": int(fp.gather.bytes_per_frame())}
    # the other kernels: the same split over 20 pipelined frames right after (every kernel marked).
    # One GPU only: rt_time_frame_kernels runs frames without FramePipeline's row exchanges, so on
    # a rank of N > 1 its denoise would read stale peer rows; ranks report the timed kernel alone.
    timed_dom = (kernels_ms or {}).get(dom)
    if world == 1:
        split = rt.time_frame_kernels(last + 2, 20)
        split_dom = split[dom]
    else:
        split, split_dom = {}, None
    if timed_dom is not None:
        split = dict(split, **{dom: timed_dom})
    per = kernel_roofline(counters, W, rows, S, split, pmc, matches)
    dn = denoise_roofline(dst, args.width, args.height, split, pmc, matches) if dst else {}
    stage_bytes = sum(e["algorithmic_bytes"] for e in per.values())
    stage_ms = sum(e["ms"] for e in per.values())
    d = per.get(dom) or dn[dom]
    on_l2 = dom in per
    peak = L2_PEAK_GBS if on_l2 else HBM_PEAK_GBS
    a = d["achieved_GBs"]
    vi = frame_valu_issue(list(per) + list(dn), ms_per_step, pmc, matches)
    result["roofline"] = {
        "bound": "l2" if on_l2 else "hbm", "limiter": "latency",
        "kernel": dom, "kernel_ms": d["ms"], "algorithmic_bytes": d["algorithmic_bytes"],
        "achieved": a, "peak": peak, "unit": "GB/s", "frac": round(a / peak, 4),
        "traffic": d.get("hbm_bytes"),
        "traffic_source": os.path.relpath(PMC_FILE, ROOT) if matches else None,
        "valu_busy_frac": d.get("valu_busy_frac"),
        "binding_stream": bind,
        "stream_kernel_ms": stream_ms,
        "note": ("kernel = the longest kernel of the stream that binds the frame: the stream whose kernels add up to "
                 "the most time per frame in the marked warm-up frames (stream_kernel_ms; pipelined: side = camera "
                 "rays + shade, context = the bounce / shadow queue chain, post = denoise + post).  "
                 + ("A path-trace kernel: BVH nodes, triangles and textures (~34 MB) stay in L2 / Infinity Cache, so "
                    "the memory ceiling is L2 bandwidth; it waits on dependent node loads (latency)." if on_l2 else
                    "A denoise / post kernel: algorithmic bytes are its compulsory G-buffer / colour traffic against "
                    "HBM; its time is the noise-gated tiles' stencil arithmetic and its waves' wait for issue slots "
                    "beside the next frame's path-trace waves (valu_busy_frac: share of wave time issuing VALU)")),
        "kernels": dict(per, **dn),
        "valu_issue": vi,
        # what binds the whole frame, as against the named kernel's memory roofline above
        "frame_limiter": ({"resource": "VALU issue", "frac": vi["frac"],
                           "note": "the frame's VALU wave-instructions at 4 cycles each on 1024 SIMDs need this share "
                                   "of ms_per_step (valu_issue); the memory rooflines of its kernels are far from peak"}
                          if vi and vi.get("frac") is not None else None),
        "denoise_gating": dst,
        "stage": {"kernels": " -> ".join(per), "algorithmic_bytes": stage_bytes, "sum_kernel_ms": round(stage_ms, 5),
                  "achieved_GBs": round(stage_bytes / (stage_ms * 1e-3) / 1e9, 1),
                  "frac_l2": round(stage_bytes / (stage_ms * 1e-3) / 1e9 / L2_PEAK_GBS, 4),
                  "rays": n_rays, "node_visits": visits, "tri_tests": tests, "diffuse_events": diffuse,
                  "hbm_bytes": pmc.get("stage_hbm_bytes") if matches else None},
        "timing": ("%s: HIP events right before / after it on the stream it runs on, in every one of the %d "
                   "timed frames (rt_frame_marks); chosen from warm-up frames 2..%d with every kernel marked; the "
                   "other kernels: the same events over 20 pipelined frames after the timed ones "
                   "(rt_time_frame_kernels); rocprofv3 --kernel-trace --stats of this command: "
                   "profiles/r06_kernel_stats.csv (this process: warm-up, timed, 1 detail and the 20 split frames)"
                   % (dom, marked, args.warmup)),
        "kernel_ms_split_frames": round(split_dom, 5) if split_dom is not None else None,
    }
    rt.cleanup()

    if rank == 0 and world == 1 and not args.no_extras:
        cf = None
        if final is not None:
            cf = os.path.join(tmp, "final.npz")
            np.savez(cf, **final)
        result.update(run_extras(args, cf, last))
    elif final is not None:
        result["self_check"] = self_check(rtx, W, H, S, tmp, last, final)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(W, H, S)
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()
    sc = result.get("self_check")
    if rank == 0 and sc is not None and not sc["ok"]:
        sys.exit("bench self-check failed: the timed frames differ from a serial re-render")


if __name__ == "__main__":
    main()
