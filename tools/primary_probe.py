#!/usr/bin/env python3
"""Primary rays through the persistent queue tracer: the default view's 1080p x 4 spp camera
rays (oracle.primary_rays, frame indices 1..4) minus the ones the scene cull settles, in 8x8-tile
order (as a camera kernel would queue them) and shuffled, traced with rt_trace_rays.  Tuning aid:
the cost of moving the camera kernel's inline traversal into the queue tracer."""
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]


def main():
    import rtx
    from oracle import oracle

    W, H = 1920, 1080
    cfg = rtx.write_config(os.path.join(tempfile.mkdtemp(), "p.toml"), W, H, spp=4)
    rt = rtx.RayTracer(W, H, cfg).init()
    rt.build_bvh()
    rt.sync()
    box = rt.download("TLAS_SCENE_AABB", np.float32)[:6].astype(np.float32)
    mn, mx = box[:3], box[3:]
    m = np.float32(0.01) * np.max(mx - mn) + np.float32(0.01)
    sets = []
    for s in range(4):
        rays, _ = oracle.primary_rays(W, H, frame_num=1 + s)
        o, d = rays[:, :3], rays[:, 3:]
        with np.errstate(divide="ignore", invalid="ignore"):
            inv = np.float32(1.0) / d
            a = (mn - m - o) * inv
            b = (mx + m - o) * inv
        tn = np.max(np.minimum(a, b), 1)
        tf = np.min(np.maximum(a, b), 1)
        keep = (tn <= tf) & (tf > 0)
        # 8x8 tile order of the pixels, sample-major within a tile group (camera wave order)
        idx = np.arange(W * H).reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1)
        idx = idx[keep[idx]]
        sets.append((o[idx], d[idx]))
    o = np.concatenate([x[0] for x in sets])
    d = np.concatenate([x[1] for x in sets])
    n = len(o)
    res = dict(rays=n, of_samples=4 * W * H)
    t, tri, u, v, it, _ = rt.trace_rays(o, d, want_iters=True)
    res["iters_sum"] = int(it.sum())
    res["hit_fraction"] = float((tri >= 0).mean())
    rng = np.random.default_rng(2)
    perm = rng.permutation(n)
    res["tile_order_ms"] = min(rt.trace_rays(o, d)[-1] for _ in range(5))
    res["shuffled_ms"] = min(rt.trace_rays(o[perm], d[perm])[-1] for _ in range(3))
    print(json.dumps(res), flush=True)
    rt.cleanup()


if __name__ == "__main__":
    main()
