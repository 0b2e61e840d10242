#!/usr/bin/env python3
"""Bounce-ray (queue 3 / queue 4) traversal profile of a bench frame: the iteration distribution,
SIMT efficiency per 64-ray wave and the queue tracer's kernel ms for several ray orders, through
rt_trace_rays on the rays the frame itself queued.  Tuning aid."""
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]


def main():
    import rtx

    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/q3"
    os.makedirs(out, exist_ok=True)
    W, H, S = 1920, 1080, 4
    cfg = rtx.write_config(os.path.join(tempfile.mkdtemp(), "q.toml"), W, H, spp=S)
    rt = rtx.RayTracer(W, H, cfg).init()
    rt.set_delta_time(16.667)
    # predictors from the previous frame (frame 2's queues, traced again: per pixel the longest
    # bounce / shadow ray) and from this frame's camera rays (per pixel TraverseBvh iterations, 1 spp)
    prev = {}
    for f in range(1, 4):
        rt.build_bvh()
        rt.path_trace(f)
        rt.sync()
        if f == 2:
            q2 = rt.download("PT_QUEUE", np.uint32)
            for step, (no, nd, cnt) in {3: ("PT_Q3_ORIGINS", "PT_Q3_DIRS", q2[0]),
                                        4: ("PT_Q4_ORIGINS", "PT_Q4_DIRS", q2[1])}.items():
                o4 = rt.download(no, np.float32).reshape(-1, 4)[:int(cnt)].copy()
                d2 = rt.download(nd, np.float32).reshape(-1, 4)[:int(cnt), :3].copy()
                it2 = rt.trace_rays(o4[:, :3].copy(), d2, want_iters=True)[4].astype(np.int64)
                pm = np.zeros(W * H, np.int64)
                np.maximum.at(pm, np.minimum(o4[:, 3].view(np.uint32).astype(np.int64), W * H - 1), it2)
                prev[step] = pm
        if f < 3:
            rt.denoise_post(f)
    q = rt.download("PT_QUEUE", np.uint32)
    rt.trace_primary(3, detail=True)
    rt.sync()
    cam_it = rt.download("HIT_STATS", np.uint32).reshape(-1, 4)[:, 3].astype(np.int64)
    res = {}
    for step, (no, nd, cnt) in {3: ("PT_Q3_ORIGINS", "PT_Q3_DIRS", q[0]), 4: ("PT_Q4_ORIGINS", "PT_Q4_DIRS", q[1])}.items():
        n = int(cnt)
        o4 = rt.download(no, np.float32).reshape(-1, 4)[:n].copy()
        o = o4[:, :3].copy()
        pix = o4[:, 3].view(np.uint32).astype(np.int64)
        d = rt.download(nd, np.float32).reshape(-1, 4)[:n, :3].copy()
        t, tri, u, v, it, _ = rt.trace_rays(o, d, want_iters=True)
        np.save(os.path.join(out, "q%d_iters.npy" % step), it)
        np.save(os.path.join(out, "q%d_rays.npy" % step), np.concatenate([o, d], 1))
        rng = np.random.default_rng(1)
        sh = rng.permutation(n)
        keyed = lambda k: sh[np.argsort(k[sh], kind="stable")]  # noqa: E731
        dy = d[:, 1]

        def front(mask):  # the flagged rays first, each group in queue order
            return np.concatenate([np.nonzero(mask)[0], np.nonzero(~mask)[0]])

        itq = it.astype(np.int64)
        camp = cam_it[np.minimum(pix, cam_it.size - 1)]
        orders = {"queue": np.arange(n), "shuffled": sh, "by_iters": np.argsort(-itq, kind="stable"),
                  # predictors available before tracing: the ray's y direction (grazing rays skim the terrain)
                  "dy_desc": keyed(-dy), "dy_clip": keyed(-np.minimum(dy, 0.2)),
                  "dy_bins8": keyed(-np.minimum(np.floor((dy + 1.0) * 4.0), 4.0)),
                  # a few rays moved to the front, the rest in queue order (keeps the append coherence)
                  "front_oracle_1pct": front(itq >= np.quantile(itq, 0.99)),
                  "front_oracle_5pct": front(itq >= np.quantile(itq, 0.95)),
                  "front_flat10": front(np.abs(dy) < 0.1), "front_flat05": front(np.abs(dy) < 0.05),
                  "front_cam5pct": front(camp >= np.quantile(camp, 0.95))}
        if step in prev:  # the previous frame's longest bounce ray of the same pixel
            pp = prev[step]
            pred = pp[np.minimum(pix, pp.size - 1)]
            orders["front_prev2pct"] = front(pred >= np.quantile(pred, 0.98))
            orders["front_prev5pct"] = front(pred >= np.quantile(pred, 0.95))
        r = dict(rays=n, iters_sum=int(it.sum()), iters_max=int(it.max()),
                 iters_q=[int(x) for x in np.quantile(it, [0.5, 0.9, 0.99, 0.999])])
        for name, ordr in orders.items():
            ii = it[ordr]
            pad = (-n) % 64
            wv = np.concatenate([ii, np.zeros(pad, ii.dtype)]).reshape(-1, 64)
            ms = min(rt.trace_rays(o[ordr], d[ordr])[-1] for _ in range(5))
            r[name] = dict(ms=round(ms, 4), simt_eff=round(float(ii.sum() / (wv.max(1).sum() * 64)), 4),
                           wave_max_sum=int(wv.max(1).sum()))
        res[step] = r
        print(step, json.dumps(r), flush=True)
    json.dump(res, open(os.path.join(out, "q_probe.json"), "w"), indent=1)
    rt.cleanup()


if __name__ == "__main__":
    main()
