#!/usr/bin/env python3
"""Per-kernel ms of one librtx build (RTX_LIB selects it): pipelined frames as bench.py runs them,
the path-trace kernels timed in-pipeline, the denoise/post chain timed serially.  Ablation aid."""
import json
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

    W, H, S = 1920, 1080, 4
    cfg = rtx.write_config(os.path.join(tempfile.mkdtemp(), "a.toml"), W, H, spp=S)
    rt = rtx.RayTracer(W, H, cfg).init()
    rt.set_delta_time(16.667)
    dev = torch.device("cuda", 0)
    prm = rt.params
    for k in os.environ.get("ABL_OFF", "").split(","):  # e.g. enableSharpening,enableToneMapping
        if k:
            setattr(prm.pass_, k, 0)
    rt.params = prm
    fp = FramePipeline(rt, dev)
    if os.environ.get("ABL_NO_DENOISE"):
        fp.rt.denoise_post = lambda f, hdr=False: None
    for f in range(1, 4):
        fp.frame(f)
    fp.finish()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for f in range(4, 34):
        fp.frame(f)
    fp.finish()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / 30
    k = rt.time_frame_kernels(40, 20)
    dn = rt.time_stage(4, 20) / 20
    print(json.dumps({"lib": os.environ.get("RTX_LIB", "default"), "off": os.environ.get("ABL_OFF", ""),
                      "no_denoise": bool(os.environ.get("ABL_NO_DENOISE")), "ms_frame": round(ms, 4),
                      "kernels": {a: round(b, 4) for a, b in k.items()}, "denoise_serial": round(dn, 4)}))
    rt.cleanup()


if __name__ == "__main__":
    main()
