#!/usr/bin/env python3
"""LBVH build ms of both scene sizes (BASELINE configs 3 and 4), best of several 30-build
batches, for the library RTX_LIB names (ablation builds of bvh_build.hip)."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]


def main():
    import torch  # noqa: F401  (one HIP runtime: torch's)
    import rtx
    tmp = tempfile.mkdtemp()
    out = []
    for cd in (1, 4):
        cfg = rtx.write_config(os.path.join(tmp, "c%d.toml" % cd), 256, 144, chunk_dim=cd)
        rt = rtx.RayTracer(256, 144, cfg).init()
        rt.build_bvh()
        rt.sync()
        best = min(rt.time_stage(0, 30) / 30 for _ in range(5))
        out.append("%d tris %.4f ms" % (rt.info().triCount, best))
        rt.cleanup()
    print(os.environ.get("RTX_LIB", "lib"), " | ".join(out))


if __name__ == "__main__":
    main()
