#!/usr/bin/env python3
"""Regenerate tests/golden/golden.json from the CPU oracle (oracle/_build/liboracle.so).

Two kinds of content:
  * "survey_pins": known answers SURVEY.md recorded from the reference's own code and its
    scene analysis (SURVEY.md §0 #3, #8, #8c, §8 a4/c).  These pin the oracle to the
    reference; they are typed in from SURVEY.md, not computed here.
  * "oracle": SHA-256 digests of oracle outputs on the default scene, so any change in the
    restatement (or its inputs) is caught.  Regenerate only on an intended change.
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402


def hit_core(h):
    """The 76-byte OrcHit prefix the digests were taken on (fields added later are excluded)."""
    return np.ascontiguousarray(h).view(np.uint8).reshape(len(h), -1)[:, :76]


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def valid_nodes(b):
    B, n = b["batch_count"], b["tri_count"]
    parts = []
    for k in range(B):
        cnt = 1024 if k < B - 1 else n - (B - 1) * 1024
        parts.append(b["nodes"][k * 1024:k * 1024 + cnt - 1])
    return np.concatenate(parts)


def main():
    out = {
        "survey_pins": {
            "morton3_1023_0_0": 0x09249249,
            "default": {"triCount": 60800, "batchCount": 60, "lastBatch": 384, "dupKeys": 0,
                        "blasDepthMinMedMax": [10, 15, 17], "tlasDepth": 10},
            "chunk4": {"triCount": 958720, "batchCount": 937, "lastBatch": 256, "dupKeys": 0,
                       "blasDepthMinMedMax": [9, 16, 19], "tlasDepth": 16,
                       "quirkBoxMaxXY": [62.5, 13.0], "trueBoxMaxXY": [64.5, 14.0], "tlasCentresOutside": 28},
            # the reference's own TraverseBvh on a 2-triangle BLAS + 1-leaf TLAS
            # (the B == 1 special case, buildBVH.cuh:31-38) and its RayTriangleIntersect probe
            # (geometry.cuh:474-495), as printed there
            "traverse_probe": {"objectIdx": 1, "t": 2.99999952, "u": 0.6, "v": 0.2, "geometricNormal": [0, 0, 1]},
            "triangle_probe": {"t": 1.0, "u": 0.6, "v": 0.2},
        },
        "oracle": {},
    }
    for cd, key in ((1, "default"), (4, "chunk4")):
        v, i, n = O.scene(cd)
        nrm = O.smooth_normals(v, i)
        b = O.build_bvh(v, i, n, nrm)
        ent = {"triCount": n, "triCountPadded": int(i.shape[0]), "vertexCount": int(v.shape[0]),
               "vertices_sha256": sha(v), "indices_sha256": sha(i), "normals_sha256": sha(nrm),
               "morton_sha256": sha(b["morton"]), "reorder_sha256": sha(b["reorder"]),
               "nodes_sha256": sha(valid_nodes(b)), "tlas_morton_sha256": sha(b["tlas_morton"]),
               "tlas_nodes_sha256": sha(b["tlas_nodes"])}
        if cd == 1:
            rays, _ = O.primary_rays(64, 64, 1)
            hits = O.intersect(b, rays)
            ent["primary64_rays_sha256"] = sha(rays)
            ent["primary64_hits_sha256"] = sha(hit_core(hits))
        out["oracle"][key] = ent
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out["oracle"], indent=1))


if __name__ == "__main__":
    main()
