#!/usr/bin/env python3
"""Convert the reference's *data* inputs into compact binary fixtures.

Runs only in the survey/build container (needs /root/reference).  Nothing it
produces is source code: it emits number tables and triangle soups that the
hot path consumes as inputs, with a SHA-256 manifest.

Outputs (real-time-ray-tracing_amd/data/):
  roundcubes_l2.bin   the 15 level-2 marching-cube tiles loaded by
                      marchingCubes.cpp:216-225 (resources/models/roundcubes/2),
                      triangulated the way assimp's aiProcess_Triangulate does
                      (fileUtils.cu:61-80).  Layout: u32 tileCount, then per tile
                      u32 triCount + float32[triCount][3][3] (positions only;
                      VoxelToMesh(vertices, indices) never reads normals).
  bluenoise_4spp.bin  Heitz 2019 tables for OPTIMIZED_BLUE_NOISE_SPP == 4
                      (blueNoiseRandGenData.h:15-39): sobol[256*256],
                      scrambling[128*128*8], ranking[128*128*8], u8 each.
  sky_tables.bin      float32 tables of skyData.h:2-174 (Hosek-Wilkie datasets,
                      solar radiance, limb darkening, CIE XYZ matching curves),
                      preceded by a small header (u32 count, then per table
                      u32 length).

The OBJ float parse follows assimp's fast_atoreal_move: integer part as float,
fraction as double(int(digits)) * 10^-ndigits rounded to float and added.
"""
import hashlib
import json
import math
import os
import re
import struct
import sys

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "real-time-ray-tracing_amd", "data")

# assimp fast_atof_table (double literals)
_ATOF_TABLE = [0.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001, 0.00000001,
               0.000000001, 0.0000000001, 0.00000000001, 0.000000000001,
               0.0000000000001, 0.00000000000001, 0.000000000000001]


def assimp_atof(tok: str) -> np.float32:
    s = tok
    neg = s.startswith("-")
    if neg or s.startswith("+"):
        s = s[1:]
    m = re.fullmatch(r"(\d*)(?:\.(\d+))?", s)
    if m is None:
        raise ValueError("unsupported float token %r" % tok)
    ip, fp = m.group(1), m.group(2)
    f = np.float32(int(ip)) if ip else np.float32(0.0)
    if fp:
        digits = fp[:15]
        pl = float(int(digits)) * _ATOF_TABLE[len(digits)]
        f = np.float32(f + np.float32(pl))
    if neg:
        f = np.float32(-f)
    return f


def _normalize(v):
    l = np.float32(np.sqrt(np.float32(np.float32(v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])))
    if l == 0:
        return v
    inv = np.float32(np.float32(1.0) / l)
    return np.array([v[0] * inv, v[1] * inv, v[2] * inv], dtype=np.float32)


def triangulate_quad(verts):
    """assimp TriangulateProcess, quad branch: fan from the concave vertex if any."""
    start = 0
    margins = []
    for i in range(4):
        v0 = verts[(i + 3) % 4]
        v1 = verts[(i + 2) % 4]
        v2 = verts[(i + 1) % 4]
        v = verts[i]
        left = _normalize((v0 - v).astype(np.float32))
        diag = _normalize((v1 - v).astype(np.float32))
        right = _normalize((v2 - v).astype(np.float32))
        dl = np.float32(np.float32(left[0] * diag[0] + left[1] * diag[1]) + left[2] * diag[2])
        dr = np.float32(np.float32(right[0] * diag[0] + right[1] * diag[1]) + right[2] * diag[2])
        angle = np.float32(np.arccos(np.float32(np.clip(dl, -1, 1))) + np.arccos(np.float32(np.clip(dr, -1, 1))))
        margins.append(abs(float(angle) - math.pi))
        if angle > np.float32(math.pi):
            start = i
            break
    t = [(start, start + 1, start + 2), (start, start + 2, start + 3)]
    return [tuple(verts[k % 4] for k in tri) for tri in t], start, min(margins)


def load_obj(path):
    vs = []
    tris = []
    starts = []
    min_margin = 1e9
    with open(path) as f:
        for line in f:
            p = line.split()
            if not p:
                continue
            if p[0] == "v":
                vs.append(np.array([assimp_atof(p[1]), assimp_atof(p[2]), assimp_atof(p[3])], dtype=np.float32))
            elif p[0] == "f":
                idx = [int(x.split("/")[0]) - 1 for x in p[1:]]
                if len(idx) == 3:
                    tris.append(tuple(vs[i] for i in idx))
                elif len(idx) == 4:
                    t, s, mg = triangulate_quad([vs[i] for i in idx])
                    starts.append(s)
                    min_margin = min(min_margin, mg)
                    tris.extend(t)
                else:
                    raise ValueError("polygon with %d corners not supported" % len(idx))
    return tris, starts, min_margin


def c_array(text, name):
    m = re.search(re.escape(name) + r"\s*\[[^\]]*\]\s*=\s*\{(.*?)\}", text, re.S)
    if m is None:
        raise KeyError(name)
    body = re.sub(r"//[^\n]*", "", m.group(1))
    return [t for t in re.split(r"[\s,]+", body) if t]


def extract(out_dir=OUT):
    """Writes the three data files into out_dir and returns their manifest (MANIFEST.json's content)."""
    os.makedirs(out_dir, exist_ok=True)
    manifest = {}

    # ---- tiles -------------------------------------------------------------
    blob = bytearray(struct.pack("<I", 15))
    report = {}
    for k in range(1, 16):
        tris, starts, margin = load_obj(os.path.join(REF, "resources/models/roundcubes/2/%d.obj" % k))
        arr = np.array(tris, dtype=np.float32).reshape(-1, 3, 3)
        blob += struct.pack("<I", arr.shape[0]) + arr.tobytes()
        report[k] = {"tris": int(arr.shape[0]), "nonzero_fan_start": int(sum(1 for s in starts if s)),
                     "min_|anglesum-pi|": round(margin, 6)}
    path = os.path.join(out_dir, "roundcubes_l2.bin")
    open(path, "wb").write(bytes(blob))
    manifest["roundcubes_l2.bin"] = {"sha256": hashlib.sha256(bytes(blob)).hexdigest(),
                                     "source": "resources/models/roundcubes/2/{1..15}.obj",
                                     "tiles": report}

    # ---- blue noise ---------------------------------------------------------
    text = open(os.path.join(REF, "src/blueNoiseRandGenData.h")).read()
    sec = text[text.index("#if OPTIMIZED_BLUE_NOISE_SPP == 4"):]
    sob = np.array([int(x) for x in c_array(sec, "h_sobol_256spp_256d")], dtype=np.uint8)
    scr = np.array([int(x) for x in c_array(sec, "h_scramblingTile")], dtype=np.uint8)
    rnk = np.array([int(x) for x in c_array(sec, "h_rankingTile")], dtype=np.uint8)
    assert sob.size == 256 * 256 and scr.size == 128 * 128 * 8 and rnk.size == 128 * 128 * 8
    blob = sob.tobytes() + scr.tobytes() + rnk.tobytes()
    path = os.path.join(out_dir, "bluenoise_4spp.bin")
    open(path, "wb").write(blob)
    manifest["bluenoise_4spp.bin"] = {"sha256": hashlib.sha256(blob).hexdigest(),
                                      "source": "src/blueNoiseRandGenData.h (OPTIMIZED_BLUE_NOISE_SPP==4)"}

    # ---- sky tables ---------------------------------------------------------
    text = open(os.path.join(REF, "src/skyData.h")).read()
    names = ["skyDataSets", "skyDataSetsRad", "h_solarDatasets", "h_limbDarkeningDatasets",
             "spectrumCieX", "spectrumCieY", "spectrumCieZ"]
    tables = []
    for n in names:
        vals = np.array([float(x.rstrip("fF")) for x in c_array(text, n)], dtype=np.float32)
        tables.append(vals)
    blob = struct.pack("<I", len(tables)) + b"".join(struct.pack("<I", t.size) for t in tables)
    blob += b"".join(t.tobytes() for t in tables)
    path = os.path.join(out_dir, "sky_tables.bin")
    open(path, "wb").write(blob)
    manifest["sky_tables.bin"] = {"sha256": hashlib.sha256(blob).hexdigest(), "source": "src/skyData.h",
                                  "tables": {n: int(t.size) for n, t in zip(names, tables)}}

    return manifest


def main():
    manifest = extract(OUT)
    json.dump(manifest, open(os.path.join(OUT, "MANIFEST.json"), "w"), indent=1, sort_keys=True)
    json.dump(manifest, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
