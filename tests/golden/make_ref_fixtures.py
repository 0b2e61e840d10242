#!/usr/bin/env python3
"""Regenerates the reference-run fixtures under tests/golden/ (run here, where /root/reference is
present; the GPU box and the tests only read the committed outputs).

1. Builds oracle/_ref/ from the reference's own standalone sources (oracle/ref/Makefile: perlin.h,
   settingParams.h, skyData.h compiled with plain g++ where they lie) and records their output:
     ref_perlin.bin     perlin_dump: [20480][3] float32 inputs, then [20480] Perlin::noise3D values
                        (the kChunkDim = 8 terrain lattice of Chunk::Generate, then scattered points)
     ref_settings.json  settings_dump: the default SkyParams .. DenoisingParams member values
     sky table digest   skydata_dump: the tables in data/sky_tables.bin's layout (sha256 only: the
                        shipped file must equal it byte for byte)
2. Records the denoiser's precomputed Gaussian tables, gaussian.cuh:12-43 (GetGaussian3x3 / 5x5 /
   7x7 under USE_PRECALCULATED_GAUSSIAN 1): each literal as written and as the float it becomes
   (ref_gaussian.json).  Data read from the header's text, not source.
3. Records the reference's only meshProcessor scene, resources/models/test.bin: its size, sha256,
   header count and first 64 records (64 B each, ref_test_bin_head.bin).  Data, not source.
Writes ref_fixtures.json with the sha256 of every output and the commands that made them."""
import hashlib
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
OUT = os.path.join(ROOT, "oracle", "_ref")


def sha(b):
    return hashlib.sha256(b).hexdigest()


def gaussian_tables(text):
    """The three precomputed tables of gaussian.cuh (float arrays cGaussian3x3 / 5x5 / 7x7 inside the
    USE_PRECALCULATED_GAUSSIAN branch): literal tokens and their float32 values (bit patterns)."""
    import re
    import struct
    out = {}
    for n in (3, 5, 7):
        m = re.search(r"float\s+cGaussian%dx%d\[\]\s*=\s*\{(.*?)\}" % (n, n), text, re.S)
        toks = [t for t in re.split(r"[\s,]+", m.group(1)) if t]
        assert len(toks) == n * n, (n, len(toks))
        bits = [struct.unpack("<I", struct.pack("<f", float(t)))[0] for t in toks]
        out["%dx%d" % (n, n)] = {"literals": toks, "float32_bits": bits}
    return out


def main():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle", "ref"), "REF=%s/src" % REF], check=True)
    man = {"generator": "tests/golden/make_ref_fixtures.py", "reference": REF}
    perlin = subprocess.run([os.path.join(OUT, "perlin_dump")], check=True, capture_output=True).stdout
    open(os.path.join(HERE, "ref_perlin.bin"), "wb").write(perlin)
    man["ref_perlin.bin"] = {"sha256": sha(perlin), "bytes": len(perlin), "points": len(perlin) // 16,
                             "lattice_points": 16384, "command": "oracle/_ref/perlin_dump",
                             "source": "src/perlin.h:50-78 (Perlin::noise3D), lattice of src/terrain.cpp:5-17"}
    settings = subprocess.run([os.path.join(OUT, "settings_dump")], check=True, capture_output=True).stdout
    json.loads(settings)
    open(os.path.join(HERE, "ref_settings.json"), "wb").write(settings)
    man["ref_settings.json"] = {"sha256": sha(settings), "command": "oracle/_ref/settings_dump",
                                "source": "src/settingParams.h:26-157"}
    sky = subprocess.run([os.path.join(OUT, "skydata_dump")], check=True, capture_output=True).stdout
    man["sky_tables"] = {"sha256": sha(sky), "bytes": len(sky), "command": "oracle/_ref/skydata_dump",
                         "source": "src/skyData.h:2-174", "compare": "real-time-ray-tracing_amd/data/sky_tables.bin"}
    g = gaussian_tables(open(os.path.join(REF, "src", "gaussian.cuh")).read())
    gj = (json.dumps(g, indent=1, sort_keys=True) + "\n").encode()
    open(os.path.join(HERE, "ref_gaussian.json"), "wb").write(gj)
    man["ref_gaussian.json"] = {"sha256": sha(gj), "command": "tests/golden/make_ref_fixtures.py gaussian_tables",
                                "source": "src/gaussian.cuh:12-43"}
    tb = open(os.path.join(REF, "resources", "models", "test.bin"), "rb").read()
    head = tb[4:4 + 64 * 64]
    open(os.path.join(HERE, "ref_test_bin_head.bin"), "wb").write(head)
    man["test.bin"] = {"sha256": sha(tb), "bytes": len(tb), "count": int.from_bytes(tb[:4], "little"),
                       "record_bytes": (len(tb) - 4) // int.from_bytes(tb[:4], "little"),
                       "head_file": "ref_test_bin_head.bin", "head_sha256": sha(head),
                       "source": "resources/models/test.bin"}
    with open(os.path.join(HERE, "ref_fixtures.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
        f.write("\n")
    print(json.dumps(man, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
