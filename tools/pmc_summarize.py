#!/usr/bin/env python3
"""HBM traffic of one path-trace stage launch from two rocprofv3 --pmc passes.

    python tools/pmc_summarize.py <fetch_dir> <write_dir> > profiles/rNN_pmc_pathtrace.json

Per kernel of the stage the median FETCH_SIZE / WRITE_SIZE per dispatch is taken (KB); the
stage's bytes are the sum over its kernels.  gfx950 correction (MI355X_MICROARCH.md, HBM
section): FETCH_SIZE counts half the bytes of wide reads, so it is doubled."""
import collections
import csv
import glob
import json
import statistics
import sys

STAGE = ("k_pt_camera", "k_pt_shade0", "k_trace_queue<3>", "k_pt_resume<3>", "k_trace_queue<4>",
         "k_pt_resume<4>", "k_pt_resolve")


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    return n.replace("<true>", "").replace("<false>", "")


def load(d, counter):
    per = collections.defaultdict(list)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return per


def main():
    fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    kernels = {}
    total = 0
    for k in STAGE:
        f = statistics.median(fetch[k]) if fetch.get(k) else None
        w = statistics.median(write[k]) if write.get(k) else None
        if f is None or w is None:
            raise SystemExit("kernel %s missing from the PMC output" % k)
        b = int(round((2.0 * f + w) * 1024))
        kernels[k] = {"FETCH_SIZE_KB_median": f, "WRITE_SIZE_KB_median": w, "hbm_bytes": b,
                      "dispatches": len(fetch[k])}
        total += b
    print(json.dumps({
        "kernel": "path-trace stage: " + " -> ".join(STAGE),
        "workload": "bench.py default: 1920x1080, 4 spp, default scene/camera (rocprofv3 --pmc runs of "
                    "`bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras`)",
        "correction": "MI355X_MICROARCH.md HBM section: FETCH_SIZE reports half the bytes of wide reads on gfx950 "
                      "-> doubled; KB -> bytes x1024; separate --pmc passes for FETCH_SIZE and WRITE_SIZE",
        "kernels": kernels,
        "hbm_bytes_per_launch": total,
        "note": "BVH nodes/triangles and textures stay L2/MALL resident; the algorithmic bytes in bench.py count "
                "every node/triangle/texel read, so traffic << algorithmic bytes",
    }, indent=1))


if __name__ == "__main__":
    main()
