#!/usr/bin/env python3
"""Per-launch PMC summary of BASELINE configs 2 and 4 (tools/c2c4_probe.py) from separate
rocprofv3 --pmc passes.

    python tools/pmc_c2c4.py <out.json> <pass_dir>...

Kernels: k_trace_primary (config 2, 1920x1080 1 spp: one launch = 2,073,600 rays) and k_build_bvh
at 937 workgroups (config 4, 958,720 triangles; the probe's other build, the 60,800-triangle init
build, has 60).  Per kernel the median per-dispatch value of every counter is taken, then
(MI355X_MICROARCH.md HBM and L2 sections):
  hbm_bytes   = (2 * FETCH_SIZE + WRITE_SIZE) * 1024   (FETCH_SIZE in KB counts half the bytes of
                wide reads on gfx950, so it is doubled; WRITE_SIZE in KB)
  l2_hit_rate = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)"""
import collections
import csv
import glob
import json
import statistics
import sys


def label(row):
    name = row["Kernel_Name"]
    grid = int(row.get("Grid_Size", row.get("Grid_Size_X", "0")) or 0)
    wg = int(row.get("Workgroup_Size", row.get("Workgroup_Size_X", "0")) or 0)
    if "k_trace_primary" in name:
        return "k_trace_primary"
    if "k_build_bvh" in name:
        blocks = grid // wg if wg else 0
        # 937 batch workgroups (+ the TLAS workgroup since round 4)
        return "k_build_bvh@958720" if blocks in (937, 938) else "k_build_bvh@%dwg" % blocks
    return None


def main():
    out_path, dirs = sys.argv[1], sys.argv[2:]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            per = collections.defaultdict(lambda: collections.defaultdict(float))
            for r in csv.DictReader(open(f)):
                k = label(r)
                if k:
                    per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
            for (k, _), c in per.items():
                for n, v in c.items():
                    vals[k][n].append(v)
    kernels = {}
    for k, cv in sorted(vals.items()):
        c = {n: statistics.median(v) for n, v in cv.items()}
        e = {"counters_median": c, "dispatches": max(len(v) for v in cv.values())}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["hbm_bytes"] = int(round((2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024))
            e["fetch_bytes_doubled"] = int(round(2.0 * c["FETCH_SIZE"] * 1024))
            e["write_bytes"] = int(round(c["WRITE_SIZE"] * 1024))
        hit, miss = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
        if hit is not None and miss is not None and hit + miss > 0:
            e["l2_hit_rate"] = round(hit / (hit + miss), 4)
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n, f in (("SQ_WAIT_INST_ANY", "wait_inst_any_frac"), ("SQ_ACTIVE_INST_VALU", "valu_busy_frac"),
                         ("SQ_WAIT_ANY", "wait_any_frac")):
                if n in c:
                    e[f] = round(c[n] / wc, 4)
        kernels[k] = e
    res = {"workload_key": {"k_trace_primary": "1920x1080x1 primary", "k_build_bvh@958720": "958720 tris"},
           "workload": "tools/c2c4_probe.py (config 2: rt_time_stage(1, N) at 1920x1080; config 4: "
                       "rt_time_stage(0, N) on the chunkDim-4 scene)",
           "passes": dirs, "kernels": kernels,
           "correction": "FETCH_SIZE doubled (gfx950 counts half the bytes of wide reads), KB x 1024",
           "note": "every counter from its own rocprofv3 --pmc run; medians over all dispatches of the kernel"}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: {f: v for f, v in e.items() if f != "counters_median"} for k, e in kernels.items()},
                     indent=1))


if __name__ == "__main__":
    main()
