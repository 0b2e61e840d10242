#!/usr/bin/env python3
"""Per-kernel PMC summary of the bench workload from separate rocprofv3 --pmc passes.

    python tools/pmc_r02.py <out.json> <pass_dir>...

Each pass directory holds one `rocprofv3 --pmc ... --kernel-trace --output-format csv` run of
`bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-self-check` (pipelined frames,
1920x1080, 4 spp).  Per kernel the median per-dispatch value of every counter is taken, then:
  hbm_bytes          = (2 * FETCH_SIZE + WRITE_SIZE) * 1024   (KB; FETCH_SIZE counts half the bytes
                       of wide reads on gfx950: MI355X_MICROARCH.md HBM section)
  l2_hit_rate        = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)  (MI355X_MICROARCH.md L2 section)
  wait_inst_any_frac = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES  (share of wave time waiting to issue)
  valu_busy_frac     = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES"""
import collections
import re
import csv
import glob
import json
import statistics
import sys

STAGE = ("k_pt_camera", "k_pt_shade0", "k_trace_queue<3>", "k_pt_resume<3>", "k_trace_queue<4>",
         "k_pt_resume<4>", "k_pt_resolve")


def short(name):
    """Stage name of a kernel symbol: the boolean template arguments (material-table variants)
    dropped, the queue step kept: k_pt_shade0<false, false> -> k_pt_shade0, k_pt_resume<3, false>
    -> k_pt_resume<3>."""
    n = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    n = re.sub(r"<(\d+)(, (true|false))+>", r"<\1>", n)
    return re.sub(r"<(true|false)(, (true|false))*>", "", n)


def main():
    out_path, dirs = sys.argv[1], sys.argv[2:]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            per = collections.defaultdict(lambda: collections.defaultdict(float))
            for r in csv.DictReader(open(f)):
                per[(short(r["Kernel_Name"]), r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
            for (k, _), c in per.items():
                for n, v in c.items():
                    vals[k][n].append(v)
    kernels = {}
    stage_hbm = 0
    for k in STAGE:
        c = {n: statistics.median(v) for n, v in vals.get(k, {}).items()}
        e = {"counters_median": c, "dispatches": max((len(v) for v in vals.get(k, {}).values()), default=0)}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["hbm_bytes"] = int(round((2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024))
            stage_hbm += e["hbm_bytes"]
        hit, miss = c.get("TCC_HIT_sum", c.get("TCC_HIT")), c.get("TCC_MISS_sum", c.get("TCC_MISS"))
        if hit is not None and miss is not None and hit + miss > 0:
            e["l2_hit_rate"] = round(hit / (hit + miss), 4)
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            if "SQ_WAIT_INST_ANY" in c:
                e["wait_inst_any_frac"] = round(c["SQ_WAIT_INST_ANY"] / wc, 4)
            if "SQ_ACTIVE_INST_VALU" in c:
                e["valu_busy_frac"] = round(c["SQ_ACTIVE_INST_VALU"] / wc, 4)
        kernels[k] = e
    res = {"workload_key": "1920x1080x4",
           "workload": "bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-self-check "
                       "(1920x1080, 4 spp, default scene/camera, pipelined frames)",
           "passes": dirs, "kernels": kernels, "stage_hbm_bytes": stage_hbm,
           "correction": "FETCH_SIZE doubled (gfx950 counts half the bytes of wide reads), KB x 1024",
           "note": "every counter from its own rocprofv3 --pmc run; medians over all dispatches of the kernel"}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: {f: v for f, v in e.items() if f != "counters_median"} for k, e in kernels.items()}, indent=1))


if __name__ == "__main__":
    main()
