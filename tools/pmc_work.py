#!/usr/bin/env python3
"""Per-kernel work counters (mean per dispatch) from rocprofv3 --pmc CSV directories.

    python tools/pmc_work.py <dir> [<dir> ...]

Prints one row per kernel: dispatches and the mean of every SQ counter found, plus the VALU
issue share of one frame (SQ_INSTS_VALU summed over the frame's kernels)."""
import collections
import csv
import glob
import json
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    return n.strip()


def main():
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in vals.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[k]["dispatches"] = max(len(v) for v in cs.values())
    tot = sum(v.get("SQ_INSTS_VALU", 0.0) * 1.0 for v in out.values())
    for k in sorted(out, key=lambda k: -out[k].get("SQ_INSTS_VALU", 0.0)):
        v = out[k]
        print("%-40s n=%4d %s" % (k[:40], v["dispatches"], " ".join(
            "%s=%.3g" % (c.replace("SQ_", ""), x) for c, x in sorted(v.items()) if c != "dispatches")))
    print(json.dumps({"valu_total_mean_per_dispatch_sum": tot}))


if __name__ == "__main__":
    main()
