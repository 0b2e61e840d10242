#!/usr/bin/env python3
"""Print a kernel timeline (µs from the first shown kernel) of frames a..b from a rocprofv3
--kernel-trace CSV.  Usage: tools/timeline.py <kernel_trace.csv> [first_frame] [frames]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
a = int(sys.argv[2]) if len(sys.argv) > 2 else 5
nf = int(sys.argv[3]) if len(sys.argv) > 3 else 2
idx = [i for i, r in enumerate(rows) if "k_build_bvh" in r["Kernel_Name"]]
start, end = idx[a], idx[min(a + nf, len(idx) - 1)]
t0 = int(rows[start]["Start_Timestamp"])
for r in rows[start:end]:
    s = (int(r["Start_Timestamp"]) - t0) / 1000
    e = (int(r["End_Timestamp"]) - t0) / 1000
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:30]
    print("%8.1f %8.1f %7.1f q%s %s" % (s, e, e - s, r["Queue_Id"], n))
print("frame period: %.1f us" % ((int(rows[end]["Start_Timestamp"]) - t0) / 1000 / nf))
