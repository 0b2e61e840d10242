#!/usr/bin/env python3
"""GPU busy time and idle gaps per synchronous draw from a rocprofv3 --kernel-trace CSV of
tools/draw_probe.py sync: frames are delimited by the camera kernel (one per draw); prints the
union of kernel intervals per frame, the idle time inside it and the gap before each frame's
first kernel.  Usage: tools/sync_timeline.py <kernel_trace.csv> [first_frame] [frames]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
a = int(sys.argv[2]) if len(sys.argv) > 2 else 10
nf = int(sys.argv[3]) if len(sys.argv) > 3 else 10
cam = [i for i, r in enumerate(rows) if "k_pt_camera" in r["Kernel_Name"]]
for f in range(a, min(a + nf, len(cam) - 1)):
    seg = rows[cam[f]:cam[f + 1]]
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in seg)
    busy, cur_s, cur_e, idle, gaps = 0, iv[0][0], iv[0][1], 0, []
    for s, e, n in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, n.split("(")[0][-28:]))
            idle += s - cur_e
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    period = int(rows[cam[f + 1]]["Start_Timestamp"]) - iv[0][0]
    big = sorted(gaps, reverse=True)[:4]
    print("frame %d: period %.1f us, busy %.1f, idle %.1f; largest gaps before: %s" % (
        f, period / 1e3, busy / 1e3, idle / 1e3, ", ".join("%.1f %s" % (g / 1e3, n) for g, n in big)))
