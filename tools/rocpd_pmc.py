#!/usr/bin/env python3
"""Per-kernel PMC summary from a rocprofv3 --pmc SQLite result: dispatches, mean duration, VGPRs,
waves, VALU instructions per wave, wave cycles per wave (quad-cycles x4), VALU-busy share, and any
other counters as per-dispatch means.  Usage: rocpd_pmc.py results.db [name-filter]"""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
d = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(dict)
for n, did, cn, v, dur, vg in c.execute(
        "select kernel_name, dispatch_id, counter_name, value, duration, vgpr_count from counters_collection"):
    k = n.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    if flt not in k:
        continue
    d[k][cn] += v
    disp[k][did] = (dur, vg)
for k, v in sorted(d.items(), key=lambda kv: -sum(x[0] for x in disp[kv[0]].values())):
    nd = len(disp[k])
    dur = sum(x[0] for x in disp[k].values()) / nd / 1e3
    vg = max(x[1] for x in disp[k].values())
    w = v.get("SQ_WAVES", 0)
    s = "%-34s n=%4d %8.2f us vgpr=%3d" % (k[:34], nd, dur, vg)
    if w:
        s += " waves/d=%7.0f" % (w / nd)
        if "SQ_INSTS_VALU" in v:
            s += " valu/wave=%6.0f" % (v["SQ_INSTS_VALU"] / w)
        if "SQ_WAVE_CYCLES" in v:
            s += " cyc/wave=%7.0f" % (4 * v["SQ_WAVE_CYCLES"] / w)
        for extra in ("SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU"):
            if extra in v:
                s += " %s/wave=%.0f" % (extra[9:].lower(), v[extra] / w)
    if v.get("SQ_BUSY_CYCLES"):
        for a in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
            if a in v and "SQ_WAVE_CYCLES" in v:
                s += " %s=%.2f" % (a[3:].lower(), v[a] / v["SQ_WAVE_CYCLES"])
    print(s)
