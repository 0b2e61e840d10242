#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd SQLite output) as a kernel-stats CSV.

Usage: tools/rocpd_summary.py <run_results.db> [out.csv]
Columns follow rocprofv3's kernel_stats.csv: Name, Calls, TotalDurationNs, AverageNs, Percentage,
plus VGPR / LDS / grid from the dispatch records.
"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else None)
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    extra = {}
    for name, vgpr, agpr, lds, gx, gy, wx, wy in c.execute(
            "select name, vgpr_count, accum_vgpr_count, lds_size, grid_x, grid_y, workgroup_x, workgroup_y from kernels"):
        extra.setdefault(name, (vgpr, agpr, lds, gx, gy, wx, wy))
    f = open(out, "w", newline="") if out else sys.stdout
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "VGPR", "AGPR", "LDS", "Grid", "Workgroup"])
    for name, calls, tot, avg, pct in rows:
        vg, ag, lds, gx, gy, wx, wy = extra.get(name, ("", "", "", "", "", "", ""))
        w.writerow([name, calls, round(tot * 1e3), round(avg * 1e3), "%.3f" % pct, vg, ag, lds, "%sx%s" % (gx, gy),
                    "%sx%s" % (wx, wy)])


if __name__ == "__main__":
    main()
