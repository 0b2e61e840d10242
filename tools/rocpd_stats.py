#!/usr/bin/env python3
"""Per-kernel median / mean duration (us) and calls from a rocprofv3 SQLite result (rocpd views)."""
import collections
import sqlite3
import statistics
import sys

c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "name" if "name" in cols else "kernel_name"
d = collections.defaultdict(list)
for n, s, e in c.execute("select %s, start, end from kernels" % name):
    d[n.replace("(anonymous namespace)::", "").split("(")[0][-44:]].append((e - s) / 1e3)
tot = sum(sum(v) for v in d.values())
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print("%-46s calls %4d  median %8.2f us  mean %8.2f us  %5.1f%%" % (k, len(v), statistics.median(v), statistics.mean(v), 100 * sum(v) / tot))
