#!/usr/bin/env python3
"""Median per-dispatch PMC values by kernel name from rocprofv3 --pmc CSV output directories."""
import collections
import csv
import glob
import statistics
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + '/*counter_collection.csv'):
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            per[(r['Kernel_Name'], r['Dispatch_Id'])][r['Counter_Name']] = float(r['Counter_Value'])
        for (k, _), c in per.items():
            for n, v in c.items():
                vals[k.replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0][-40:]][n].append(v)
for k, c in sorted(vals.items()):
    print('%-40s %s' % (k, ' '.join('%s=%.3g' % (n.replace('SQ_', ''), statistics.median(v)) for n, v in sorted(c.items()))))
