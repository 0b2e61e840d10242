#!/usr/bin/env python3
"""Per-kernel PMC values of the path-trace stages for each probe camera (frame 3 of each)."""
import collections
import csv
import glob
import sys

names = ['k_pt_camera', 'k_pt_shade0', 'k_trace_queue<3>', 'k_pt_resume<3>', 'k_trace_queue<4>', 'k_pt_resume<4>', 'k_pt_resolve']
for d in sys.argv[1:]:
    f = glob.glob(d + '/*counter_collection.csv')[0]
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        k = next((k for k in names if k in r['Kernel_Name']), None)
        if k is None:
            continue
        key = int(r['Dispatch_Id'])
        disp.setdefault(key, [k, {}])[1][r['Counter_Name']] = float(r['Counter_Value'])
    seq = [disp[k] for k in sorted(disp)]
    N = len(names)
    frames = [seq[i:i + N] for i in range(0, len(seq), N)]
    per_cam = len(frames) // 3
    for ci, cam in enumerate(('default', 'down', 'up')):
        fr = frames[ci * per_cam + 2]
        print(cam)
        for k, c in fr:
            print('   %-18s %s' % (k, ' '.join('%s=%.3g' % (n.replace('SQ_', ''), v) for n, v in sorted(c.items()))))
