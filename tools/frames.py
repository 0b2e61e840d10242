#!/usr/bin/env python3
"""Per-stage durations (us) of the path-trace launches of one probe run, third frame per camera."""
import csv
import glob
import sys

names = ['k_pt_camera', 'k_pt_shade0', 'k_trace_queue<3>', 'k_pt_resume<3>', 'k_trace_queue<4>', 'k_pt_resume<4>', 'k_pt_resolve']
f = glob.glob(sys.argv[1] + '/*kernel_trace.csv')[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
seq = [(k, (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3, int(r['Start_Timestamp']),
        int(r['End_Timestamp'])) for r in rows for k in names if k in r['Kernel_Name']]
N = len(names)
frames = [seq[i:i + N] for i in range(0, len(seq), N)]
per = len(frames) // 3
for ci, cam in enumerate(('default', 'down', 'up')):
    fr = frames[ci * per + 4]
    print('%-8s span %7.1f  ' % (cam, (fr[-1][3] - fr[0][2]) / 1e3) + '  '.join('%s %.1f' % (k, d) for k, d, s, e in fr))
