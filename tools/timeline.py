#!/usr/bin/env python3
"""Kernel timelines from a rocprofv3 --kernel-trace CSV (tools/prof.sh trace).

  timeline.py <kernel_trace.csv> [first_frame] [frames]          every kernel of pipelined frames
      a..a+frames (frames delimited by the LBVH build), µs from the first shown kernel, with its
      hardware queue, and the frame period; per stream (queue) the summed kernel time per frame
  timeline.py --sync <kernel_trace.csv> [first_frame] [frames]   synchronous draws (frames delimited
      by the camera kernel): per frame the union of kernel intervals (GPU busy), the idle time
      inside it and the largest gaps"""
import collections
import csv
import sys


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def pipelined(rows, a, nf):
    idx = [i for i, r in enumerate(rows) if "k_build_bvh" in r["Kernel_Name"]]
    start, end = idx[a], idx[min(a + nf, len(idx) - 1)]
    t0 = int(rows[start]["Start_Timestamp"])
    busy = collections.defaultdict(float)
    for r in rows[start:end]:
        s = (int(r["Start_Timestamp"]) - t0) / 1000
        e = (int(r["End_Timestamp"]) - t0) / 1000
        busy[r["Queue_Id"]] += e - s
        print("%8.1f %8.1f %7.1f q%s %s" % (s, e, e - s, r["Queue_Id"], short(r["Kernel_Name"])[:30]))
    print("frame period: %.1f us" % ((int(rows[end]["Start_Timestamp"]) - t0) / 1000 / nf))
    # the chip's idle time: moments with no kernel of any queue running (host-bound gaps)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows[start:end])
    idle, cur_e, one = 0, iv[0][1], 0
    for s_, e_ in iv[1:]:
        if s_ > cur_e:
            idle += s_ - cur_e
        cur_e = max(cur_e, e_)
    # time with exactly one kernel running (no overlap) vs two or more
    ev = sorted([(s_, 1) for s_, _ in iv] + [(e_, -1) for _, e_ in iv])
    depth, last, alone = 0, ev[0][0], 0
    for t_, d_ in ev:
        if depth == 1:
            alone += t_ - last
        depth += d_
        last = t_
    print("no kernel running: %.1f us per frame; one kernel alone: %.1f us per frame" % (idle / 1000 / nf, alone / 1000 / nf))
    print("kernel time per frame by queue: " + ", ".join("q%s %.1f us" % (q, v / nf) for q, v in sorted(busy.items())))


def synchronous(rows, a, nf):
    cam = [i for i, r in enumerate(rows) if "k_pt_camera" in r["Kernel_Name"]]
    for f in range(a, min(a + nf, len(cam) - 1)):
        seg = rows[cam[f]:cam[f + 1]]
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in seg)
        busy, cur_s, cur_e, idle, gaps = 0, iv[0][0], iv[0][1], 0, []
        for s, e, n in iv[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, short(n)[-28:]))
                idle += s - cur_e
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        period = int(rows[cam[f + 1]]["Start_Timestamp"]) - iv[0][0]
        big = sorted(gaps, reverse=True)[:4]
        print("frame %d: period %.1f us, busy %.1f, idle %.1f; largest gaps before: %s" % (
            f, period / 1e3, busy / 1e3, idle / 1e3, ", ".join("%.1f %s" % (g / 1e3, n) for g, n in big)))


def main():
    args = sys.argv[1:]
    sync = args and args[0] == "--sync"
    if sync:
        args = args[1:]
    rows = sorted(csv.DictReader(open(args[0])), key=lambda r: int(r["Start_Timestamp"]))
    a = int(args[1]) if len(args) > 1 else (10 if sync else 5)
    nf = int(args[2]) if len(args) > 2 else (10 if sync else 2)
    (synchronous if sync else pipelined)(rows, a, nf)


if __name__ == "__main__":
    main()
