#!/usr/bin/env python3
"""Host API calls between synchronous frames (rocprofv3 --hip-runtime-trace --kernel-trace CSVs).

For frames i of a `tools/probe.py draw --modes sync` trace: the time from the last kernel of frame
i-1 to the first kernel of frame i, the HIP API calls the host made in that gap, and each kernel's
API call (launch) time against its GPU start.
  tools/api_gap.py <api_hip_api_trace.csv> <api_kernel_trace.csv> [first] [count]
"""
import csv
import sys


def rows(path):
    out = list(csv.DictReader(open(path)))
    for r in out:
        r["s"] = int(r["Start_Timestamp"])
        r["e"] = int(r["End_Timestamp"])
    out.sort(key=lambda r: r["s"])
    return out


def main():
    api, ker = rows(sys.argv[1]), rows(sys.argv[2])
    first = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    count = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    corr = {r["Correlation_Id"]: r for r in api}
    cams = [k for k in ker if "k_pt_camera" in k["Kernel_Name"]]
    gaps = []
    for ci in range(1, len(cams)):
        cam = cams[ci]
        prev = [k for k in ker if k["e"] < cam["s"] and "k_scale_post" in k["Kernel_Name"]]
        if prev:
            gaps.append((cam["s"] - prev[-1]["e"]) / 1000)
        if not (first <= ci < first + count) or not prev:
            continue
        t0 = prev[-1]["e"]
        print(f"--- frame {ci}: {(cam['s'] - t0) / 1000:.1f} us from the last kernel to the camera kernel")
        for r in api:
            if r["e"] >= t0 - 2000 and r["s"] <= cam["s"]:
                mark = "  <- camera launch" if r["Correlation_Id"] == cam["Correlation_Id"] else ""
                print(f"{(r['s'] - t0) / 1000:8.1f} {(r['e'] - t0) / 1000:8.1f} {(r['e'] - r['s']) / 1000:7.1f}  {r['Function']}{mark}")
        nxt = cams[ci + 1]["s"] if ci + 1 < len(cams) else 1 << 62
        print("kernels: GPU start-end, launch call start (us from the last kernel of the previous frame)")
        for k in ker:
            if cam["s"] - 300000 <= k["s"] < nxt:
                a = corr.get(k["Correlation_Id"])
                print(f"   {k['Kernel_Name'][:44]:44s} {(k['s'] - t0) / 1000:8.1f} {(k['e'] - t0) / 1000:8.1f}"
                      f"  {(a['s'] - t0) / 1000 if a else float('nan'):8.1f}")
    if gaps:
        gaps.sort()
        print(f"gaps over {len(gaps)} frames: min {gaps[0]:.1f} median {gaps[len(gaps) // 2]:.1f} max {gaps[-1]:.1f} us")


if __name__ == "__main__":
    main()
