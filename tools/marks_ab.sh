#!/bin/bash
# Cost of the timed region's per-kernel HIP events: bench.py with and without them, alternating.
B="bench.py --steps 30 --warmup 5 --no-extras --no-cpu-baseline --no-self-check"
for r in 1 2 3; do
  for m in "" "--no-marks"; do
    echo "rep=$r marks=${m:-on} $(timeout -k 10 120 python3 $B $m | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["kernel"], r["kernel_ms"], r["kernel_ms_split_frames"])')" || exit 1
  done
done
