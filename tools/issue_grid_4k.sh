#!/bin/bash
# Pipelined 4K frame (bench.py, no extras) under several issue points, a fresh process each.
# Usage: tools/issue_grid_4k.sh "<CA:OA list>"
SETS=${1:-"0:1 0:0 0:2 2:1"}
for s in $SETS; do
  ca=${s%%:*}; oa=${s##*:}
  RTX_CAMERA_AFTER=$ca RTX_OVERLAP_AFTER=$oa timeout -k 10 200 python bench.py --width 3840 --height 2160 --steps 15 --warmup 3 \
      --no-cpu-baseline --no-extras --no-self-check > gpurun_out/ig4k.json 2> gpurun_out/ig4k.err || { tail -5 gpurun_out/ig4k.err; exit 1; }
  echo "CA=$ca OA=$oa $(python -c "import json; d=json.load(open('gpurun_out/ig4k.json')); print(d['ms_per_step'])")"
done
