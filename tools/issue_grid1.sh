#!/bin/bash
# Issue-point grid (RTX_CAMERA_AFTER x RTX_OVERLAP_AFTER) of the 1-GPU pipelined frame via
# tools/abl_run.py, one fresh process per setting.  Usage: tools/issue_grid1.sh <outdir> "<CA:OA list>"
set -u
OUT=${1:-gpurun_out/grid}; SETS=${2:-"3:1"}
mkdir -p "$OUT"
for s in $SETS; do
  ca=${s%%:*}; oa=${s##*:}
  RTX_CAMERA_AFTER=$ca RTX_OVERLAP_AFTER=$oa timeout -k 10 120 python tools/abl_run.py > "$OUT/ca${ca}_oa${oa}.json" 2> "$OUT/ca${ca}_oa${oa}.err" || { tail -5 "$OUT/ca${ca}_oa${oa}.err"; exit 1; }
  echo "CA=$ca OA=$oa $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_frame'])" "$OUT/ca${ca}_oa${oa}.json")"
done
