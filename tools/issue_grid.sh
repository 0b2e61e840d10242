#!/bin/bash
# Issue-point comparison (RTX_CAMERA_AFTER x RTX_OVERLAP_AFTER) of one rank's pipelined frame
# (tools/rank_probe.py) at N ranks, each setting in a fresh process, repeated.
# Usage: tools/issue_grid.sh "<N list>" "<CA:OA list>" [repeats]
NS=${1:-8}; SETS=${2:-"2:5 3:2 1:0"}; REP=${3:-3}
for r in $(seq $REP); do for n in $NS; do for s in $SETS; do
  ca=${s%%:*}; oa=${s##*:}
  echo "rep=$r CA=$ca OA=$oa $(QUICK=1 RTX_CAMERA_AFTER=$ca RTX_OVERLAP_AFTER=$oa timeout -k 10 120 python tools/rank_probe.py $n 2>&1 | grep N=)"
done; done; done
