#!/bin/bash
# One rank's pipelined frame (tools/rank_probe.py, strip-local denoise) at N ranks for several
# camera issue points (RTX_CAMERA_AFTER) with the fused chain on or off, a fresh process each.
# Usage: tools/rank_gate_grid.sh "<N list>" "<CA list>" "<chain list>" [repeats]
NS=${1:-8}; CAS=${2:-"0 1 2 3"}; CHS=${3:-"off"}; REP=${4:-2}
for r in $(seq $REP); do for n in $NS; do for ch in $CHS; do for ca in $CAS; do
  echo "rep=$r N=$n chain=$ch CA=$ca $(STRIP_DN=1 RTX_CHAIN=$ch RTX_CAMERA_AFTER=$ca timeout -k 10 120 python tools/rank_probe.py $n 2>&1 | grep N=)"
done; done; done; done
