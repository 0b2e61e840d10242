#!/bin/bash
# One rank's pipelined frame (tools/rank_probe.py, strip-local denoise) at each N, one fresh
# process per setting, with the fused chain forced on or off.  Usage: tools/rank_grid.sh "<N list>" [repeats]
NS=${1:-"1 2 4 8"}; REP=${2:-2}
for r in $(seq $REP); do for n in $NS; do for ch in serial always off; do
  echo "rep=$r N=$n RTX_CHAIN=$ch $(STRIP_DN=1 RTX_CHAIN=$ch timeout -k 10 120 python tools/rank_probe.py $n 2>&1 | grep N=)"
done; done; done
