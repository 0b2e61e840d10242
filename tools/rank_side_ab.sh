#!/bin/bash
# One rank's compute share (tools/rank_probe.py, strip-local denoise, exchanges left out) at N ranks
# with the shade kernel on the context stream (RTX_SHADE_SIDE=0) and on the side stream (=1), one
# fresh process per point, each under its own time limit.  Usage: tools/rank_side_ab.sh [N ...]
set -u
for n in ${@:-2 4 8}; do
  for side in 0 1 0 1; do
    echo "N=$n RTX_SHADE_SIDE=$side"
    RTX_SHADE_SIDE=$side QUICK=1 STRIP_DN=1 FRAMES=30 timeout -k 10 150 python -u tools/rank_probe.py $n || exit $?
  done
done
