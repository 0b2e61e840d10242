#!/bin/bash
# One rank's compute share of the 1080p, 4 spp frame at N = 1, 2, 4, 8 (tools/rank_probe.py,
# strip-local denoise, exchanges left out), one fresh process per N, serial stage split too.
for n in ${1:-1 2 4 8}; do
  QUICK=1 STRIP_DN=1 STAGES=1 FRAMES=30 timeout -k 10 150 python -u tools/rank_probe.py $n || exit $?
done
