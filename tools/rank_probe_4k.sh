#!/bin/bash
# One rank's compute share of config 5 (3840x2160, 4 spp) at N = 1, 2, 4, 8: tools/rank_probe.py with
# the strip-local denoise (exchanges left out), one fresh process per N, serial stage split too.
for n in ${1:-1 2 4 8}; do
  W=3840 H=2160 QUICK=1 STRIP_DN=1 STAGES=1 FRAMES=20 timeout -k 10 150 python -u tools/rank_probe.py $n || exit $?
done
