#!/bin/bash
# (record of a measured and reverted A/B: the switch it builds against is no longer in the sources; DESIGN.md has the result)
# LBVH: triangle records written as whole 64-B lines (abl_fullrec) vs 48 of 64 B (product)
set -o pipefail
mkdir -p gpurun_out/fullrec
A=real-time-ray-tracing_amd/abl_fullrec/librtx.so
for r in 1 2; do
  timeout -k 10 200 python -u tools/lbvh_probe.py > gpurun_out/fullrec/base$r.txt 2>&1 &&
  RTX_LIB=$A timeout -k 10 200 python -u tools/lbvh_probe.py > gpurun_out/fullrec/full$r.txt 2>&1 || exit 1
done
RTX_LIB=$A timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "bvh or bin_scene" > gpurun_out/fullrec/tests.log 2>&1
rc=$?; tail -1 gpurun_out/fullrec/tests.log; grep -h tris gpurun_out/fullrec/*.txt; exit $rc
