#!/bin/bash
# overlapped TLAS builder: BVH parity, C2/C4 build times, phase stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bvh or bin_scene or scene" > gpurun_out/tlas_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/c2c4_probe.py 20 > gpurun_out/tlas_c2c4.log 2>&1 &&
RTX_LIB=real-time-ray-tracing_amd/abl_bvhstamps/librtx.so timeout -k 10 200 python -u tools/lbvh_stamps.py > gpurun_out/tlas_stamps.log 2>&1
rc=$?; tail -3 gpurun_out/tlas_tests.log; cat gpurun_out/tlas_c2c4.log | tail -8; tail -20 gpurun_out/tlas_stamps.log; exit $rc
