#!/bin/bash
# TLAS workgroup beside the BLAS builds: BVH parity, build times of both scenes, phase stamps, frame
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bvh or bin_scene or scene or pipeline" > gpurun_out/tlas_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/lbvh_probe.py > gpurun_out/tlas_lbvh.log 2>&1 &&
RTX_LIB=real-time-ray-tracing_amd/abl_bvhstamps/librtx.so timeout -k 10 200 python -u tools/lbvh_stamps.py > gpurun_out/tlas_stamps.log 2>&1 &&
timeout -k 10 200 python tools/view_ab.py 30 - > gpurun_out/tlas_view.log 2>&1
rc=$?; tail -3 gpurun_out/tlas_tests.log; tail -4 gpurun_out/tlas_lbvh.log; tail -2 gpurun_out/tlas_stamps.log; tail -2 gpurun_out/tlas_view.log; exit $rc
