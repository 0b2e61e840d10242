#!/bin/bash
# (record of a measured and reverted A/B: the switch it builds against is no longer in the sources; DESIGN.md has the result)
# denoise 5x5 / 7x7 batch loops not unrolled (product) vs fully unrolled (abl_unroll8): parity, serial
# stages, pipelined frame
set -o pipefail
mkdir -p gpurun_out/unroll
A=real-time-ray-tracing_amd/abl_unroll8/librtx.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "denoise or bench_path or pipeline or multirank" > gpurun_out/unroll/tests.log 2>&1 &&
timeout -k 10 200 python -u tools/stage_probe.py > gpurun_out/unroll/stage_new.json 2>&1 &&
timeout -k 10 200 python -u tools/stage_probe.py $A > gpurun_out/unroll/stage_old.json 2>&1 &&
bash tools/env_ab.sh gpurun_out/unroll/ab none 2 - RTX_LIB=$A
rc=$?; tail -2 gpurun_out/unroll/tests.log; grep -v amdgpu gpurun_out/unroll/stage_new.json; grep -v amdgpu gpurun_out/unroll/stage_old.json; exit $rc
