#!/bin/bash
# k_downscale_chain without release/acquire fences (product) vs with (abl_olddn): parity, serial
# denoise, pipelined frame
set -o pipefail
mkdir -p gpurun_out/dnchain
A=real-time-ray-tracing_amd/abl_olddn/librtx.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "denoise or bench_path or pipeline or exposure or post" > gpurun_out/dnchain/tests.log 2>&1 &&
timeout -k 10 200 python -u tools/stage_probe.py > gpurun_out/dnchain/stage_new.json 2>&1 &&
timeout -k 10 200 python -u tools/stage_probe.py $A > gpurun_out/dnchain/stage_old.json 2>&1 &&
bash tools/env_ab.sh gpurun_out/dnchain/ab none 2 - RTX_LIB=$A
rc=$?; tail -1 gpurun_out/dnchain/tests.log; grep -v amdgpu gpurun_out/dnchain/stage_new.json; grep -v amdgpu gpurun_out/dnchain/stage_old.json; exit $rc
