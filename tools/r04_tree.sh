#!/bin/bash
# (record of a measured and reverted A/B: the switch it builds against is no longer in the sources; DESIGN.md has the result)
# sky light-CDF heap: 14 levels in LDS (product) vs 12 (abl_tree4k, the round-3 layout)
set -o pipefail
mkdir -p gpurun_out/tree
A=real-time-ray-tracing_amd/abl_tree4k/librtx.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "pathtrace or bench_path or pipeline or sky" > gpurun_out/tree/tests.log 2>&1 &&
timeout -k 10 200 python -u tools/stage_probe.py > gpurun_out/tree/stage_new.json 2>&1 &&
timeout -k 10 200 python -u tools/stage_probe.py $A > gpurun_out/tree/stage_old.json 2>&1 &&
bash tools/env_ab.sh gpurun_out/tree/ab none 2 - RTX_LIB=$A
rc=$?; tail -1 gpurun_out/tree/tests.log; grep -v amdgpu gpurun_out/tree/stage_new.json; grep -v amdgpu gpurun_out/tree/stage_old.json; exit $rc
