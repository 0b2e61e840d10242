#!/bin/bash
# (record of a measured and reverted A/B: the switch it builds against is no longer in the sources; DESIGN.md has the result)
# sky light-CDF heap levels staged in LDS: 12 (product, 4096 nodes) vs 11 (abl_sky2k) vs 10 (abl_sky1k)
set -o pipefail
mkdir -p gpurun_out/tree2
A=real-time-ray-tracing_amd/abl_sky2k/librtx.so; B=real-time-ray-tracing_amd/abl_sky1k/librtx.so
RTX_LIB=$B timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "pathtrace or bench_path or sky" > gpurun_out/tree2/tests.log 2>&1 &&
timeout -k 10 200 python -u tools/stage_probe.py > gpurun_out/tree2/stage_4k.json 2>&1 &&
timeout -k 10 200 python -u tools/stage_probe.py $A > gpurun_out/tree2/stage_2k.json 2>&1 &&
timeout -k 10 200 python -u tools/stage_probe.py $B > gpurun_out/tree2/stage_1k.json 2>&1 &&
bash tools/env_ab.sh gpurun_out/tree2/ab none 2 - RTX_LIB=$A RTX_LIB=$B
rc=$?; tail -1 gpurun_out/tree2/tests.log; for f in 4k 2k 1k; do grep -v amdgpu gpurun_out/tree2/stage_$f.json; done; exit $rc
