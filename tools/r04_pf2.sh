#!/bin/bash
# (record of a measured and reverted A/B: the switch it builds against is no longer in the sources; DESIGN.md has the result)
# push-time record touch (RTX_TRAV_PF2): lone-ray anatomy, queue-tracer latency, pipelined frame
set -o pipefail
mkdir -p gpurun_out/pf2
L=real-time-ray-tracing_amd/abl_pf2/librtx.so
timeout -k 10 200 python -u tools/probe/lat_probe.py > gpurun_out/pf2/lat_base.txt 2>&1 &&
LATPROBE_LIB=tools/probe/liblatprobe_pf.so timeout -k 10 200 python -u tools/probe/lat_probe.py > gpurun_out/pf2/lat_pf.txt 2>&1 &&
timeout -k 10 200 python -u tools/trace_lat.py > gpurun_out/pf2/tl_base.txt 2>&1 &&
timeout -k 10 200 python -u tools/trace_lat.py $L > gpurun_out/pf2/tl_pf.txt 2>&1 &&
RTX_LIB=$L timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pathtrace or bench_path or trace" > gpurun_out/pf2/tests.log 2>&1 &&
bash tools/env_ab.sh gpurun_out/pf2/ab none 2 - RTX_LIB=$L
rc=$?; for f in lat_base lat_pf tl_base tl_pf; do echo "== $f"; grep -v amdgpu gpurun_out/pf2/$f.txt | tail -8; done; tail -2 gpurun_out/pf2/tests.log; exit $rc
