#!/bin/bash
# Round-4 GPU session 5: the record-arena traversal (traverse.h) — full GPU suite (bit-exact vs the
# oracle), lone-ray anatomy, queue latency, bench lines and the config-2/4 probe.
set -u
O=gpurun_out/r04_s5
mkdir -p $O
export TMPDIR=/tmp
L=real-time-ray-tracing_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python tools/probe/lat_probe.py > $O/lat_probe.txt 2>&1 || { tail -20 $O/lat_probe.txt; exit 1; }
grep -v amdgpu.ids $O/lat_probe.txt
timeout -k 10 200 python tools/trace_lat.py > $O/lat.txt 2>&1 || { tail -20 $O/lat.txt; exit 1; }
grep -E "queue|longest alone|64 longest|all but" $O/lat.txt
bash tools/lib_ab.sh $O/libab $L/lib/librtx.so || exit 1
echo "[$(date +%T)] session done"
