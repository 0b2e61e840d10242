#!/bin/bash
# Quick traversal check: the trace/pathtrace GPU tests (bit-exact vs the oracle), the lone-ray
# anatomy probe, queue latency and one bench line + the config-2/4 probe.  Usage: tools/r04_quick.sh <tag>
set -u
O=gpurun_out/q_$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "trace or pathtrace or bench_path or primary or bvh" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python tools/probe/lat_probe.py > $O/lat_probe.txt 2>&1 || { tail -20 $O/lat_probe.txt; exit 1; }
grep -A1 "^longest" $O/lat_probe.txt
timeout -k 10 200 python tools/trace_lat.py > $O/lat.txt 2>&1 || { tail -20 $O/lat.txt; exit 1; }
grep -E "queue|longest alone" $O/lat.txt
bash tools/lib_ab.sh $O/libab real-time-ray-tracing_amd/lib/librtx.so || exit 1
