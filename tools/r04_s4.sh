#!/bin/bash
# Round-4 GPU session 4: trav_step_pf2 (one divergent region per iteration) A/B — trace/pathtrace
# parity on the ablation build, lone-ray latency and bench/probe against the product build.
set -u
O=gpurun_out/r04_s4
mkdir -p $O
export TMPDIR=/tmp
L=real-time-ray-tracing_amd
RTX_LIB=$L/abl_step2/librtx.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "trace or pathtrace or bench_path or pipeline or primary" > $O/pytest_step2.log 2>&1 || { tail -30 $O/pytest_step2.log; exit 1; }
tail -1 $O/pytest_step2.log
for lib in $L/lib/librtx.so $L/abl_step2/librtx.so; do
  n=$(basename $(dirname $lib))
  timeout -k 10 200 python tools/trace_lat.py $lib > $O/lat_$n.txt 2>&1 || { tail -20 $O/lat_$n.txt; exit 1; }
  echo "$lib"; grep -E "queue|longest alone|64 longest" $O/lat_$n.txt
done
bash tools/lib_ab.sh $O/libab $L/lib/librtx.so $L/abl_step2/librtx.so || exit 1
echo "[$(date +%T)] session done"
