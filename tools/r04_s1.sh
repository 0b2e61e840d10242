#!/bin/bash
# Round-4 GPU session 1: suite + smoke + bench (product build), configs 2/4 under rocprofv3, a
# pipelined timeline, and the A/B of the queue tracers' record prefetch (product vs abl_nopf).
set -u
O=gpurun_out/r04_s1
mkdir -p $O
bash tools/gpu_check.sh $O/check all || exit 1
bash tools/prof_r04_c2c4.sh $O/c2c4 || exit 1
bash tools/prof_timeline.sh $O/tl || exit 1
bash tools/perf_ab.sh $O/ab none real-time-ray-tracing_amd/lib/librtx.so real-time-ray-tracing_amd/abl_nopf/librtx.so || exit 1
echo "[$(date +%T)] session done"
