#!/bin/bash
# Round-4 GPU session 2: the LBVH refit change under the BVH tests, then A/B of library variants
# (bench lines + config 2/4 probe) and of stream priorities.
set -u
O=gpurun_out/r04_s2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "bvh or bin_scene" > $O/pytest_bvh.log 2>&1 || { tail -30 $O/pytest_bvh.log; exit 1; }
tail -1 $O/pytest_bvh.log
L=real-time-ray-tracing_amd
bash tools/lib_ab.sh $O/libab $L/lib/librtx.so $L/abl_oldrefit/librtx.so $L/abl_cam5/librtx.so $L/abl_cam4/librtx.so \
    $L/abl_gb4/librtx.so $L/abl_campf5/librtx.so $L/abl_primpf/librtx.so || exit 1
for th in 1024 512; do
  RTX_BVH_THREADS=$th timeout -k 10 120 python tools/c2c4_probe.py 20 > $O/probe_th$th.json 2> $O/probe_th$th.err || { tail -20 $O/probe_th$th.err; exit 1; }
  echo "bvh threads $th: $(cat $O/probe_th$th.json)"
done
bash tools/prio_ab.sh $O/prio || exit 1
echo "[$(date +%T)] session done"
