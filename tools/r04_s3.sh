#!/bin/bash
# Round-4 GPU session 3: full GPU suite on the product build (templated LBVH, while-while tails,
# prefetching primary rays), lone-ray latency and bench/probe A/B against ablation builds, and the
# LBVH workgroup shapes on the 1M-triangle scene.
set -u
O=gpurun_out/r04_s3
mkdir -p $O
export TMPDIR=/tmp
L=real-time-ray-tracing_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for lib in $L/lib/librtx.so $L/abl_notail/librtx.so; do
  timeout -k 10 200 python tools/trace_lat.py $lib > $O/lat_$(basename $(dirname $lib)).txt 2>&1 || { tail -20 $O/lat_$(basename $(dirname $lib)).txt; exit 1; }
  echo "$lib"; grep -E "queue|longest alone|64 longest" $O/lat_$(basename $(dirname $lib)).txt
done
bash tools/lib_ab.sh $O/libab $L/lib/librtx.so $L/abl_notail/librtx.so $L/abl_primstep/librtx.so $L/abl_prim0/librtx.so \
    $L/abl_oldrefit/librtx.so || exit 1
for th in 1024 512; do
  RTX_BVH_THREADS=$th timeout -k 10 120 python tools/c2c4_probe.py 20 > $O/probe_th$th.json 2> $O/probe_th$th.err || { tail -20 $O/probe_th$th.err; exit 1; }
  echo "bvh threads $th: $(cat $O/probe_th$th.json)"
done
echo "[$(date +%T)] session done"
