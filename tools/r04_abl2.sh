#!/bin/bash
# Serial stage times (tools/stage_probe.py) of the scale/post ablations, and config-4 build times of
# the LBVH phase ablations (tools/c2c4_probe.py).
set -u
O=gpurun_out/r04_abl2
mkdir -p $O
export TMPDIR=/tmp
L=real-time-ray-tracing_amd
for l in lib abl_sp2 abl_sp3 abl_sp4 abl_sc384; do
  timeout -k 10 150 python tools/stage_probe.py $L/$l/librtx.so > $O/stage_$l.json 2> $O/stage_$l.err || { tail -20 $O/stage_$l.err; exit 1; }
  echo "$l $(cat $O/stage_$l.json)"
done
for l in lib abl_bvhnotlas abl_bvhnorefit; do
  RTX_LIB=$L/$l/librtx.so timeout -k 10 150 python tools/c2c4_probe.py 20 > $O/c4_$l.json 2> $O/c4_$l.err || { tail -20 $O/c4_$l.err; exit 1; }
  echo "$l $(cat $O/c4_$l.json)"
done
RTX_LIB=$L/abl_bvhstamps/librtx.so timeout -k 10 150 python tools/lbvh_stamps.py > $O/stamps.json 2> $O/stamps.err || { tail -20 $O/stamps.err; exit 1; }
cat $O/stamps.json
RTX_LIB=$L/abl_bvhstamps/librtx.so RTX_BVH_THREADS=512 timeout -k 10 150 python tools/lbvh_stamps.py > $O/stamps512.json 2> $O/stamps512.err || { tail -20 $O/stamps512.err; exit 1; }
cat $O/stamps512.json
bash tools/lib_ab.sh $O/libab $L/lib/librtx.so $L/abl_sc384/librtx.so || exit 1
