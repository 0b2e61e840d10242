#!/bin/bash
# Camera workgroups per CU (RTX_CAM_LDS_PAD: extra dynamic LDS) against the pipelined frame.
set -u
O=gpurun_out/r04_campad
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in 0 6000 14000 27000; do
    RTX_CAM_LDS_PAD=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --no-self-check > $O/b$v.$r.json 2> $O/b$v.$r.err || { tail -20 $O/b$v.$r.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[2]));k=d['roofline']['kernels'];print('pad', sys.argv[1], d['ms_per_step'], round(k['k_pt_camera']['ms'],4))" $v $O/b$v.$r.json
  done
done
