#!/bin/bash
# VALU instructions per wave and kernel times of serial frames (tools/denoise_probe.py) for a list
# of builds: "tag:lib" ("tag:-" = the in-tree build).  Usage: tools/pmc_abl.sh <outdir> <view> tag:lib ...
set -u
OUT=$1; VIEW=$2; shift 2
mkdir -p $OUT; export TMPDIR=/tmp
for s in "$@"; do
  tag=${s%%:*}; lib=${s#*:}
  envs=(); [ "$lib" != "-" ] && envs=(RTX_LIB=$lib)
  env "${envs[@]}" timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU \
      --kernel-trace -d $OUT/$tag -o p -- python3 tools/denoise_probe.py 4 $VIEW > $OUT/$tag.log 2>&1 || { tail $OUT/$tag.log; exit 1; }
  echo "== $tag"; python3 tools/rocpd_pmc.py $(ls $OUT/$tag/*.db | head -1) k_pt
done
