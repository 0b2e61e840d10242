#!/bin/bash
# Denoise/post kernel stats of serial frames (tools/denoise_probe.py) under a list of settings, each
# "tag:ENV=V,ENV=V" ("tag:-" = none), plus one PMC pass on the first setting.
# Usage: tools/denoise_ab.sh <outdir> [view] setting...
set -u
OUT=$1; VIEW=$2; shift 2
mkdir -p $OUT; export TMPDIR=/tmp
first=1
for s in "$@"; do
  tag=${s%%:*}; e=${s#*:}
  envs=(); [ "$e" != "-" ] && IFS=',' read -ra envs <<< "$e"
  echo "[$(date +%T)] $tag ${envs[*]:-}"
  env "${envs[@]}" timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/$tag -o r -- \
      python3 tools/denoise_probe.py 20 $VIEW > $OUT/$tag.log 2>&1 || { tail $OUT/$tag.log; exit 1; }
  grep '^{' $OUT/$tag.log
  if [ $first = 1 ]; then
    first=0
    env "${envs[@]}" timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_ANY \
        --kernel-trace -d $OUT/pmc_$tag -o p -- python3 tools/denoise_probe.py 6 $VIEW > $OUT/pmc_$tag.log 2>&1 || { tail $OUT/pmc_$tag.log; exit 1; }
  fi
done
echo done
