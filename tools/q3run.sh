#!/bin/bash
# Bounce-ray probe (tools/q3_probe.py) under a list of env settings, one process each.
# Usage: tools/q3run.sh <outdir> "<NAME=VAL,... list>"   ("-" = no extra env)
set -u
OUT=${1:-gpurun_out/q3}; SETS=${2:-"-"}
mkdir -p "$OUT"
for s in $SETS; do
  tag=$(echo "$s" | tr ',=/' '___')
  envs=(); [ "$s" != "-" ] && IFS=',' read -ra envs <<< "$s"
  env "${envs[@]}" timeout -k 10 120 python tools/q3_probe.py "$OUT/$tag" > "$OUT/$tag.log" 2>&1 || { tail "$OUT/$tag.log"; exit 1; }
  echo "== $s"; grep -v amdgpu.ids "$OUT/$tag.log"
done
