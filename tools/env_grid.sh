#!/bin/bash
# Pipelined 1-GPU frame time (tools/abl_run.py) under several environment settings, one fresh
# process each.  Usage: tools/env_grid.sh <outdir> "label:VAR=v,VAR2=w label2:VAR=x ..."
set -u
OUT=${1:-gpurun_out/envgrid}; SETS=${2:-"base:"}
mkdir -p "$OUT"
for s in $SETS; do
  label=${s%%:*}; kv=${s#*:}
  envs=()
  IFS=',' read -ra pairs <<< "$kv"
  for p in "${pairs[@]}"; do [[ -n $p ]] && envs+=("$p"); done
  env "${envs[@]}" timeout -k 10 120 python tools/abl_run.py > "$OUT/$label.json" 2> "$OUT/$label.err" || { tail -5 "$OUT/$label.err"; exit 1; }
  echo "$label $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_frame'], {k: round(v, 3) for k, v in d.get('kernels', {}).items()})" "$OUT/$label.json")"
done
