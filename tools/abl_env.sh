#!/bin/bash
# Frame ablation (tools/abl_run.py) under a list of env settings, one process each, repeated.
# Usage: tools/abl_env.sh <outdir> "<NAME=VAL,... list>" [repeats]   ("-" = no extra env)
set -u
OUT=${1:-gpurun_out/abl}; SETS=${2:-"-"}; REP=${3:-1}
mkdir -p "$OUT"
for r in $(seq $REP); do for s in $SETS; do
  tag=$(echo "$s" | tr ',=/' '___')_$r
  envs=(); [ "$s" != "-" ] && IFS=',' read -ra envs <<< "$s"
  env "${envs[@]}" timeout -k 10 120 python tools/abl_run.py > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { tail "$OUT/$tag.err"; exit 1; }
  echo "$s rep$r $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_frame'], d['kernels'])" "$OUT/$tag.json")"
done; done
