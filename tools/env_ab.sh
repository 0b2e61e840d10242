#!/bin/bash
# A/B of environment switches on the two bench views: the bit-exact tests named by the -k expression
# (product defaults), then for each setting (space-separated VAR=VALUE list, "-" for none) and each
# repeat, tools/view_ab.py in a process of its own.  Each step under its own time limit; the chain
# stops at the first failure.  Usage: tools/env_ab.sh <outdir> "<pytest -k expr>|none" <repeats> "<setting>" ...
set -u
OUT=${1:-gpurun_out/envab}; shift
K=$1; shift
REP=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
if [[ $K != none ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
for r in $(seq 1 "$REP"); do
  i=0
  for setting in "$@"; do
    i=$((i+1))
    if [[ $setting == - ]]; then ENVS=(); else read -r -a ENVS <<< "$setting"; fi
    env "${ENVS[@]}" timeout -k 10 200 python tools/view_ab.py 30 "$setting" > "$OUT/v$i.$r.json" 2> "$OUT/v$i.$r.err" || { tail -20 "$OUT/v$i.$r.err"; exit 1; }
    cat "$OUT/v$i.$r.json"
  done
done
