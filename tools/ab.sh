#!/bin/bash
# A/B of one probe command over variants, repeats interleaved (A B A B ...), each run a fresh
# process under its own time limit; the chain stops at the first failure.
#   tools/ab.sh <outdir> <repeats> "<variant>|<variant>|..." python3 tools/probe.py frames
# A variant is a space-separated list of VAR=value settings applied to that run, e.g.
#   "RTX_LIB=real-time-ray-tracing_amd/abl_x/librtx.so" | "" (the in-tree build) | "RTX_TUNING=chain=off"
# (RTX_TUNING becomes the config's [tuning] table in rtx.write_config; the library reads no environment)
# Every run's last stdout line goes to <outdir>/ab.jsonl with its variant and repeat.
set -u
OUT=$1; REPS=$2; VARIANTS=$3; shift 3
export TMPDIR=/tmp
mkdir -p "$OUT"
IFS='|' read -ra VS <<< "$VARIANTS"
for r in $(seq 1 "$REPS"); do
  i=0
  for v in "${VS[@]}"; do
    i=$((i+1))
    log="$OUT/v${i}_r${r}"
    # shellcheck disable=SC2086
    env $v timeout -k 10 300 "$@" > "$log.out" 2> "$log.err" || { echo "variant $i ($v) failed"; tail -20 "$log.err"; exit 1; }
    line=$(tail -1 "$log.out")
    echo "{\"variant\": \"$v\", \"repeat\": $r, \"out\": $line}" | tee -a "$OUT/ab.jsonl"
  done
done
