#!/bin/bash
# One rocprofv3 --pmc pass over a short bench run.  Usage: tools/pmc_bench.sh <outdir> <counters...>
set -u
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT" -o pmc -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > "$OUT/bench.json" 2> "$OUT/prof.err" || { tail -20 "$OUT/prof.err"; exit 1; }
echo ok
