#!/bin/bash
# One rocprofv3 --pmc pass over tools/pt_probe.py.  Usage: tools/pmc_probe.sh <outdir> <counters...>
set -u
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT" -o pmc -- \
    python3 tools/pt_probe.py --iters 3 > "$OUT/probe.json" 2> "$OUT/prof.err" || { tail -20 "$OUT/prof.err"; exit 1; }
echo ok
