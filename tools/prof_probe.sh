#!/bin/bash
# rocprofv3 kernel stats of tools/pt_probe.py (three cameras).  Usage: tools/prof_probe.sh <outdir>
set -u
OUT=${1:-gpurun_out/pp}
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o pp -- \
    python3 tools/pt_probe.py --iters 10 > "$OUT/probe.json" 2> "$OUT/prof.err" || { tail -20 "$OUT/prof.err"; exit 1; }
cat "$OUT/probe.json"
find "$OUT" -name "*kernel_stats.csv" -exec head -20 {} \;
