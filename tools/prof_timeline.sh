#!/bin/bash
# Kernel timeline of pipelined bench frames (rocprofv3 --kernel-trace, csv) and its per-frame
# summary (tools/timeline.py).  Usage: tools/prof_timeline.sh <outdir> [extra bench args]
set -u
OUT=${1:-gpurun_out/tl}; shift || true
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o tl -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-self-check "$@" > "$OUT/bench.json" 2> "$OUT/trace.err" || { tail -20 "$OUT/trace.err"; exit 1; }
F=$(find "$OUT/trace" -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py "$F" 6 3 > "$OUT/timeline.txt"
tail -3 "$OUT/timeline.txt"
