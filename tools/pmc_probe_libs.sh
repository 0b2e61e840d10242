#!/bin/bash
# SQ_INSTS_VALU / SQ_WAVES per path-trace kernel of a kprobe run for several librtx builds.
# Usage: [PITCH=p] tools/pmc_probe_libs.sh <outdir> lib.so ...
set -u
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for lib in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d "$OUT/l$i" -o p -- \
      python3 tools/kprobe.py "$lib" > "$OUT/l$i.txt" 2> "$OUT/l$i.err" || { tail -5 "$OUT/l$i.err"; exit 1; }
  echo "== $lib"
  python3 tools/pmc_kernels.py "$OUT/l$i" | grep -E "k_pt_camera|k_pt_shade0|k_pt_resume<3>|k_trace_queue<3>" || true
done
