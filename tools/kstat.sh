#!/bin/bash
# rocprofv3 kernel stats of serial frames (tools/serial_frames.py) for each library given.
# Usage: tools/kstat.sh <outdir> lib.so ...
set -u
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for lib in "$@"; do
  i=$((i+1))
  RTX_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/s$i" -o s -- \
      python3 tools/serial_frames.py 10 > "$OUT/s$i.log" 2>&1 || { tail -20 "$OUT/s$i.log"; exit 1; }
  f=$(find "$OUT/s$i" -name "*kernel_stats.csv" | head -1)
  echo "== $lib"
  python3 -c "
import csv,sys
for r in csv.reader(open(sys.argv[1])):
    if r[0]=='Name': continue
    n=r[0].replace('(anonymous namespace)::','').split('(')[0]
    if float(r[3])>5000: print('  %-40s %6.1f us' % (n[:40], float(r[3])/1000))
" "$f"
done
