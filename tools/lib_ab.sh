#!/bin/bash
# A/B of librtx builds: per library two pipelined bench lines (no extras) and the config-2/4 probe
# (primary-ray and 1M-triangle LBVH event times).  Usage: tools/lib_ab.sh <outdir> lib.so ...
set -u
OUT=${1:-gpurun_out/libab}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1))
  for r in 1 2; do
    RTX_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --no-self-check > "$OUT/b$i.$r.json" 2> "$OUT/b$i.$r.err" || { tail -20 "$OUT/b$i.$r.err"; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[2]));print(sys.argv[1], d['ms_per_step'], d['value'], {k: round(v['ms'],4) for k, v in d['roofline']['kernels'].items()})" "$lib" "$OUT/b$i.$r.json"
  done
  RTX_LIB=$lib timeout -k 10 120 python tools/c2c4_probe.py 20 > "$OUT/p$i.json" 2> "$OUT/p$i.err" || { tail -20 "$OUT/p$i.err"; exit 1; }
  echo "$lib $(cat $OUT/p$i.json)"
done
