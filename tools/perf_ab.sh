#!/bin/bash
# A/B timing of librtx builds after a kernel change: the bit-exact tests that cover it (product
# build), then per library two pipelined bench lines and the queue-tail latency anatomy
# (tools/trace_lat.py).  Usage: tools/perf_ab.sh <outdir> "<pytest -k expr>" lib.so ...
set -u
OUT=${1:-gpurun_out/ab}; shift
K=${1:-"trace or pathtrace or bench_path or pipeline"}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
if [[ $K != none ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
i=0
for lib in "$@"; do
  i=$((i+1))
  for r in 1 2; do
    RTX_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --no-self-check > "$OUT/b$i.$r.json" 2> "$OUT/b$i.$r.err" || { tail -20 "$OUT/b$i.$r.err"; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[2]));print(sys.argv[1], d['ms_per_step'], d['value'], {k: round(v['ms'],4) for k, v in d['roofline']['kernels'].items()})" "$lib" "$OUT/b$i.$r.json"
  done
  timeout -k 10 200 python tools/trace_lat.py "$lib" > "$OUT/lat$i.txt" 2>&1 || { tail -20 "$OUT/lat$i.txt"; exit 1; }
  grep -E "queue|longest alone|64 longest|all but the longest 1%" "$OUT/lat$i.txt"
done
