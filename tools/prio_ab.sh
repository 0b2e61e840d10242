#!/bin/bash
# A/B of stream priorities in the pipelined frame (FramePipeline RTX_MAIN_PRIO / RTX_POST_PRIO, the
# renderer's RTX_STREAMS): two bench lines per variant.  Usage: tools/prio_ab.sh <outdir>
set -u
OUT=${1:-gpurun_out/prio}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for v in "RTX_POST_PRIO=lo" "RTX_POST_PRIO=hi" "RTX_POST_PRIO=0" "RTX_MAIN_PRIO=0 RTX_POST_PRIO=0" \
         "RTX_STREAMS=prio RTX_POST_PRIO=hi" "RTX_STREAMS=prio RTX_POST_PRIO=lo"; do
  i=$((i+1))
  for r in 1 2; do
    env $v timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --no-self-check > "$OUT/b$i.$r.json" 2> "$OUT/b$i.$r.err" || { tail -20 "$OUT/b$i.$r.err"; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[2]));print(sys.argv[1], d['ms_per_step'], d['value'], {k: round(v['ms'],4) for k, v in d['roofline']['kernels'].items()})" "$v" "$OUT/b$i.$r.json"
  done
done
