#!/bin/bash
# Rehearsal of the N-rank bench path on one GPU (ranks share it over gloo; not a measurement):
# strip blocks, G-buffer gather, strip-local denoise, and rank 0's self-check against a serial
# single-rank re-render.  Usage: tools/gloo_bench.sh <outdir> [ranks]
set -u
OUT=${1:-gpurun_out/gloo}
N=${2:-2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus "$N" --steps 5 --warmup 2 --no-extras --no-cpu-baseline --dist-backend gloo \
    > "$OUT/gloo_bench_$N.json" 2> "$OUT/gloo_bench_$N.err" || { tail -30 "$OUT/gloo_bench_$N.err"; exit 1; }
cat "$OUT/gloo_bench_$N.json"
