#!/bin/bash
# Instruction-mix passes over serial frames (bench.py --no-pipeline): one rocprofv3 --pmc run per
# pass, each under its own limit; then the kernel-trace stats of the same command.
# Usage: tools/pmc_work.sh <outdir> [bench args...]
set -u
OUT=${1:-gpurun_out/work}; shift
ARGS="${@:---no-pipeline}"
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
            "SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  echo "[$(date +%T)] pass $i"
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$OUT/p$i" -o p$i -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-self-check $ARGS > "$OUT/p$i.json" 2> "$OUT/p$i.err" || { tail -20 "$OUT/p$i.err"; exit 1; }
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/st" -o st -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --no-self-check $ARGS > "$OUT/st.json" 2> "$OUT/st.err" || { tail -20 "$OUT/st.err"; exit 1; }
python3 tools/pmc_work.py "$OUT/p1" "$OUT/p2" > "$OUT/work.txt"
echo done
