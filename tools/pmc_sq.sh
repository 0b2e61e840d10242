#!/bin/bash
# SQ-counter passes over the bench workload (one rocprofv3 --pmc run per pass, each under its own
# time limit; the chain stops at the first failure).  Usage: tools/pmc_sq.sh <outdir>
set -u
OUT=${1:-gpurun_out/sq}
export TMPDIR=/tmp
mkdir -p "$OUT"
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH" \
            "${EXTRA_PASS:-SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_CVT}"; do
  i=$((i+1))
  echo "[$(date +%T)] pass $i: $pass"
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d "$OUT/p$i" -o p$i -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > "$OUT/p$i.json" 2> "$OUT/p$i.err" || { tail -20 "$OUT/p$i.err"; exit 1; }
done
echo done
