#!/bin/bash
# Instruction-mix and instruction-cache passes over serial frames of one view (four-kernel form,
# RTX_CHAIN=off), one rocprofv3 --pmc run per pass, each under its own time limit; the chain stops at
# the first failure.  Usage: tools/pmc_terrain.sh <outdir> [view]
set -u
OUT=${1:-gpurun_out/pmct}
VIEW=${2:-terrain}
export TMPDIR=/tmp RTX_CHAIN=off
mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" \
            "SQC_ICACHE_HITS SQC_ICACHE_MISSES" \
            "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_CVT" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F64 SQ_IFETCH"; do
  i=$((i+1))
  echo "[$(date +%T)] pass $i: $pass"
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d "$OUT/p$i" -o p$i -- \
      python3 tools/terrain_frames.py "$VIEW" 3 > "$OUT/p$i.log" 2> "$OUT/p$i.err" || { tail -20 "$OUT/p$i.err"; exit 1; }
done
echo done
