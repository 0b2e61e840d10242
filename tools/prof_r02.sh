#!/bin/bash
# Profiling session of the bench workload: the rocprofv3 kernel-trace --stats summary of a bench
# run (pipelined frames only: --no-extras) and four PMC passes, each its own rocprofv3 run under
# its own time limit; the chain stops at the first failure.  Usage: tools/prof_r02.sh <outdir>
set -u
OUT=${1:-gpurun_out/prof}
export TMPDIR=/tmp
mkdir -p "$OUT"
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-self-check"
echo "[$(date +%T)] stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o stats -- \
    python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-extras --no-self-check > "$OUT/stats_bench.json" 2> "$OUT/stats.err" || { tail -20 "$OUT/stats.err"; exit 1; }
i=0
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
            "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"; do
  i=$((i+1))
  echo "[$(date +%T)] pmc pass $i: $pass"
  timeout -s KILL 150 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d "$OUT/pmc$i" -o pmc$i -- \
      python3 $B > "$OUT/pmc$i.json" 2> "$OUT/pmc$i.err" || { tail -20 "$OUT/pmc$i.err"; exit 1; }
done
python3 tools/pmc_r02.py "$OUT/pmc_kernels.json" "$OUT/pmc1" "$OUT/pmc2" "$OUT/pmc3" "$OUT/pmc4" > "$OUT/pmc_summary.txt" 2>&1
echo "[$(date +%T)] done"
