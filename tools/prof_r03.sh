#!/bin/bash
# Round-3 profiling session.  1) rocprofv3 --kernel-trace --stats of the driver's exact bench command
# (the timed process's own stats file holds its warm-up, timed, detail and split frames; the side
# legs run in a child process with a stats file of its own); 2) four PMC passes over the pipelined
# frames, each its own rocprofv3 run under its own time limit.  Usage: tools/prof_r03.sh <outdir>
set -u
OUT=${1:-gpurun_out/prof3}
export TMPDIR=/tmp
mkdir -p "$OUT"
echo "[$(date +%T)] stats of: python3 bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o stats -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/stats_bench.json" 2> "$OUT/stats.err" || { tail -20 "$OUT/stats.err"; exit 1; }
B="bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-extras --no-self-check --no-marks"
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
