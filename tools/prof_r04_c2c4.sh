#!/bin/bash
# BASELINE configs 2 and 4 under rocprofv3: one --kernel-trace --stats run of
# tools/c2c4_probe.py, then one --pmc pass per counter group, each its own run under its own time
# limit; the chain stops at the first failure.  Usage: tools/prof_r04_c2c4.sh <outdir>
set -u
OUT=${1:-gpurun_out/c2c4}
export TMPDIR=/tmp
mkdir -p "$OUT"
echo "[$(date +%T)] stats"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o stats -- \
    python3 tools/c2c4_probe.py 20 > "$OUT/stats_probe.json" 2> "$OUT/stats.err" || { tail -20 "$OUT/stats.err"; exit 1; }
i=0
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
            "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  echo "[$(date +%T)] pmc pass $i: $pass"
  timeout -s KILL 150 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d "$OUT/pmc$i" -o pmc$i -- \
      python3 tools/c2c4_probe.py 10 > "$OUT/pmc$i.json" 2> "$OUT/pmc$i.err" || { tail -20 "$OUT/pmc$i.err"; exit 1; }
done
python3 tools/pmc_c2c4.py "$OUT/pmc_c2c4.json" "$OUT/pmc1" "$OUT/pmc2" "$OUT/pmc3" "$OUT/pmc4" > "$OUT/pmc_summary.txt" 2>&1
cat "$OUT/pmc_summary.txt"
echo "[$(date +%T)] done"
