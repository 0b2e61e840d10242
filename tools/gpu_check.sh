#!/bin/bash
# One GPU-box session: parity tests, smoke, bench line, rocprofv3 kernel stats and the two
# PMC passes (FETCH_SIZE, WRITE_SIZE) of the bench workload.  Each step has its own time limit
# and the chain stops at the first failure.  Usage: tools/gpu_check.sh <outdir> [tests|bench|prof|all]
set -u
OUT=${1:-gpurun_out/run}
WHAT=${2:-all}
export TMPDIR=/tmp
mkdir -p "$OUT"
step() { echo "[$(date +%T)] $*"; }
if [[ $WHAT == tests || $WHAT == all ]]; then
  step pytest-gpu
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
  step smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -30 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
if [[ $WHAT == bench || $WHAT == all ]]; then
  step bench
  timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
  cat "$OUT/bench.json"
fi
if [[ $WHAT == prof || $WHAT == all ]]; then
  step rocprof-stats
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o stats -- \
      python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { tail -30 "$OUT/prof.err"; exit 1; }
  step rocprof-pmc-fetch
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o fetch -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err" || { tail -30 "$OUT/pmc_fetch.err"; exit 1; }
  step rocprof-pmc-write
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o write -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err" || { tail -30 "$OUT/pmc_write.err"; exit 1; }
  find "$OUT" -name "*.csv" | head -20
fi
step done
