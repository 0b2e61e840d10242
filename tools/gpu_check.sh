#!/bin/bash
# One GPU-box session: parity tests, smoke, bench line.  Each step has its own time limit and the
# chain stops at the first failure.  Usage: tools/gpu_check.sh <outdir> [tests|bench|all] [pytest -k expr]
set -u
OUT=${1:-gpurun_out/run}
WHAT=${2:-all}
KEXPR=${3:-}
export TMPDIR=/tmp
export RTX_REPORT_DIR="$OUT"
mkdir -p "$OUT"
step() { echo "[$(date +%T)] $*"; }
if [[ $WHAT == tests || $WHAT == all ]]; then
  step pytest-gpu
  if [[ -n $KEXPR ]]; then K=(-k "$KEXPR"); else K=(); fi
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
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
step done
