#!/bin/bash
# Quick GPU check after a kernel change: the bit-exact tests that cover it, then the bench line
# (no extras).  Usage: tools/quick_perf.sh <outdir> "<pytest -k expr>"
set -u
OUT=${1:-gpurun_out/q}
K=${2:-"trace or pathtrace or bench_path"}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("ms/frame", d["ms_per_step"], "Mray/s", d["value"], "self_check", d.get("self_check", {}).get("ok"))
print({k: v["ms"] for k, v in d["roofline"]["kernels"].items()})
PY
