#!/bin/bash
# rocprofv3 runs of one command: a --kernel-trace --stats run and/or the PMC passes, each its own
# rocprofv3 process under its own time limit (counters never combined with other trace domains);
# the chain stops at the first failure.  The PMC summary (tools/pmc_report.py) goes to
# <outdir>/pmc.json.
#   tools/prof.sh <outdir> stats|pmc|both|trace [python args...]
# e.g. tools/prof.sh gpurun_out/dn both tools/probe.py denoise --n 10
#      tools/prof.sh gpurun_out/b stats bench.py --gpus 1 --steps 20 --warmup 5
#      tools/prof.sh gpurun_out/tl trace bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-self-check
# PASSES overrides the counter groups (';'-separated); KEY / WORKLOAD label pmc.json (bench.py reads
# the committed copy when its workload_key matches, e.g. KEY=1920x1080x4).  trace: a kernel trace and
# its pipelined-frame timeline (tools/timeline.py) in <outdir>/timeline.txt.
set -u
OUT=$1; MODE=$2; shift 2
export TMPDIR=/tmp
mkdir -p "$OUT"
if [[ $MODE == stats || $MODE == both ]]; then
  echo "[$(date +%T)] stats: python3 $*"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o stats -- \
      python3 "$@" > "$OUT/stats.out" 2> "$OUT/stats.err" || { tail -20 "$OUT/stats.err"; exit 1; }
  f=$(find "$OUT/stats" -name "*kernel_stats.csv" | head -1)
  cp "$f" "$OUT/kernel_stats.csv"
fi
if [[ $MODE == trace ]]; then
  echo "[$(date +%T)] trace: python3 $*"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o tl -- \
      python3 "$@" > "$OUT/trace.out" 2> "$OUT/trace.err" || { tail -20 "$OUT/trace.err"; exit 1; }
  F=$(find "$OUT/trace" -name "*kernel_trace.csv" | head -1)
  python3 tools/timeline.py "$F" 6 3 > "$OUT/timeline.txt"
  tail -4 "$OUT/timeline.txt"
fi
if [[ $MODE == pmc || $MODE == both ]]; then
  DEF="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS"
  IFS=';' read -ra GROUPS_ <<< "${PASSES:-$DEF}"
  dirs=()
  i=0
  for pass in "${GROUPS_[@]}"; do
    i=$((i+1))
    echo "[$(date +%T)] pmc pass $i: $pass"
    # shellcheck disable=SC2086
    timeout -s KILL 180 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d "$OUT/pmc$i" -o pmc$i -- \
        python3 "$@" > "$OUT/pmc$i.out" 2> "$OUT/pmc$i.err" || { tail -20 "$OUT/pmc$i.err"; exit 1; }
    dirs+=("$OUT/pmc$i")
  done
  python3 tools/pmc_report.py "$OUT/pmc.json" "${dirs[@]}" --key "${KEY:-}" --workload "${WORKLOAD:-python3 $*}" \
      > "$OUT/pmc_summary.txt" 2>&1
  cat "$OUT/pmc_summary.txt"
fi
echo "[$(date +%T)] done"
