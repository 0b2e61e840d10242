#!/bin/bash
# bench line, then the bench under rocprofv3 --kernel-trace --stats (per-kernel averages for profiles/)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fin5
timeout -k 10 600 python bench.py > gpurun_out/fin5/bench.json 2> gpurun_out/fin5/bench.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin5/stats -o stats -- python3 bench.py --steps 20 > gpurun_out/fin5/stats_bench.json 2> gpurun_out/fin5/stats.err
rc=$?; tail -c 1500 gpurun_out/fin5/bench.json; tail -5 gpurun_out/fin5/bench.err; exit $rc
