#!/bin/bash
# round-4 records: rocprofv3 stats + PMC passes of the bench (tools/prof_r03.sh), then the 4K line
set -o pipefail
bash tools/prof_r03.sh gpurun_out/prof4 > gpurun_out/prof4.log 2>&1 &&
timeout -k 10 300 python bench.py --width 3840 --height 2160 --no-cpu-baseline > gpurun_out/prof4/bench4k.json 2> gpurun_out/prof4/bench4k.err
rc=$?; tail -5 gpurun_out/prof4.log; tail -c 600 gpurun_out/prof4/bench4k.json; exit $rc
