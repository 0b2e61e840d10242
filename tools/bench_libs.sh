#!/bin/bash
# Pipelined bench ms/frame for several librtx builds (RTX_LIB picks the library).  Usage: tools/bench_libs.sh lib.so ...
for lib in "$@"; do
  for i in 1 2; do
    RTX_LIB=$lib timeout -k 10 100 python bench.py --no-cpu-baseline --no-extras > gpurun_out/bl.json || exit 1
    python -c "import json,sys;d=json.load(open('gpurun_out/bl.json'));print(sys.argv[1], d['ms_per_step'], d['value'])" "$lib"
  done
done
