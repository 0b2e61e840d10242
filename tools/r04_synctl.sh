#!/bin/bash
# kernel timeline of synchronous draws (rt_draw_device without RT_DRAW_ASYNC) and its gaps
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/synctl
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/synctl/trace -o tl -- \
    python3 tools/draw_probe.py sync > gpurun_out/synctl/probe.txt 2> gpurun_out/synctl/trace.err || { tail -20 gpurun_out/synctl/trace.err; exit 1; }
F=$(find gpurun_out/synctl/trace -name "*kernel_trace.csv" | head -1)
python3 tools/sync_timeline.py "$F" 10 12 > gpurun_out/synctl/gaps.txt && cat gpurun_out/synctl/probe.txt gpurun_out/synctl/gaps.txt
