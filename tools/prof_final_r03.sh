#!/bin/bash
# End-of-round records: the GPU suite + smoke + the driver's bench line (tools/gpu_check.sh), the
# rocprofv3 stats + PMC passes of the bench (tools/prof_r03.sh), the serial denoise kernels of both
# views under rocprofv3 (tools/denoise_probe.py) and the one-GPU 4K bench line.  Each step under its
# own time limit; the chain stops at the first failure.  Usage: tools/prof_final_r03.sh <outdir>
set -u
OUT=${1:-gpurun_out/final3}
export TMPDIR=/tmp
mkdir -p "$OUT"
bash tools/gpu_check.sh "$OUT/check" all || exit 1
bash tools/prof_r03.sh "$OUT/prof" || exit 1
for v in default terrain; do
  echo "[$(date +%T)] denoise kernels, $v view"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/dn_$v" -o dn -- \
      python3 tools/denoise_probe.py 20 $v > "$OUT/dn_$v.json" 2> "$OUT/dn_$v.err" || { tail -20 "$OUT/dn_$v.err"; exit 1; }
done
echo "[$(date +%T)] 4K bench line"
timeout -k 10 300 python bench.py --width 3840 --height 2160 --no-cpu-baseline > "$OUT/bench4k.json" 2> "$OUT/bench4k.err" || { tail -20 "$OUT/bench4k.err"; exit 1; }
echo "[$(date +%T)] done"
