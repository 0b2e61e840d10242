set -o pipefail
bash tools/gpu_check.sh gpurun_out/fin4 tests && bash tools/prof_r04_c2c4.sh gpurun_out/c2c4 > gpurun_out/c2c4.log 2>&1 && bash tools/rank_probe_1080.sh > gpurun_out/rank1080.log 2>&1
rc=$?; tail -3 gpurun_out/c2c4.log; tail -12 gpurun_out/rank1080.log; exit $rc
