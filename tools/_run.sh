set -u
export TMPDIR=/tmp
O=gpurun_out/r05_t2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_denoise.py tests/test_gpu_bench_path.py tests/test_gpu_multirank.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
grep -E "FAILED|PASSED" $O/pytest.log | head -60
exit $rc
