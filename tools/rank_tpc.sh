set -u
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "pipeline or bench_path or multirank" > gpurun_out/fin_pytest.log 2>&1 || { tail -20 gpurun_out/fin_pytest.log; exit 1; }
tail -1 gpurun_out/fin_pytest.log
for n in 2 4 8; do for pc in 3 2; do
  echo "N=$n perCu=$pc $(STRIP_DN=1 RTX_TRACE_PER_CU=$pc timeout -k 10 120 python tools/rank_probe.py $n 2>&1 | grep N=)"
done; done
