set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_kmpp_gpu.py tests/test_ipe_fused_gpu.py tests/test_mstep_incremental_gpu.py tests/test_pipeline_gpu.py tests/test_dmeans_pinned_gpu.py tests/test_failure_pruning_gpu.py tests/test_distributed_gpu.py > gpurun_out/r4_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r4_tests.log | tail -40
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python -u benchmarks/ipe_bench.py --steps 3 > gpurun_out/ipe_bench.log 2>&1
  echo "ipe bench rc=$?"
  tail -6 gpurun_out/ipe_bench.log
  timeout -k 10 300 python -u benchmarks/kmpp_bench.py --k 1024 --center > gpurun_out/kmpp_bench.log 2>&1
  echo "kmpp bench rc=$?"
  tail -4 gpurun_out/kmpp_bench.log
fi
