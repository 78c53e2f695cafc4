set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_ipe_fused_gpu.py > gpurun_out/ipe_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -25 gpurun_out/ipe_tests.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python -u benchmarks/ipe_bench.py --steps 3 > gpurun_out/ipe_bench.log 2>&1
  echo "bench rc=$?"
  cat gpurun_out/ipe_bench.log | tail -12
fi
