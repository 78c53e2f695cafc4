set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
T="python -u -m pytest -v --timeout 240 --timeout-method thread"
timeout -k 10 300 $T tests/test_ipe_fused_gpu.py tests/test_kmpp_gpu.py > gpurun_out/r4_t1.log 2>&1
rc=$?; echo "t1 rc=$rc"; grep -E "FAIL|ERROR|passed|failed" gpurun_out/r4_t1.log | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u benchmarks/ipe_bench.py --steps 3 > gpurun_out/ipe_bench.log 2>&1
rc=$?; echo "ipe bench rc=$rc"; tail -3 gpurun_out/ipe_bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/kmpp_bench.py --k 1024 --center > gpurun_out/kmpp_bench.log 2>&1
rc=$?; echo "kmpp bench rc=$rc"; tail -4 gpurun_out/kmpp_bench.log
exit $rc
